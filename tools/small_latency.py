#!/usr/bin/env python
"""Small-message latency of the allreduce paths, as N processes on the local
GPU(s) (spawns its own ranks; RdcInit rendezvous, no torch.distributed).

    python tools/small_latency.py [--world 2] [--iters 2000] [--bytes 4096,65536]

Per size, per rank 0 (median of per-call times, microseconds):
  dev_async : RdcCommAllreduceEx on a device buffer, back-to-back, one sync at the end
  dev_sync  : RdcAllreduce on a device buffer (synchronous: launch + completion token)
  host_sync : RdcAllreduce on a pageable numpy array (cfg1's path)
Every rank checks one host result against a closed-form sum per size.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, world, port, iters, sizes):
    import numpy as np
    import torch
    import rdc_amd
    from rdc_amd._lib import _LIB, check_call
    rdc_amd.init(["RDC_RANK=%d" % rank, "RDC_WORLD_SIZE=%d" % world, "RDC_TRACKER_PORT=%d" % port,
                  "RDC_TRACKER_URI=127.0.0.1"])
    dev = int(os.environ.get("RDC_DEVICE", rank % max(1, torch.cuda.device_count())))
    torch.cuda.set_device(dev)
    comm = rdc_amd.get_comm("main")
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = {}
    for nb in sizes:
        count = nb // 4
        d = torch.ones(count, dtype=torch.float32, device="cuda")
        res = {}

        def timed(fn, n):
            ts = []
            for _ in range(n):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            ts.sort()
            return ts[len(ts) // 2] * 1e6

        # device, asynchronous chain
        for _ in range(20):
            check_call(_LIB.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(d.data_ptr()), count, 6, 2, 0, sp))
        torch.cuda.synchronize()
        rdc_amd.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            check_call(_LIB.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(d.data_ptr()), count, 6, 2, 0, sp))
        torch.cuda.synchronize()
        res["dev_async"] = (time.perf_counter() - t0) / iters * 1e6
        comm.check(sp)
        rdc_amd.barrier()
        # device, synchronous per call
        res["dev_sync"] = timed(lambda: check_call(_LIB.RdcAllreduce(ctypes.c_void_p(d.data_ptr()), count, 6, 2,
                                                                     None, None)), iters)
        rdc_amd.barrier()
        # host (pageable), synchronous per call
        a = np.ones(count, dtype=np.float32)
        res["host_sync"] = timed(lambda: check_call(_LIB.RdcAllreduce(ctypes.c_void_p(a.ctypes.data), count, 6, 2,
                                                                      None, None)), iters)
        rdc_amd.barrier()
        # correctness of the host path: rank r holds r + 1 + i % 7 (small
        # integers, exact in fp32 in any order), the sum has a closed form
        i = np.arange(count, dtype=np.float64)
        x = (rank + 1 + i % 7).astype(np.float32)
        check_call(_LIB.RdcAllreduce(ctypes.c_void_p(x.ctypes.data), count, 6, 2, None, None))
        want = (world * (world + 1) / 2 + world * (i % 7)).astype(np.float32)
        res["host_ok"] = x.tobytes() == want.tobytes()
        out[str(nb)] = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}
        del d
    if rank == 0:
        print(json.dumps({"world": world, "iters": iters, "us_per_call_median": out}), flush=True)
    rdc_amd.finalize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--bytes", nargs="+", default=["4096,65536"])
    ap.add_argument("--rank", type=int, default=-1)
    ap.add_argument("--port", type=int, default=0)
    a = ap.parse_args()
    sizes = [int(x) for b in a.bytes for x in b.split(",")]
    if a.rank >= 0:
        worker(a.rank, a.world, a.port, a.iters, sizes)
        return
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--world", str(a.world), "--iters",
                               str(a.iters), "--bytes", ",".join(map(str, sizes)), "--rank", str(r), "--port", str(port)])
             for r in range(a.world)]
    rc = 0
    for p in procs:
        rc |= p.wait()
    sys.exit(rc)


if __name__ == "__main__":
    main()
