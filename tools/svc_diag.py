#!/usr/bin/env python
"""Diagnostic for the small host-allreduce service: N ranks on the local GPU,
fp32 SUM of rank-dependent small integers (exact in any order), a few sizes
and repeats; prints per call the number of wrong elements and the first few
values (got / want).  python tools/svc_diag.py [--world 2]"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, world, port):
    import numpy as np
    import torch
    import rdc_amd
    from rdc_amd._lib import _LIB, check_call
    rdc_amd.init(["RDC_RANK=%d" % rank, "RDC_WORLD_SIZE=%d" % world, "RDC_TRACKER_PORT=%d" % port,
                  "RDC_TRACKER_URI=127.0.0.1"])
    torch.cuda.set_device(0)
    rows = []
    for it, count in enumerate([1, 4, 64, 1024, 1024, 1024, 4099, 16384, 16384]):
        i = np.arange(count, dtype=np.float64)
        x = (rank + 1 + (i + it) % 7).astype(np.float32)
        inp = x.copy()
        check_call(_LIB.RdcAllreduce(ctypes.c_void_p(x.ctypes.data), count, 6, 2, None, None))
        want = (world * (world + 1) / 2 + world * ((i + it) % 7)).astype(np.float32)
        bad = np.nonzero(x != want)[0]
        rows.append({"count": count, "bad": int(bad.size), "first_bad": int(bad[0]) if bad.size else -1,
                     "got": x[:4].tolist(), "want": want[:4].tolist(), "input": inp[:4].tolist(),
                     "got_eq_input": bool(bad.size and np.array_equal(x[bad], inp[bad]))})
    print(json.dumps({"rank": rank, "env_strict": os.environ.get("RDC_STRICT_FENCES", ""), "rows": rows}), flush=True)
    rdc_amd.finalize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--rank", type=int, default=-1)
    ap.add_argument("--port", type=int, default=0)
    a = ap.parse_args()
    if a.rank >= 0:
        worker(a.rank, a.world, a.port)
        return
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--world", str(a.world), "--rank", str(r),
                               "--port", str(port)]) for r in range(a.world)]
    rc = 0
    for p in procs:
        rc |= p.wait()
    sys.exit(rc)


if __name__ == "__main__":
    main()
