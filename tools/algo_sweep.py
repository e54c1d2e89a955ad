#!/usr/bin/env python
"""Per-launch time of each allreduce schedule over a range of sizes, on the
communicator's own stream, max over ranks (the schedule-choice data for
RDC_ONESHOT_BYTES / RDC_DIRECT_BYTES).  fp32 sum; algo 0 = the automatic
choice (its schedule in auto_schedule), algo 1 = ring (reference
schedule), 2 = mesh, 3 = one-shot (skipped where it does not fit the slot
half), 5 = pull-mode mesh, 6 = direct (registered buffers).  SWEEP_ALGOS
(e.g. "0/1/6") picks the schedules.  Direct-schedule calls also report the
host side of their rendezvous per call (<name>_rendezvous_us: publish, map,
confirm; <name>_export_us: the export step alone; max over ranks).

    python -m torch.distributed.run --nproc-per-node N tools/algo_sweep.py [sizes_MiB] [steps]
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    sizes = [float(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,4,16,64,256").replace("/", ",").split(",")]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    import torch
    import torch.distributed as dist
    import rdc_amd
    from rdc_amd._lib import _LIB, check_call
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    dist.init_process_group("gloo")
    rdc_amd.init([])
    comm = rdc_amd.get_comm("main")
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    half = ctypes.c_uint64()
    check_call(_LIB.RdcCommGetParam(comm.handle, b"slot_bytes", ctypes.byref(half)))
    big = int(max(sizes) * (1 << 20))
    buf = torch.empty(big // 4, dtype=torch.float32, device="cuda")
    rdc_amd.fill_(buf, 0x5EED0000, rank)
    out = {}
    for mib in sizes:
        nb = int(mib * (1 << 20))
        row = {}
        for algo, name in ((0, "auto"), (1, "ring"), (2, "mesh"), (3, "oneshot"), (5, "mesh_pull"), (6, "direct")):
            if str(algo) not in os.environ.get("SWEEP_ALGOS", "0/1/2/3").replace(",", "/").split("/"):
                continue
            if algo == 3 and nb > half.value // 2:
                continue

            def one():
                check_call(_LIB.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(buf.data_ptr()), nb // 4, 6, 2, algo,
                                                   sp))

            def stats():
                r = {}
                for k in ("direct_calls", "direct_rendezvous_ns", "direct_export_ns"):
                    v = ctypes.c_uint64()
                    check_call(_LIB.RdcCommGetParam(comm.handle, k.encode(), ctypes.byref(v)))
                    r[k] = int(v.value)
                return r
            for _ in range(3):
                one()
            torch.cuda.synchronize()
            comm.check(sp)
            dist.barrier()
            n_steps = max(steps, int(2e8 // max(nb, 1)) if nb < (16 << 20) else steps)
            d0 = stats()
            t0 = time.perf_counter()
            for _ in range(n_steps):
                one()
            torch.cuda.synchronize()
            t = torch.tensor([(time.perf_counter() - t0) / n_steps], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            comm.check(sp)
            row[name] = round(float(t[0]) * 1e3, 4)
            ll = (ctypes.c_uint64 * 6)()
            check_call(_LIB.RdcCommLastLaunch(comm.handle, ll))
            if algo == 0:  # the schedule the automatic choice launched
                row["auto_schedule"] = {1: "ring", 2: "mesh", 3: "oneshot", 4: "tree", 5: "mesh_pull",
                                        6: "direct"}.get(int(ll[5]), int(ll[5]))
            d1 = stats()
            if d1["direct_calls"] > d0["direct_calls"]:  # host side of the direct rendezvous, per call (max over ranks)
                nc = d1["direct_calls"] - d0["direct_calls"]
                v = torch.tensor([(d1["direct_rendezvous_ns"] - d0["direct_rendezvous_ns"]) / nc / 1e3,
                                  (d1["direct_export_ns"] - d0["direct_export_ns"]) / nc / 1e3], dtype=torch.float64)
                dist.all_reduce(v, op=dist.ReduceOp.MAX)
                row[name + "_rendezvous_us"] = round(float(v[0]), 2)
                row[name + "_export_us"] = round(float(v[1]), 2)
        out["%g MiB" % mib] = row
    if rank == 0:
        print(json.dumps({"algo_sweep_ms_per_launch": out, "world": world, "ranks_share_gpu": True,
                          "RDC_DIRECT_BYTES": os.environ.get("RDC_DIRECT_BYTES", "auto (default)")}), flush=True)
    dist.barrier()
    rdc_amd.finalize()


if __name__ == "__main__":
    main()
