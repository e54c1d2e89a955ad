#!/usr/bin/env python
"""How much a buffer's placement moves the direct schedule on the shared
HBM: K buffers of S bytes allocated one after another on every rank, each
timed with R direct allreduces (algo 6, fp32 sum; max over ranks of the mean),
twice in turn (so a slow buffer shows up as slow both times), next to a plain
device copy of the same buffer on one rank (the single-process streaming rate
of that buffer).

    python -m torch.distributed.run --nproc-per-node N tools/placement_probe.py [K] [MiB] [R]
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    mib = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    R = int(sys.argv[3]) if len(sys.argv) > 3 else 10
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
    count = (mib << 20) // 4
    bufs = [torch.empty(count, dtype=torch.float32, device="cuda") for _ in range(K)]
    for k, b in enumerate(bufs):
        rdc_amd.fill_(b, 0x5EED0000 + k, rank)
    scratch = torch.empty(count, dtype=torch.float32, device="cuda")

    def direct_ms(b):
        def one():
            check_call(_LIB.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(b.data_ptr()), count, 6, 0, 6, sp))
        one()  # maps the buffer (first use)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(R):
            one()
        torch.cuda.synchronize()
        t = torch.tensor([(time.perf_counter() - t0) / R * 1e3], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        comm.check(sp)
        return round(float(t[0]), 4)

    def copy_ms(b):
        dist.barrier()
        if rank != 0:
            dist.barrier()
            return None
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        scratch.copy_(b)
        e0.record()
        for _ in range(R):
            scratch.copy_(b)
        e1.record()
        e1.synchronize()
        dist.barrier()
        return round(e0.elapsed_time(e1) / R, 4)

    rows = []
    for rnd in range(2):
        for k, b in enumerate(bufs):
            rows.append({"round": rnd, "buffer": k, "direct_ms": direct_ms(b), "copy_ms_rank0": copy_ms(b)})
    if rank == 0:
        print(json.dumps({"world": world, "MiB": mib, "reps": R, "rows": rows}), flush=True)
    dist.barrier()
    rdc_amd.finalize()


if __name__ == "__main__":
    main()
