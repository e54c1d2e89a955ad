"""PCIe-inclusive rate of the host-resident allreduce (rdc's native setting:
buffers begin and end in host memory).  Each call: H2D copy, device
allreduce, D2H copy, synchronise (RdcAllreduce on a numpy buffer).

    python -m torch.distributed.run --nproc-per-node N tools/host_path.py [bytes] [iters]
    python tools/host_path.py [bytes] [iters]          # N = 1: H2D + reduce + D2H
    RDC_BENCH_PINNED=1 ...: the buffer is a registered RdcNewBuffer(pinned=1)
    range (page-aligned mmap), so the library DMAs it in place
    (RDC_BENCH_THP=1: madvise(MADV_HUGEPAGE) on that mmap first)
    RDC_BENCH_GAP_MS=G: the host idles G ms before every call (untimed), as a
    training step's compute would between allreduces

Prints one JSON line (rank 0) with GB/s = S / t per call (max over ranks).
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    S = int(float(sys.argv[1])) if len(sys.argv) > 1 else (256 << 20)
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    import numpy as np
    import torch
    import rdc_amd
    from rdc_amd._lib import _LIB, check_call
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    count = S // 4
    pinned = os.environ.get("RDC_BENCH_PINNED", "0") == "1" and world > 1
    host = np.random.default_rng(rank).standard_normal(count).astype(np.float32)
    reg = None
    if pinned:
        import mmap
        span = (S + mmap.PAGESIZE - 1) // mmap.PAGESIZE * mmap.PAGESIZE
        mm = mmap.mmap(-1, span)
        if os.environ.get("RDC_BENCH_THP") == "1":  # transparent huge pages behind the registered range
            mm.madvise(mmap.MADV_HUGEPAGE)
        backing = np.frombuffer(mm, dtype=np.uint8)
        backing[:S].view(np.float32)[:] = host
        host = backing[:S].view(np.float32)
    p = host.ctypes.data_as(ctypes.c_void_p)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        rdc_amd.init([])
        if pinned:
            reg = ctypes.c_void_p()
            check_call(_LIB.RdcNewBuffer(ctypes.byref(reg), ctypes.c_void_p(backing.ctypes.data), span, 1))

        def call():
            check_call(_LIB.RdcAllreduce(p, count, 6, 2, None, None))
    else:
        d = torch.empty(count, dtype=torch.float32, device="cuda")
        s = torch.empty(count, dtype=torch.float32, device="cuda")
        src = np.ones(count, dtype=np.float32)

        def call():  # the 1-GPU data point with host buffers: H2D x2, reduce, D2H
            d.copy_(torch.from_numpy(host))
            s.copy_(torch.from_numpy(src))
            rdc_amd.reduce_(d, s, rdc_amd.Op.SUM)
            host[:] = d.cpu().numpy()
    call()
    if world > 1:
        dist.barrier()
    per = []
    gap = float(os.environ.get("RDC_BENCH_GAP_MS", "0")) / 1e3  # idle host time before every call (not timed)
    idle = 0.0
    t0 = time.perf_counter()
    for _ in range(iters):
        if gap > 0:
            time.sleep(gap)
            idle += gap
        t1 = time.perf_counter()
        call()
        per.append(time.perf_counter() - t1)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0 - idle) / iters
    per_call_ms = [round(x * 1e3, 3) for x in per]
    per.sort()
    med_us, max_us = per[len(per) // 2] * 1e6, per[-1] * 1e6
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t[0])
    if rank == 0:
        print(json.dumps({"host_path": True, "n": world, "bytes": S, "ms_per_call": round(dt * 1e3, 4),
                          "us_per_call_mean": round(dt * 1e6, 2), "us_per_call_median_rank0": round(med_us, 2),
                          "us_per_call_max_rank0": round(max_us, 1),
                          "per_call_ms_rank0": per_call_ms if os.environ.get("RDC_BENCH_PER_CALL") else None,
                          "GBps": round(S / dt / 1e9, 3),
                          "memory": "registered (RdcNewBuffer pinned)" if pinned else "pageable numpy"}), flush=True)
    if world > 1:
        dist.barrier()
        if reg is not None:
            check_call(_LIB.RdcDelBuffer(reg))
        rdc_amd.finalize()


if __name__ == "__main__":
    main()
