"""Timing sweep of the device allreduce in a single-process group on one GPU
(all ranks share GPU 0, so this measures the protocol + HBM side, not xGMI).

    RDC_ALLOC=uncached|fine|coarse python tools/group_perf.py n size [size...]
    GP_BUCKETS=K: each size split into K buckets, one coalesced call (plus the
    same K buckets as separate calls, for comparison)
"""
import ctypes
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import rdc_amd  # noqa: E402
from rdc_amd._lib import _LIB, check_call  # noqa: E402


def main():
    n = int(sys.argv[1])
    # ranks sharing one GPU from one process each need their own hardware
    # queue; beyond 3 ranks + the null stream two ranks can share one and
    # deadlock (measured: n=4 times out).  Use processes for more ranks.
    assert n <= 3, "single-process groups on one GPU: at most 3 ranks"
    sizes = [int(float(x)) for x in sys.argv[2:]] or [1 << 20]
    scratch = int(os.environ.get("RDC_SCRATCH_BYTES_PY", str(1 << 30)))
    comms = rdc_amd.init_group([0] * n, scratch_bytes=scratch)
    streams = [torch.cuda.Stream() for _ in range(n)]
    print("alloc kind", comms[0].alloc_kind, "n", n, flush=True)
    for S in sizes:
        count = S // 4
        bufs = [torch.empty(count, dtype=torch.float32, device="cuda") for _ in range(n)]
        for r in range(n):
            rdc_amd.fill_(bufs[r], 1, r)
        torch.cuda.synchronize()
        K = int(os.environ.get("GP_BUCKETS", "1"))
        modes = (2, 1) if K == 1 else ("coalesced", "separate")
        per = count // K
        views = [[bufs[r][b * per:(b + 1) * per] for b in range(K)] for r in range(n)]
        for algo in modes:
            def once():
                for r in range(n):
                    sp = ctypes.c_void_p(streams[r].cuda_stream)
                    if algo == "coalesced":
                        comms[r].allreduce_coalesced(views[r], 2, stream=sp)
                    elif algo == "separate":
                        for v in views[r]:
                            comms[r].allreduce(v, 2, stream=sp)
                    else:
                        check_call(_LIB.RdcCommAllreduceEx(comms[r].handle, ctypes.c_void_p(bufs[r].data_ptr()),
                                                           count, 6, 2, algo, sp))
            once()
            for r in range(n):
                comms[r].check(ctypes.c_void_p(streams[r].cuda_stream))
            it = 5 if S >= (64 << 20) else 20
            t0 = time.perf_counter()
            for _ in range(it):
                once()
            for r in range(n):
                comms[r].check(ctypes.c_void_p(streams[r].cuda_stream))
            dt = (time.perf_counter() - t0) / it
            name = {2: "mesh", 1: "ring"}.get(algo, "%s x%d" % (algo, K))
            print("n=%d S=%9d algo=%s  %.3f ms  algbw %.1f GB/s" % (n, S, name, dt * 1e3, S / dt / 1e9), flush=True)
    for c in comms:
        c.destroy()


if __name__ == "__main__":
    main()
