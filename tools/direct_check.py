#!/usr/bin/env python
"""The direct schedule (algo 6) against the ring (algo 1) on the same inputs,
bit for bit, over sizes and dtypes; prints the mismatching elements' first
index per rank.  A debugging aid for k_direct at sizes the oracle tests do
not reach (the ring's own parity with the oracle is tested).

    python -m torch.distributed.run --nproc-per-node N tools/direct_check.py [MiB,...] [dtypes] [realloc]
With "realloc", each size first goes through the direct schedule on a
buffer that is then freed (torch.cuda.empty_cache) before the checked one
is allocated: the case of a peer mapping that outlives its allocation.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    sizes = [float(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "64,256,1024").replace("/", ",").split(",")]
    dts = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "6,10").replace("/", ",").split(",")]
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
    tdt = {6: torch.float32, 10: torch.float16, 11: torch.bfloat16, 2: torch.int32}
    esz = {6: 4, 10: 2, 11: 2, 2: 4}
    realloc = len(sys.argv) > 3 and sys.argv[3] == "realloc"
    hip = ctypes.CDLL("libamdhip64.so")

    def buffer_id(t):
        v = ctypes.c_uint64(0)
        hip.hipPointerGetAttribute(ctypes.byref(v), 7, ctypes.c_void_p(t.data_ptr()))  # HIP_POINTER_ATTRIBUTE_BUFFER_ID
        return int(v.value)

    rows = []
    for mib in sizes:
        for dt in dts:
            count = int(mib * (1 << 20)) // esz[dt]
            prev = None
            if realloc:
                z = torch.empty(count, dtype=tdt[dt], device="cuda")
                check_call(_LIB.RdcFill(ctypes.c_void_p(z.data_ptr()), count, dt, 0x5EEDD000 + dt, rank, sp))
                check_call(_LIB.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(z.data_ptr()), count, dt, 2, 6, sp))
                torch.cuda.synchronize()
                prev = (hex(z.data_ptr()), buffer_id(z))
                del z
                torch.cuda.empty_cache()
            a = torch.empty(count, dtype=tdt[dt], device="cuda")
            now = (hex(a.data_ptr()), buffer_id(a))
            check_call(_LIB.RdcFill(ctypes.c_void_p(a.data_ptr()), count, dt, 0x5EEDC000 + dt, rank, sp))
            b = a.clone()
            check_call(_LIB.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(a.data_ptr()), count, dt, 2, 6, sp))
            check_call(_LIB.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(b.data_ptr()), count, dt, 2, 1, sp))
            torch.cuda.synchronize()
            comm.check(sp)
            ai, bi = a.view(torch.int16 if esz[dt] == 2 else torch.int32), b.view(torch.int16 if esz[dt] == 2 else torch.int32)
            bad = (ai != bi).nonzero().flatten()
            nb = int(bad.numel())
            first = int(bad[0]) if nb else -1
            last = int(bad[-1]) if nb else -1
            rows.append({"rank": rank, "MiB": mib, "dtype": dt, "bad": nb, "first": first, "last": last,
                         "chunk_of_first": (first * world // count) if nb else None,
                         "a_first": float(a[first]) if nb else None, "b_first": float(b[first]) if nb else None,
                         "freed": prev, "checked": now})
            del a, b, ai, bi, bad
    allrows = [None] * world
    dist.all_gather_object(allrows, rows)
    if rank == 0:
        for rr in allrows:
            for r in rr:
                print(json.dumps(r), flush=True)
    dist.barrier()
    rdc_amd.finalize()


if __name__ == "__main__":
    main()
