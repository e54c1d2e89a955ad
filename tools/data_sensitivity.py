"""Does the allreduce's speed depend on the data?  (autotune timed zeros and
picked a shape at 1.09 ms; the timed region, on random data, ran 1.36 ms.)

    python -m torch.distributed.run --nproc-per-node N tools/data_sensitivity.py [MiB]

Same communicator, same schedule and shape, 1 GiB fp32 by default: zeros
(Sum stays zero), random synthetic data under Max (stays random), random data
under Sum (grows, stays random-looking for the few calls timed), alternating,
HIP events on the stream over 10 calls each, max over ranks.  Prints JSON.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    import rdc_amd
    from rdc_amd._lib import _LIB, check_call
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    dist.init_process_group("gloo")
    rdc_amd.init([])
    comm = rdc_amd.get_comm("main")
    s = torch.cuda.current_stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    count = (mib << 20) // 4
    zeros = torch.zeros(count, dtype=torch.float32, device="cuda")
    rnd = torch.empty(count, dtype=torch.float32, device="cuda")
    rdc_amd.fill_(rnd, 0x5EED0000, rank)
    algo = int(os.environ.get("ALGO", "0"))

    def timed(t, op, calls=10):
        check_call(_LIB.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(t.data_ptr()), count, 6, op, algo, sp))
        comm.check(sp)
        dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(calls):
            check_call(_LIB.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(t.data_ptr()), count, 6, op, algo, sp))
        e1.record(s)
        comm.check(sp)
        v = torch.tensor([e0.elapsed_time(e1) / calls], dtype=torch.float64)
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        return round(float(v[0]), 4)

    res = {"zeros_sum": [], "random_max": [], "random_sum": []}
    for _ in range(3):
        res["zeros_sum"].append(timed(zeros, 2))
        res["random_max"].append(timed(rnd, 0))
        rdc_amd.fill_(rnd, 0x5EED0000, rank)
        res["random_sum"].append(timed(rnd, 2, calls=5))
        rdc_amd.fill_(rnd, 0x5EED0000, rank)
    if rank == 0:
        print(json.dumps({"world": world, "MiB": mib, "algo": algo, "ms_per_call": res}), flush=True)
    dist.barrier()
    rdc_amd.finalize()


if __name__ == "__main__":
    main()
