"""Comparison point ("RCCL is a comparison point only"): the same
in-place fp32 sum allreduce through torch.distributed's nccl backend (= RCCL
on ROCm), one process per GPU.  bench.py starts one of these per rank as a
child process after its own measurements, with a time limit, and reports the
result beside its own line; a failure or hang here never costs the main line.

    python tools/rccl_allreduce.py RANK WORLD LOCAL_RANK MASTER_ADDR PORT BYTES STEPS

Rank 0 prints one JSON line: {"rccl": true, "ms_per_step": ..., "busbw_GBps": ...}.
"""
import json
import os
import sys
import time


def main():
    rank, world, local = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    addr, port, S, steps = sys.argv[4], int(sys.argv[5]), int(sys.argv[6]), int(sys.argv[7])
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local % torch.cuda.device_count())
    dist.init_process_group("nccl", init_method="tcp://%s:%d" % (addr, port), rank=rank, world_size=world)
    x = torch.ones(S // 4, dtype=torch.float32, device="cuda")
    for _ in range(3):
        dist.all_reduce(x)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        dist.all_reduce(x)
    torch.cuda.synchronize()
    t = torch.tensor([(time.perf_counter() - t0) / steps], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms = float(t.item()) * 1e3
    if rank == 0:
        bus = S / (ms * 1e-3) / 1e9 * 2 * (world - 1) / max(world, 1)
        print(json.dumps({"rccl": True, "ms_per_step": round(ms, 4), "busbw_GBps": round(bus, 2), "steps": steps,
                          "bytes_per_gpu": S, "torch": torch.__version__,
                          "note": "torch.distributed all_reduce (nccl backend = RCCL), fp32 sum, in place"}),
              flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
