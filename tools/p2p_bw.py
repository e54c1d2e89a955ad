"""Point-to-point throughput and latency (ICommunicator::ISend/IRecv on the
device path): rank 0 sends a device buffer to rank 1, which sends it back
(ping-pong), for a range of sizes.  Ranks are processes; on the 1-GPU box they
share GPU 0, so the bytes move through one HBM instead of xGMI.

    python -m torch.distributed.run --nproc-per-node 2 tools/p2p_bw.py [sizes...]

Prints one JSON line per size (rank 0): one-way time = round trip / 2.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    sizes = [int(float(x)) for x in sys.argv[1:]] or [4096, 1 << 20, 16 << 20, 256 << 20]
    import torch
    import torch.distributed as dist
    import rdc_amd
    rank = int(os.environ["RANK"])
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    dist.init_process_group("gloo")
    rdc_amd.init([])
    comm = rdc_amd.get_comm("main")
    peer = 1 - rank
    for S in sizes:
        x = torch.full((S,), rank + 1, dtype=torch.uint8, device="cuda")
        y = torch.zeros(S, dtype=torch.uint8, device="cuda")
        iters = max(3, min(200, (2 << 30) // max(S, 1)))

        def ping():
            if rank == 0:
                comm.send(x, peer)
                comm.recv(y, peer)
            else:
                comm.recv(y, peer)
                comm.send(y, peer)

        ping()
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            ping()
        dt = (time.perf_counter() - t0) / iters / 2
        ok = bool((y == 1).all()) if rank == 0 else True
        if rank == 0:
            print(json.dumps({"p2p": True, "bytes": S, "one_way_us": round(dt * 1e6, 2),
                              "GBps": round(S / dt / 1e9, 3), "check": ok}), flush=True)
        dist.barrier()
    rdc_amd.finalize()


if __name__ == "__main__":
    main()
