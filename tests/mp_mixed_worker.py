"""One rank of a randomized mixed-collective chain (spawned by
tests/test_gpu_mixed.py): a seeded sequence of allreduce (every schedule),
broadcast (rotating roots, direct and forwarded), variable-size allgather and
coalesced allreduce launches on ONE communicator and ONE stream with no host
synchronisation in between, so consecutive launches of different kinds
overlap across ranks the way a training step issues them; synchronous
host-buffer allreduces (the small-allreduce service, or the launch path above
64 KiB) run in between while earlier launches may still be in flight.  Every op has its
own output buffers; all are saved at the end for the parent to check against
the CPU oracle.

argv: rank world port outdir seed nops
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests.mixed_plan import ESZ, make_plan  # noqa: E402


def main():
    rank, world, port, outdir = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    seed, nops = int(sys.argv[5]), int(sys.argv[6])
    import torch
    import rdc_amd
    from rdc_amd._lib import _LIB, check_call
    rdc_amd.init(["RDC_RANK=%d" % rank, "RDC_WORLD_SIZE=%d" % world, "RDC_TRACKER_PORT=%d" % port,
                  "RDC_TRACKER_URI=127.0.0.1", "RDC_DEVICE=0"])
    torch.cuda.set_device(0)
    comm = rdc_amd.get_comm("main")
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    keep = []

    def dev(nbytes):
        t = torch.zeros(max(nbytes, 1) + 64, dtype=torch.uint8, device="cuda")
        keep.append(t)
        return t

    outs = []
    for op in make_plan(seed, nops, world):
        kind = op["kind"]
        if kind == "allreduce":
            n, dt = op["count"], op["dtype"]
            t = dev(n * ESZ[dt])
            check_call(_LIB.RdcFill(ctypes.c_void_p(t.data_ptr()), n, dt, op["seed"], rank, sp))
            check_call(_LIB.RdcCommAllreduceEx(comm.handle, ctypes.c_void_p(t.data_ptr()), n, dt, op["op"],
                                               op["algo"], sp))
            outs.append((t, n * ESZ[dt]))
        elif kind == "host":
            from oracle import oracle as O  # the checker's generator (same bits as RdcFill)
            h = O.fill(op["count"], op["dtype"], op["seed"], rank).copy()
            check_call(_LIB.RdcAllreduce(ctypes.c_void_p(h.ctypes.data), op["count"], op["dtype"], op["op"], None, None))
            outs.append((h, h.nbytes))
        elif kind == "bcast":
            nb = op["bytes"]
            t = dev(nb)
            check_call(_LIB.RdcFill(ctypes.c_void_p(t.data_ptr()), nb, 1, op["seed"], rank, sp))
            check_call(_LIB.RdcCommBroadcast(comm.handle, ctypes.c_void_p(t.data_ptr()), nb, op["root"], sp))
            outs.append((t, nb))
        elif kind == "allgather":
            sizes = op["sizes"]
            ts = [dev(s) for s in sizes]
            check_call(_LIB.RdcFill(ctypes.c_void_p(ts[rank].data_ptr()), sizes[rank], 1, op["seed"], rank, sp))
            ptrs = (ctypes.c_void_p * world)(*[x.data_ptr() for x in ts])
            szs = (ctypes.c_size_t * world)(*sizes)
            check_call(_LIB.RdcCommAllgather(comm.handle, ptrs, szs, sp))
            outs.extend(zip(ts, sizes))
        else:
            counts, dt = op["counts"], op["dtype"]
            ts = [dev(c * ESZ[dt]) for c in counts]
            for b, (x, c) in enumerate(zip(ts, counts)):
                check_call(_LIB.RdcFill(ctypes.c_void_p(x.data_ptr()), c, dt, op["seed"] + b, rank, sp))
            ptrs = (ctypes.c_void_p * len(counts))(*[x.data_ptr() for x in ts])
            cnt = (ctypes.c_size_t * len(counts))(*counts)
            check_call(_LIB.RdcCommAllreduceCoalesced(comm.handle, ptrs, cnt, len(counts), dt, op["op"], op["algo"],
                                                      sp))
            outs.extend((x, c * ESZ[dt]) for x, c in zip(ts, counts))
    comm.check(sp)
    blob = np.concatenate([np.frombuffer(t.tobytes(), np.uint8) if isinstance(t, np.ndarray) else t[:nb].cpu().numpy()
                           for t, nb in outs]) if outs else np.zeros(0, np.uint8)
    np.save(os.path.join(outdir, "mixed_rank%d.npy" % rank), blob)
    print("rank %d: mixed OK" % rank, flush=True)
    rdc_amd.finalize()


if __name__ == "__main__":
    main()
