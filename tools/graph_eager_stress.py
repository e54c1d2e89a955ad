"""Stress of the sequence behind GPUTEST_r04's red test: hipGraph replays of an
allreduce, then an eager allreduce on the same communicators (n = 2 ranks in
one process on one GPU, tests/test_gpu_allreduce.py:233-267), repeated.

For every round: capture one allreduce of `count` fp32 per rank (schedule
--graph-algo), replay it --replays times with fresh inputs, then run one eager
allreduce of --eager-count elements with --eager-algo; every result is
compared with the oracle and every mismatch is reported with its rank, the
element ranges that differ and which Split chunk they lie in, together with
both ranks' device launch counters.  --no-graph replaces the replays with
eager launches of the same size (the control).

    python tools/graph_eager_stress.py --rounds 50
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

ALGOS = {"mesh": 2, "ring": 1, "oneshot": 3, "mesh_pull": 5}


def split_chunks(count, n):
    k, m = divmod(count, n)
    bounds, b = [], 0
    for c in range(n):
        e = b + k + (1 if c < m else 0)
        bounds.append((b, e))
        b = e
    return bounds


def diff_ranges(got, want, n):
    bad = np.flatnonzero(got.view(np.uint32) != want.view(np.uint32))
    if bad.size == 0:
        return []
    chunks = split_chunks(want.size, n)
    runs, start, prev = [], bad[0], bad[0]
    for i in bad[1:]:
        if i != prev + 1:
            runs.append((int(start), int(prev) + 1))
            start = i
        prev = i
    runs.append((int(start), int(prev) + 1))
    out = []
    for a, b in runs[:8]:
        c = next(ci for ci, (lo, hi) in enumerate(chunks) if lo <= a < hi)
        out.append({"range": [a, b], "chunk": c})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=50)
    ap.add_argument("--count", type=int, default=300007)
    ap.add_argument("--replays", type=int, default=4)
    ap.add_argument("--graph-algo", default="mesh")
    ap.add_argument("--eager-count", type=int, default=1001)
    ap.add_argument("--eager-algo", type=int, default=2)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--scratch", type=int, default=16 << 20)
    args = ap.parse_args()

    import torch
    import rdc_amd
    from rdc_amd._lib import _LIB
    from oracle import oracle as O

    comms = rdc_amd.init_group([0, 0], scratch_bytes=args.scratch)
    streams = [torch.cuda.Stream() for _ in range(2)]
    rng = np.random.default_rng(21)
    fails = []

    def counters():
        out = []
        for c in comms:
            v = ctypes.c_uint64()
            assert _LIB.RdcCommLaunchCounter(c.handle, ctypes.byref(v)) == 0
            out.append(v.value)
        return out

    for rnd in range(args.rounds):
        ts = [torch.zeros(args.count, dtype=torch.float32, device="cuda") for _ in range(2)]
        graphs = []
        torch.cuda.synchronize()
        if not args.no_graph:
            for r in range(2):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=streams[r], capture_error_mode="thread_local"):
                    comms[r].allreduce(ts[r], rdc_amd.Op.SUM, algo=args.graph_algo,
                                       stream=ctypes.c_void_p(streams[r].cuda_stream))
                graphs.append(g)
            torch.cuda.synchronize()
        for it in range(args.replays):
            xs = [rng.standard_normal(args.count).astype(np.float32) for _ in range(2)]
            for r in range(2):
                ts[r].copy_(torch.from_numpy(xs[r]))
            torch.cuda.synchronize()
            for r in range(2):
                if args.no_graph:
                    comms[r].allreduce(ts[r], rdc_amd.Op.SUM, algo=args.graph_algo,
                                       stream=ctypes.c_void_p(streams[r].cuda_stream))
                else:
                    with torch.cuda.stream(streams[r]):
                        graphs[r].replay()
            for r in range(2):
                comms[r].check(ctypes.c_void_p(streams[r].cuda_stream))
            want = O.expected_allreduce(xs, O.DT_FLOAT32, O.OP_SUM)
            for r in range(2):
                got = ts[r].cpu().numpy()
                if got.tobytes() != want.tobytes():
                    fails.append({"round": rnd, "phase": "replay", "it": it, "rank": r, "counters": counters(),
                                  "diff": diff_ranges(got, want, 2)})
        xs = [rng.standard_normal(args.eager_count).astype(np.float32) for _ in range(2)]
        bufs = [torch.from_numpy(x.copy()).cuda() for x in xs]
        torch.cuda.synchronize()
        c_before = counters()
        for r in range(2):
            rc = _LIB.RdcCommAllreduceEx(comms[r].handle, ctypes.c_void_p(bufs[r].data_ptr()), args.eager_count,
                                         O.DT_FLOAT32, O.OP_SUM, args.eager_algo,
                                         ctypes.c_void_p(streams[r].cuda_stream))
            assert rc == 0, _LIB.RdcGetLastError()
        for r in range(2):
            comms[r].check(ctypes.c_void_p(streams[r].cuda_stream))
        want = O.expected_allreduce(xs, O.DT_FLOAT32, O.OP_SUM)
        for r in range(2):
            got = bufs[r].cpu().numpy()
            if got.tobytes() != want.tobytes():
                fails.append({"round": rnd, "phase": "eager", "rank": r, "counters_before": c_before,
                              "counters": counters(), "diff": diff_ranges(got, want, 2)})
        del graphs
    print(json.dumps({"rounds": args.rounds, "graph_algo": args.graph_algo, "no_graph": args.no_graph,
                      "env": {k: v for k, v in os.environ.items() if k.startswith("RDC_")},
                      "failures": len(fails), "counters": counters(), "first": fails[:6]}))
    for c in comms:
        c.destroy()
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
