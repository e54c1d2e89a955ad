"""Generate tests/golden/ring_allreduce.npz — golden vectors for the ring allreduce.

Expected outputs come from oracle/_ref/libref_ring.so: the reference's OWN
op::Reducer<OP,DType> (include/core/mpi.h:113-120) and utils::Split
(include/utils/utils.h:59-70), compiled from /root/reference/include, driven
by the restated ring schedule (src/comm/communicator_collective.cc:79-203).
Every rank's output is checked identical before rank 0's is stored.

float16 cases (no reference half type, mpi.h:40-81) come from the C oracle
alone and are flagged ``oracle_only``: parity for them is unpinned by the
reference.

Run (needs /root/reference to rebuild oracle/_ref):  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle as O  # noqa: E402

SEED = 0x5EED0000


def inputs_for(rng, n, count, dtype):
    npd = O.NP_DTYPE[dtype]
    if dtype in (O.DT_FLOAT32, O.DT_FLOAT64, O.DT_FLOAT16):
        # full-mantissa values at mixed magnitudes (a coarse grid hides order effects)
        return [(rng.standard_normal(count) * rng.choice([1e-2, 1.0, 1e2], count)).astype(npd) for _ in range(n)]
    info = np.iinfo(npd)
    return [rng.integers(info.min, info.max, count, dtype=npd, endpoint=True) for _ in range(n)]


def cases():
    out = []
    for n in (2, 3, 5, 8):
        for count in sorted({1, n - 1, 7, 1001, 4099}):
            if count >= 1:
                out.append((n, count, O.DT_FLOAT32, O.OP_SUM))
    out += [
        (3, 1001, O.DT_FLOAT32, O.OP_MAX), (5, 1001, O.DT_FLOAT32, O.OP_MIN),
        (8, 1001, O.DT_FLOAT64, O.OP_SUM), (4, 4099, O.DT_FLOAT64, O.OP_MAX),
        (5, 1001, O.DT_INT32, O.OP_SUM), (3, 513, O.DT_INT8, O.OP_SUM),
        (6, 777, O.DT_UINT8, O.OP_BITOR), (7, 1001, O.DT_INT64, O.OP_MAX),
        (4, 1001, O.DT_UINT32, O.OP_MIN), (8, 999, O.DT_LONGLONG, O.OP_SUM),
        (2, 1001, O.DT_FLOAT16, O.OP_SUM), (8, 1001, O.DT_FLOAT16, O.OP_SUM),
    ]
    return out


def main():
    O.build()
    if not O.ref_available():
        raise SystemExit("oracle/_ref not built (needs /root/reference)")
    rng = np.random.default_rng(SEED)
    blob = {}
    meta = []
    for k, (n, count, dt, op) in enumerate(cases()):
        xs = inputs_for(rng, n, count, dt)
        oracle_only = dt == O.DT_FLOAT16
        bufs = [x.copy() for x in xs]
        if oracle_only:
            O.allreduce_ring(bufs, dt, op)
        else:
            O.ref_allreduce_ring(bufs, dt, op)
        for r in range(1, n):
            assert bufs[r].tobytes() == bufs[0].tobytes(), "ranks disagree"
        blob["c%d_in" % k] = np.stack(xs)
        blob["c%d_out" % k] = bufs[0]
        meta.append([n, count, dt, op, int(oracle_only)])
    blob["meta"] = np.array(meta, dtype=np.int64)
    path = os.path.join(HERE, "ring_allreduce.npz")
    np.savez_compressed(path, **blob)
    print("wrote %s (%d cases, %d bytes)" % (path, len(meta), os.path.getsize(path)))


if __name__ == "__main__":
    main()
