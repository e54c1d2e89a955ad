"""Seeded plan of a mixed-collective chain (tests/mp_mixed_worker.py) and its
expected output computed with the CPU oracle (tests/test_gpu_mixed.py; the
plan itself is checked on CPU in tests/test_plan.py)."""
import random

import numpy as np

ESZ = {0: 1, 1: 1, 2: 4, 3: 4, 4: 8, 5: 8, 6: 4, 7: 8, 8: 8, 9: 8, 10: 2, 11: 2}
# (dtype, op) pairs with reference semantics (BitOR only on integers)
PAIRS = [(6, 2), (6, 0), (7, 2), (2, 2), (2, 3), (10, 2), (11, 2), (4, 1), (1, 0)]


def make_plan(seed, nops, world):
    rng = random.Random(seed)
    plan = []
    for k in range(nops):
        kind = rng.choice(["allreduce", "allreduce", "bcast", "allgather", "coalesced", "host"])
        s = 0x5EED0000 + 1000 * k
        if kind == "allreduce":
            dt, op = rng.choice(PAIRS)
            count = rng.choice([1, 7, 1000, 4099, 65536 + 3, 300001])
            plan.append({"kind": kind, "count": count, "dtype": dt, "op": op, "algo": rng.choice([0, 1, 2, 3]),
                         "seed": s})
        elif kind == "bcast":
            plan.append({"kind": kind, "bytes": rng.choice([1, 100, 4096, 100003, 1 << 20, 3 << 20]),
                         "root": rng.randrange(world), "seed": s})
        elif kind == "allgather":
            plan.append({"kind": kind, "sizes": [rng.choice([0, 3, 64, 5000, 70001]) for _ in range(world)],
                         "seed": s})
        elif kind == "host":  # synchronous, host buffer: the small-allreduce service or the launch path
            dt, op = rng.choice(PAIRS)
            plan.append({"kind": kind, "count": rng.choice([1, 7, 1000, 4099, 16384, 20000]), "dtype": dt, "op": op,
                         "seed": s})
        else:
            dt, op = rng.choice([(6, 2), (2, 0), (10, 2)])
            nb = rng.randint(2, 9)
            plan.append({"kind": kind, "counts": [rng.choice([0, 1, 5, 1024, 33333, 131072]) for _ in range(nb)],
                         "dtype": dt, "op": op, "algo": rng.choice([0, 0, 1, 2, 3]), "seed": s})
    return plan


def output_bytes(plan):
    """Total bytes of every op's outputs, in the worker's order."""
    tot = 0
    for op in plan:
        if op["kind"] in ("allreduce", "host"):
            tot += op["count"] * ESZ[op["dtype"]]
        elif op["kind"] == "bcast":
            tot += op["bytes"]
        elif op["kind"] == "allgather":
            tot += sum(op["sizes"])
        else:
            tot += sum(op["counts"]) * ESZ[op["dtype"]]
    return tot


def expected(plan, world):
    """Concatenated bytes every rank must hold after the chain (allreduce and
    broadcast results are identical everywhere, and allgather lands every
    rank's data everywhere)."""
    from oracle import oracle as O
    parts = []
    for op in plan:
        kind = op["kind"]
        if kind in ("allreduce", "host"):
            xs = [O.fill(op["count"], op["dtype"], op["seed"], r) for r in range(world)]
            parts.append(np.frombuffer(O.expected_allreduce(xs, op["dtype"], op["op"]).tobytes(), np.uint8))
        elif kind == "bcast":
            parts.append(np.frombuffer(O.fill(op["bytes"], 1, op["seed"], op["root"]).tobytes(), np.uint8))
        elif kind == "allgather":
            for r, s in enumerate(op["sizes"]):
                parts.append(np.frombuffer(O.fill(s, 1, op["seed"], r).tobytes(), np.uint8))
        else:
            for b, c in enumerate(op["counts"]):
                xs = [O.fill(c, op["dtype"], op["seed"] + b, r) for r in range(world)]
                parts.append(np.frombuffer(O.expected_allreduce(xs, op["dtype"], op["op"]).tobytes(), np.uint8))
    return np.concatenate(parts) if parts else np.zeros(0, np.uint8)
