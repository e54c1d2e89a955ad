"""Long randomized stress on the GPU box: the seeded fuzz of
tests/test_gpu_allreduce.py (fuzz_cases) over many seeds, worlds 2-6 and
scratch / tile / grid settings, every byte against the oracle.
    python tools/fuzz_stress.py <first seed> <runs>
FUZZ_ENV="A=1,B=2" adds variables to every run (e.g. the debug modes
RDC_POISON_SCRATCH=1,RDC_SEQ_CHECK=1)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.test_gpu_allreduce import expected_for, fuzz_cases, run_mp  # noqa: E402

first, runs = int(sys.argv[1]), int(sys.argv[2])
envs = [{}, {"RDC_SCRATCH_BYTES": "8M", "RDC_TILE_BYTES": "16K"}, {"RDC_SCRATCH_BYTES": "4M", "RDC_NBLOCKS": "5"},
        {"RDC_ALGO": "ring"}, {"RDC_ALGO": "mesh", "RDC_SCRATCH_BYTES": "16M"}, {"RDC_HOST_SERVICE": "0"},
        {"rdc_reduce_ring_mincount": "64K"}, {"RDC_HOST_PIECE_BYTES": "1M", "RDC_HOST_INLINE_BYTES": "2M"}]
extra = dict(kv.split("=", 1) for kv in os.environ.get("FUZZ_ENV", "").replace(";", ",").split(",") if "=" in kv)
fails = 0
for k in range(runs):
    seed = first + k
    world = 2 + seed % 5
    env = dict(envs[seed % len(envs)], **extra)
    t0 = time.time()
    cases = fuzz_cases(seed, world, n=30)
    if "rdc_reduce_ring_mincount" in env:  # the expected order: the tree's at or below it (any schedule)
        for c in cases:
            c["mincount"] = 64 << 10
    bad = []
    try:
        tmp = run_mp(world, cases, timeout=400, env_extra=env)
        for i, c in enumerate(cases):
            want = expected_for(c, world)
            for r in range(world):
                got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
                if got.tobytes() != np.frombuffer(want[r].tobytes(), dtype=np.uint8).tobytes():
                    bad.append((i, r, c))
    except Exception as e:  # noqa: BLE001 - reported
        bad.append(("run", str(e)[-2000:]))
    print("seed %d world %d env %s: %s (%.1f s)" % (seed, world, env, "OK" if not bad else "FAIL %r" % bad[:3],
                                                   time.time() - t0), flush=True)
    if bad:
        fails += 1
        break  # stop at the first failure: read it before running more
sys.exit(1 if fails else 0)
