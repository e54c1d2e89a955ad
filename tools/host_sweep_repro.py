"""The host size sweep of tests/test_gpu_allreduce.py (test_mp_host_size_sweep)
at any rank count, K times, every byte against the oracle: the rehearsal of
round 4's lost one-shot hand-off outside pytest.

    python tools/host_sweep_repro.py WORLD [K]
Environment passes through (RDC_DEBUG_LDS_PAD, GPU_MAX_HW_QUEUES with
RDC_TEST_KEEP_QUEUES=1, RDC_TIMEOUT, ...).  Prints one line per run."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.test_gpu_allreduce import HOST_SWEEP_BYTES, expected_for, run_mp  # noqa: E402

world = int(sys.argv[1])
K = int(sys.argv[2]) if len(sys.argv) > 2 else 1
cases = []
for k, nb in enumerate(HOST_SWEEP_BYTES):
    cases.append({"count": nb, "dtype": 1, "op": (0, 2)[k % 2], "kind": "host_allreduce", "seed": 0x5EEDA000 + k})
    cases.append({"count": nb // 4 + 1, "dtype": 6, "op": 2, "kind": "host_allreduce", "seed": 0x5EEDB000 + k})
fails = 0
for run in range(K):
    t0 = time.time()
    try:
        tmp = run_mp(world, cases, timeout=300, env_extra={"RDC_HOST_BALANCE": "0"})
        bad = []
        for i, c in enumerate(cases):
            want = expected_for(c, world)
            for r in range(world):
                got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
                if got.tobytes() != np.frombuffer(want[r].tobytes(), dtype=np.uint8).tobytes():
                    bad.append((i, r))
        msg = "OK" if not bad else "WRONG %r" % bad[:4]
    except AssertionError as e:
        msg = "FAIL " + " | ".join(ln[:260] for ln in str(e).splitlines() if "failed on" in ln)[:1500]
    fails += msg != "OK"
    print("world %d run %d queues %s: %s (%.1f s)" % (world, run, os.environ.get("GPU_MAX_HW_QUEUES"), msg,
                                                      time.time() - t0), flush=True)
sys.exit(1 if fails else 0)
