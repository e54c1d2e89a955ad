"""Host-pipeline diagnostic: run host allreduces of int8 buffers whose Split
boundary is not 16-B aligned and report, per window, whether the result
matches the oracle (first differing element and how many differ).
usage: python tools/diag_host_windows.py <count> [<world> [<dtype> ...]]   (env passes through)
Buffers up to 1 Mi elements are compared whole."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from tests.test_gpu_allreduce import run_mp  # noqa: E402

count = int(sys.argv[1])
world = int(sys.argv[2]) if len(sys.argv) > 2 else 2
dtypes = [int(x) for x in sys.argv[3:]] or [0]
W = 4096
starts = {0, max(0, count - W)}
for b, _ in O.split(count, world)[1:]:
    starts.add(b - W // 2)
# every 8 MiB piece boundary region too
step = 8 << 20
for x in range(step, count, step):
    starts.add(x - W // 2)
wins = sorted((st, min(W, count - st)) for st in starts if st >= 0)
if count <= (1 << 20):
    wins = [(0, count)]
seed = 0x5EED9000
cases = [{"count": count, "dtype": dt, "op": 2, "kind": "host_allreduce", "seed": seed, "windows": wins}
         for dt in dtypes]
tmp = run_mp(world, cases, timeout=600)
for i, dt in enumerate(dtypes):
    bad = 0
    for r in range(world):
        got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r))).view(O.NP_DTYPE[dt])
        pos = 0
        for st, m in wins:
            want = O.expected_window(count, st, m, world, dt, 2, seed)
            g = got[pos:pos + m]
            pos += m
            d = np.nonzero((g.view(np.uint8).reshape(m, -1) != want.view(np.uint8).reshape(m, -1)).any(axis=1))[0]
            if d.size:
                bad += 1
                if bad <= 6:
                    print("dtype %d rank %d window [%d,%d): %d differ, first at element %d: got %r want %r"
                          % (dt, r, st, st + m, d.size, st + d[0], g[d[:4]], want[d[:4]]), flush=True)
    print("count %d world %d dtype %d windows %d bad %d env NT=%s RAMP=%s" % (
        count, world, dt, len(wins), bad, os.environ.get("RDC_HOST_NT_COPY"),
        os.environ.get("RDC_HOST_PIECE_RAMP")), flush=True)
