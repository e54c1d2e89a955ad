"""Randomized stress of mixed collective chains (tests/mp_mixed_worker.py) at
2-5 processes on GPU 0, 80 ops per run, every output checked bit-exactly
against the CPU oracle.  python tests/stress_mixed.py (on the GPU box)."""
import os, subprocess, sys, tempfile
import numpy as np
sys.path.insert(0, os.getcwd())
from tests.mixed_plan import expected, make_plan
from tests.conftest import free_port
fails = 0
for world, seed in [(2, 21), (3, 22), (4, 23), (5, 24), (3, 25), (4, 26), (2, 27), (5, 28)]:
    nops = 80
    tmp = tempfile.mkdtemp()
    port = free_port()
    env = dict(os.environ, RDC_DEVICE="0", RDC_NBLOCKS="24", RDC_SCRATCH_BYTES="64M")
    ps = [subprocess.Popen([sys.executable, "tests/mp_mixed_worker.py", str(r), str(world), str(port), tmp, str(seed), str(nops)],
                           env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(world)]
    outs = [p.communicate(timeout=200)[0] for p in ps]
    ok = all(p.returncode == 0 for p in ps)
    if ok:
        want = expected(make_plan(seed, nops, world), world)
        for r in range(world):
            got = np.load(os.path.join(tmp, "mixed_rank%d.npy" % r))
            if got.tobytes() != want.tobytes():
                ok = False
    print("world %d seed %d: %s" % (world, seed, "OK" if ok else "FAIL"), flush=True)
    if not ok:
        fails += 1
        for o in outs: print(o[-1500:])
sys.exit(1 if fails else 0)
