"""GPU: randomized chains mixing every collective kind and schedule on one
communicator, stream-ordered with no host synchronisation between launches
(tests/mp_mixed_worker.py), as 3 and 4 processes on GPU 0 — exercises the
cross-launch protocol (one-shot slot halves and post-one-shot gates,
broadcast/allgather done-word gates, forwarded broadcasts, unit-table
coalesced launches) the way a training step interleaves them.  Every op's
output is checked bit-exactly against the CPU oracle."""
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

from tests.conftest import ROOT, free_port
from tests.mixed_plan import expected, make_plan

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.mark.parametrize("world,seed", [(3, 11), (4, 12), (3, 13)])
def test_mixed_collective_chain(world, seed):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    nops = 40
    tmp = tempfile.mkdtemp(prefix="rdc_mixed_")
    port = free_port()
    env = dict(os.environ, RDC_DEVICE="0", RDC_NBLOCKS="32", RDC_SCRATCH_BYTES="64M")
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_mixed_worker.py"), str(r), str(world),
                               str(port), tmp, str(seed), str(nops)], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(world)]
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=150)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    report = "\n".join("--- rank %d rc=%s\n%s" % (r, p.returncode, o[-2000:]) for r, (p, o) in enumerate(zip(procs, outs)))
    for p in procs:
        assert p.returncode == 0, report
    want = expected(make_plan(seed, nops, world), world)
    for r in range(world):
        got = np.load(os.path.join(tmp, "mixed_rank%d.npy" % r))
        assert got.size == want.size, (r, got.size, want.size)
        if got.tobytes() != want.tobytes():
            bad = np.nonzero(got != want)[0]
            raise AssertionError("rank %d: %d bytes differ, first at %d" % (r, bad.size, bad[0]))
