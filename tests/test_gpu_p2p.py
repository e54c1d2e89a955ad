"""GPU: point-to-point Send/Recv (ICommunicator::ISend/IRecv,
include/comm/communicator.h:56-80; rdc/comm.py isend/irecv) over the device
path — the sender's copy kernel writes each piece into the receiver's
IPC-mapped slot, the receiver copies it out.  Bit-exact byte transport.

* single-process group of 2 ranks on GPU 0 (both engines in one process);
* multi-process: test/sendrecv.cc's "hello world %u" stream and
  pytest/comm.py's Buffer exchange as 2 processes, a 3-process ring of
  multi-piece device buffers (tests/mp_p2p_worker.py).
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from tests.conftest import ROOT, free_port

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

SLOT = 4 << 20  # CommConfig::p2p_slot_bytes default


@pytest.fixture(scope="module")
def pair():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import rdc_amd
    g = rdc_amd.init_group([0, 0], scratch_bytes=16 << 20)
    yield g
    for c in g:
        c.destroy()


def rand_bytes(n, seed):
    return np.random.default_rng(seed).integers(0, 256, size=n, dtype=np.uint8)


@pytest.mark.parametrize("nbytes", [1, 4095, SLOT, SLOT + 1, 2 * SLOT + 12345, 10 << 20])
def test_device_to_device(pair, nbytes):
    a, b = pair
    x = rand_bytes(nbytes, nbytes)
    src = torch.from_numpy(x).cuda()
    dst = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    wr = b.irecv(dst, 0)
    ws = a.isend(src, 1)
    assert ws.wait() == 0 and wr.wait() == 0
    import rdc_amd
    assert ws.status() == rdc_amd.WS_FINISHED and wr.status() == rdc_amd.WS_FINISHED
    assert np.array_equal(dst.cpu().numpy(), x)


def test_host_and_device_mixed(pair):
    """host ndarray -> device tensor, device tensor -> host ndarray, host -> host"""
    a, b = pair
    n = 3 * SLOT + 77
    x = rand_bytes(n, 1)
    d = torch.zeros(n, dtype=torch.uint8, device="cuda")
    ws, wr = a.isend(x, 1), b.irecv(d, 0)
    ws.wait(), wr.wait()
    assert np.array_equal(d.cpu().numpy(), x)
    y = np.zeros(n, np.uint8)
    ws, wr = b.isend(d, 0), a.irecv(y, 1)
    ws.wait(), wr.wait()
    assert np.array_equal(y, x)
    f = np.arange(1001, dtype=np.float32) * 0.5
    g = np.zeros_like(f)
    ws, wr = a.isend(f, 1), b.irecv(g, 0)
    ws.wait(), wr.wait()
    assert np.array_equal(f, g)


def test_many_messages_in_order_both_directions(pair):
    """Messages on one (src, dst) pair match in post order; both directions at once."""
    a, b = pair
    sizes = [17, SLOT, 5, 2 * SLOT + 3, 1 << 20, 64, 3 * SLOT, 9]
    xs = [torch.from_numpy(rand_bytes(s, 100 + i)).cuda() for i, s in enumerate(sizes)]
    ys = [torch.from_numpy(rand_bytes(s, 200 + i)).cuda() for i, s in enumerate(sizes)]
    rx = [torch.zeros(s, dtype=torch.uint8, device="cuda") for s in sizes]
    ry = [torch.zeros(s, dtype=torch.uint8, device="cuda") for s in sizes]
    torch.cuda.synchronize()
    ws = [a.isend(x, 1) for x in xs] + [b.isend(y, 0) for y in ys]
    wr = [b.irecv(r, 0) for r in rx] + [a.irecv(r, 1) for r in ry]
    for w in ws + wr:
        w.wait()
    for x, r in zip(xs, rx):
        assert torch.equal(x, r)
    for y, r in zip(ys, ry):
        assert torch.equal(y, r)


def test_recv_posted_first_and_stream_ordering(pair):
    """irecv before isend; the send's data is produced on the current stream
    right before isend with no host sync (the engine waits for that stream)."""
    a, b = pair
    n = 2 * SLOT + 100
    dst = torch.zeros(n, dtype=torch.uint8, device="cuda")
    wr = b.irecv(dst, 0)
    src = torch.empty(n, dtype=torch.uint8, device="cuda")
    torch.cuda._sleep(20_000_000)  # ~10 ms of GPU time queued ahead of the fill
    src.fill_(0xA5)
    ws = a.isend(src, 1)
    ws.wait(), wr.wait()
    assert int((dst != 0xA5).sum()) == 0


def test_zero_bytes(pair):
    a, b = pair
    e = torch.zeros(0, dtype=torch.uint8, device="cuda")
    assert a.isend(e, 1).wait() == 0
    assert b.irecv(e, 0).wait() == 0


def test_size_mismatch_is_an_error(pair):
    import rdc_amd
    a, b = pair
    src = torch.ones(1000, dtype=torch.uint8, device="cuda")
    dst = torch.zeros(999, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ws = a.isend(src, 1)
    wr = b.irecv(dst, 0)
    ws.wait()
    with pytest.raises(rdc_amd.RdcError, match="size mismatch"):
        wr.wait()
    assert wr.status() == rdc_amd.WS_ERROR
    # the pair is still usable for matched messages afterwards?  No: the
    # receiver's lane consumed nothing, so re-sync it by receiving the piece.
    fix = torch.zeros(1000, dtype=torch.uint8, device="cuda")
    b.irecv(fix, 0).wait()
    assert int(fix.sum()) == 1000


def test_bad_rank_rejected(pair):
    import rdc_amd
    a, _ = pair
    t = torch.zeros(4, dtype=torch.uint8, device="cuda")
    with pytest.raises(rdc_amd.RdcError, match="bad destination"):
        a.isend(t, 0)
    with pytest.raises(rdc_amd.RdcError, match="bad source"):
        a.irecv(t, 5)


def test_drop_pending_completion(pair):
    """Deleting a WorkComp handle before completion is safe (two owners)."""
    a, b = pair
    n = SLOT * 2
    src = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    dst = torch.zeros(n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ws = a.isend(src, 1)
    del ws
    b.irecv(dst, 0).wait()
    assert int((dst != 7).sum()) == 0


def run_workers(world, mode, timeout=180, env_extra=None):
    port = free_port()
    env = dict(os.environ, RDC_DEVICE="0", RDC_SCRATCH_BYTES="16M", RDC_NBLOCKS="16")
    env.update(env_extra or {})
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_p2p_worker.py"), str(r), str(world),
                               str(port), mode], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(world)]
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=timeout)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    report = "\n".join("--- rank %d rc=%s\n%s" % (r, p.returncode, o[-2000:]) for r, (p, o) in enumerate(zip(procs, outs)))
    for r, p in enumerate(procs):
        assert p.returncode == 0, report
        assert "rank %d: %s OK" % (r, mode) in outs[r], report
    return outs


def test_mp_sendrecv_hello_world():
    """test/sendrecv.cc: rank 0 sends "hello world %u " 100 times, rank 1
    (sleeping before its first receive) checks each; plus pytest/comm.py."""
    run_workers(2, "hello")


def test_mp_ring_device_buffers():
    """3 processes: every rank sends a multi-piece device buffer to the next
    and receives from the previous, several rounds, bit-exact."""
    run_workers(3, "ring")


@pytest.mark.parametrize("world", [2, 3])
def test_mp_sendrecv_fuzz(world):
    """60 seeded messages between random pairs (0 B .. ~24 MiB, device or host
    buffers on either side, multi-piece, up to 8 in flight per rank), every
    byte checked on the receiver."""
    run_workers(world, "fuzz", timeout=300)


def test_mp_peer_never_sends_times_out():
    """A receive whose sender never posts ends in error after RDC_TIMEOUT."""
    run_workers(2, "timeout", env_extra={"RDC_TIMEOUT": "3"})
