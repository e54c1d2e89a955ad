"""GPU parity of the device allreduce / broadcast against the CPU oracle
(the reference's ring, bit-exact), through the C ABI.

* single-process groups: n communicators on GPU 0, one stream each;
* multi-process: n processes on GPU 0 exchanging HIP IPC handles over the
  TCP bootstrap — the same code path as one process per GPU on an 8-GPU node.
"""
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np
import pytest

from oracle import oracle as O
from tests.conftest import ROOT, free_port
from tests.gpu_util import VALID, from_dev, ptr, rand_input, same_bits, to_dev

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


# Ranks of a single-process group that share one GPU must run concurrently:
# each gets ONE stream for the whole module, created up front, so every rank
# sits on its own hardware queue (the box exports GPU_MAX_HW_QUEUES=4, HIP's
# default; groups here have at most 3 ranks).
# Creating fresh streams per call would eventually put two ranks on one
# queue, serialising a waiting kernel in front of the one it waits for.
class Group(list):
    streams = None


def make_group(n, scratch):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import rdc_amd
    g = Group(rdc_amd.init_group([0] * n, scratch_bytes=scratch))
    g.streams = [torch.cuda.Stream() for _ in range(n)]
    return g


@pytest.fixture(scope="module")
def group3():
    g = make_group(3, 24 << 20)
    yield g
    for c in g:
        c.destroy()


@pytest.fixture(scope="module")
def group2():
    g = make_group(2, 16 << 20)
    yield g
    for c in g:
        c.destroy()


def run_group(comms, inputs, dtype, op, algo, pads=None):
    """Launch every rank's allreduce on its own stream, then collect."""
    from rdc_amd._lib import _LIB
    import ctypes
    n = len(comms)
    count = inputs[0].size
    pads = pads or [0] * n
    esz = np.dtype(O.NP_DTYPE[dtype]).itemsize
    bufs = [to_dev(x, p * esz) for x, p in zip(inputs, pads)]
    streams = comms.streams
    torch.cuda.synchronize()
    for r in range(n):
        rc = _LIB.RdcCommAllreduceEx(comms[r].handle, ptr(bufs[r], pads[r] * esz), count, dtype, op, algo,
                                     ctypes.c_void_p(streams[r].cuda_stream))
        assert rc == 0, _LIB.RdcGetLastError()
    for r in range(n):
        comms[r].check(ctypes.c_void_p(streams[r].cuda_stream))
    return [from_dev(bufs[r], pads[r] * esz, count, dtype) for r in range(n)]


@pytest.mark.parametrize("algo", [1, 2, 3, 5])
@pytest.mark.parametrize("dtype,op", VALID)
def test_group3_all_types(group3, dtype, op, algo):
    rng = np.random.default_rng(77 + dtype * 8 + op)
    for count in (1, 2, 5, 1001, 4099):
        inputs = [rand_input(rng, count, dtype) for _ in range(3)]
        want = O.expected_allreduce(inputs, dtype, op)
        got = run_group(group3, inputs, dtype, op, algo, pads=[1, 0, 3])
        for r in range(3):
            assert same_bits(got[r], want, dtype), (dtype, op, algo, count, r)


@pytest.mark.parametrize("dtype,op", VALID)
def test_group3_tree_order_all_types(group3, dtype, op):
    """algo 4: the reference's small-buffer TREE order (TryAllreduceTree,
    communicator_collective.cc:14-78; rdc_reduce_ring_mincount) for every
    (dtype, op), misaligned buffers, vs the oracle's restated tree
    (oracle/tree_order.cc).  fp32 tree parity is pinned by the restatement
    only (the reference's own .cc could not be compiled here)."""
    rng = np.random.default_rng(91 + dtype * 8 + op)
    for count in (1, 2, 5, 1001, 4099, 70001):
        inputs = [rand_input(rng, count, dtype) for _ in range(3)]
        want = O.expected_tree(inputs, dtype, op)
        got = run_group(group3, inputs, dtype, op, 4, pads=[1, 0, 3])
        for r in range(3):
            assert same_bits(got[r], want, dtype), (dtype, op, count, r)


def test_group_tree_multi_piece(group2):
    """A tree-order buffer larger than half a one-shot slot goes in pieces."""
    rng = np.random.default_rng(92)
    count = (5 << 20) // 4 + 3   # 5 MiB fp32 > half of a 8 MiB slot
    inputs = [rng.standard_normal(count).astype(np.float32) for _ in range(2)]
    got = run_group(group2, inputs, O.DT_FLOAT32, O.OP_SUM, 4, pads=[0, 1])
    want = O.expected_tree(inputs, O.DT_FLOAT32, O.OP_SUM)
    for r in range(2):
        assert same_bits(got[r], want, O.DT_FLOAT32)


@pytest.mark.parametrize("algo", [1, 2])
def test_group_multi_piece(group2, algo):
    """Buffers larger than the scratch go through several launches (pieces)."""
    rng = np.random.default_rng(5)
    count = (6 << 20) // 4 * 3 + 7   # 18 MiB fp32 > 2 x 4 MiB slots
    inputs = [rng.standard_normal(count).astype(np.float32) for _ in range(2)]
    want = O.expected_allreduce(inputs, O.DT_FLOAT32, O.OP_SUM)
    got = run_group(group2, inputs, O.DT_FLOAT32, O.OP_SUM, algo, pads=[0, 5])
    for r in range(2):
        assert same_bits(got[r], want, O.DT_FLOAT32)


@pytest.mark.parametrize("s16,r16,grid,tile", [(1, 14, 0, 0), (7, 1, 24, 0), (3, 10, 48, 64 << 10),
                                               (5, 5, 16, 16 << 10)])
def test_group_tuned_mesh_bit_exact(group3, s16, r16, grid, tile):
    """RdcCommTune (role split, grid, tile) changes only who moves which
    bytes: the result stays the oracle's bits; defaults restored after."""
    rng = np.random.default_rng(s16 * 100 + r16)
    try:
        for c in group3:
            c.tune(s16, r16, grid, tile)
        for count in (3, 70001, (3 << 20) // 4 + 5):
            inputs = [rng.standard_normal(count).astype(np.float32) for _ in range(3)]
            want = O.expected_allreduce(inputs, O.DT_FLOAT32, O.OP_SUM)
            got = run_group(group3, inputs, O.DT_FLOAT32, O.OP_SUM, 2, pads=[0, 1, 2])
            for r in range(3):
                assert same_bits(got[r], want, O.DT_FLOAT32), (count, r)
    finally:
        for c in group3:
            c.tune()


def test_tune_rejects_bad_split(group2):
    import rdc_amd
    with pytest.raises(rdc_amd.RdcError):
        group2[0].tune(8, 8)
    with pytest.raises(rdc_amd.RdcError):
        group2[0].tune(4, 8, 0, 100)


def test_group_repeated_calls(group3):
    """seq-numbered flags: many back-to-back launches on the same communicator,
    schedules interleaved (one-shot parity halves, gates after one-shot)."""
    rng = np.random.default_rng(9)
    for it in range(40):
        count = int(rng.integers(1, 70000))
        algo = int(rng.choice([0, 1, 2, 3, 5]))
        inputs = [rng.standard_normal(count).astype(np.float32) for _ in range(3)]
        want = O.expected_allreduce(inputs, O.DT_FLOAT32, O.OP_SUM)
        got = run_group(group3, inputs, O.DT_FLOAT32, O.OP_SUM, algo)
        for r in range(3):
            assert same_bits(got[r], want, O.DT_FLOAT32), (it, count, algo)


@pytest.mark.parametrize("start", [(1 << 23) - 2, (1 << 32) - 3, (1 << 40) + 5])
def test_group_launch_counter_far_past_zeroed_flags(start, algo_counts=((2, 300007), (1, 300007), (3, 70001),
                                                                         (4, 4099), (0, 1 << 20))):
    """Hand-off flags are zeroed once, when the channel is made; the launch
    counter keeps growing.  On a FRESH group (every flag slot still 0) with
    the counter started at 2^23 - 2, 2^32 - 3 and 2^40 + 5 — past where a
    24-bit or 32-bit counter compare would read a never-written 0 as
    "reached"  — mesh, ring, one-shot, tree and auto launches on
    slots no earlier launch wrote stay bit-exact, broadcast and allgather
    too, and the counter advances by one per launch across 2^23 / 2^32."""
    import ctypes
    from rdc_amd._lib import _LIB
    g = make_group(3, 24 << 20)
    try:
        for c in g:
            assert _LIB.RdcCommSetLaunchCounter(c.handle, start) == 0, _LIB.RdcGetLastError()
        rng = np.random.default_rng(start & 0xFFFF)
        launches = 0
        for algo, count in algo_counts:
            inputs = [rng.standard_normal(count).astype(np.float32) for _ in range(3)]
            want = (O.expected_tree if algo == 4 else O.expected_allreduce)(inputs, O.DT_FLOAT32, O.OP_SUM)
            got = run_group(g, inputs, O.DT_FLOAT32, O.OP_SUM, algo)
            for r in range(3):
                assert same_bits(got[r], want, O.DT_FLOAT32), (start, algo, count, r)
            v = ctypes.c_uint64()
            assert _LIB.RdcCommLaunchCounter(g[0].handle, ctypes.byref(v)) == 0
            assert v.value > start + launches, (start, algo, v.value)
            launches = v.value - start
        data = [rng.integers(0, 256, (3 << 20) + 5, dtype=np.uint8) for _ in range(3)]
        bufs = [to_dev(d, r) for r, d in enumerate(data)]
        torch.cuda.synchronize()
        for r in range(3):
            assert _LIB.RdcCommBroadcast(g[r].handle, ptr(bufs[r], r), data[0].size, 2,
                                         ctypes.c_void_p(g.streams[r].cuda_stream)) == 0
        for r in range(3):
            g[r].check(ctypes.c_void_p(g.streams[r].cuda_stream))
            assert from_dev(bufs[r], r, data[0].size, O.DT_UINT8).tobytes() == data[2].tobytes()
        sizes = [1 << 20, 7, (2 << 20) + 1]
        data = [rng.integers(0, 256, s, dtype=np.uint8) for s in sizes]
        bufs = [[to_dev(data[c] if c == r else np.zeros(sizes[c], np.uint8), 0) for c in range(3)] for r in range(3)]
        torch.cuda.synchronize()
        for r in range(3):
            ptrs = (ctypes.c_void_p * 3)(*[bufs[r][c].data_ptr() for c in range(3)])
            assert _LIB.RdcCommAllgather(g[r].handle, ptrs, (ctypes.c_size_t * 3)(*sizes),
                                         ctypes.c_void_p(g.streams[r].cuda_stream)) == 0
        for r in range(3):
            g[r].check(ctypes.c_void_p(g.streams[r].cuda_stream))
            for c in range(3):
                assert from_dev(bufs[r][c], 0, sizes[c], O.DT_UINT8).tobytes() == data[c].tobytes()
        counters = []
        for c in g:
            v = ctypes.c_uint64()
            assert _LIB.RdcCommLaunchCounter(c.handle, ctypes.byref(v)) == 0
            counters.append(v.value)
        assert len(set(counters)) == 1 and counters[0] >= start + len(algo_counts) + 2, counters
    finally:
        for c in g:
            c.destroy()


def launch_counters(comms):
    import ctypes
    from rdc_amd._lib import _LIB
    out = []
    for c in comms:
        v = ctypes.c_uint64()
        assert _LIB.RdcCommLaunchCounter(c.handle, ctypes.byref(v)) == 0, _LIB.RdcGetLastError()
        out.append(v.value)
    return out


def mismatch_report(got, want, n):
    """Element ranges where got differs from want, with the Split chunk each
    starts in (rank 0's own chunk is folded by its reduce role, the others
    are gathered from their owners)."""
    bad = np.flatnonzero(np.frombuffer(got.tobytes(), np.uint32) != np.frombuffer(want.tobytes(), np.uint32))
    if bad.size == 0:
        return "equal"
    k, m = divmod(want.size, n)
    starts = [c * k + min(c, m) for c in range(n)]
    runs, lo, prev = [], bad[0], bad[0]
    for i in bad[1:]:
        if i != prev + 1:
            runs.append((lo, prev + 1))
            lo = i
        prev = i
    runs.append((lo, prev + 1))
    return "; ".join("[%d, %d) in chunk %d" % (a, b, max(c for c in range(n) if starts[c] <= a)) for a, b in runs[:6])


@pytest.mark.parametrize("algo", ["mesh", "ring", "oneshot", "mesh_pull"])
def test_group_graph_capture_replay(group2, algo):
    """Launch sequence numbers live on the device, so a captured allreduce
    replays correctly (graph per rank, several replays with fresh inputs),
    and eager launches on the same communicators afterwards stay exact.
    Runs in poison mode (RdcCommSetPoison): every consumed scratch range is
    overwritten with 0xFF, so a read ahead of its producer's publish lands
    NaNs.  Both ranks' device launch counters must agree after the replays
    (GPUTEST_r04 failed here once: rank 0's own chunk wrong in the eager
    mesh launch)."""
    import ctypes
    import rdc_amd
    rng = np.random.default_rng(21)
    count = 300007
    for c in group2:
        c.set_poison(True)
    try:
        ts = [torch.zeros(count, dtype=torch.float32, device="cuda") for _ in range(2)]
        graphs = []
        torch.cuda.synchronize()
        for r in range(2):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=group2.streams[r], capture_error_mode="thread_local"):
                group2[r].allreduce(ts[r], rdc_amd.Op.SUM, algo=algo,
                                    stream=ctypes.c_void_p(group2.streams[r].cuda_stream))
            graphs.append(g)
        torch.cuda.synchronize()
        for it in range(4):
            xs = [rng.standard_normal(count).astype(np.float32) for _ in range(2)]
            for r in range(2):
                ts[r].copy_(torch.from_numpy(xs[r]))
            torch.cuda.synchronize()
            for r in range(2):
                with torch.cuda.stream(group2.streams[r]):
                    graphs[r].replay()
            for r in range(2):
                group2[r].check(ctypes.c_void_p(group2.streams[r].cuda_stream))
            want = O.expected_allreduce(xs, O.DT_FLOAT32, O.OP_SUM)
            for r in range(2):
                got = ts[r].cpu().numpy()
                assert got.tobytes() == want.tobytes(), (algo, it, r, mismatch_report(got, want, 2))
        ctr = launch_counters(group2)
        assert ctr[0] == ctr[1], ("launch counters differ after the replays", ctr)
        # eager launches interleave with replays on the same communicators
        for eager_algo in (2, 5, 1, 0):
            xs = [rng.standard_normal(1001).astype(np.float32) for _ in range(2)]
            got = run_group(group2, xs, O.DT_FLOAT32, O.OP_SUM, eager_algo)
            want = O.expected_allreduce(xs, O.DT_FLOAT32, O.OP_SUM)
            for r in range(2):
                assert got[r].tobytes() == want.tobytes(), (algo, eager_algo, r, launch_counters(group2),
                                                            mismatch_report(got[r], want, 2))
        for it in range(2):  # and replays again after them
            xs = [rng.standard_normal(count).astype(np.float32) for _ in range(2)]
            for r in range(2):
                ts[r].copy_(torch.from_numpy(xs[r]))
            torch.cuda.synchronize()
            for r in range(2):
                with torch.cuda.stream(group2.streams[r]):
                    graphs[r].replay()
            for r in range(2):
                group2[r].check(ctypes.c_void_p(group2.streams[r].cuda_stream))
            want = O.expected_allreduce(xs, O.DT_FLOAT32, O.OP_SUM)
            for r in range(2):
                got = ts[r].cpu().numpy()
                assert got.tobytes() == want.tobytes(), (algo, "after eager", it, r, mismatch_report(got, want, 2))
        ctr = launch_counters(group2)
        assert ctr[0] == ctr[1], ("launch counters differ", ctr)
    finally:
        for c in group2:
            c.set_poison(False)


def test_group_broadcast(group3):
    import ctypes
    from rdc_amd._lib import _LIB
    rng = np.random.default_rng(3)
    for root in range(3):
        for nbytes in (1, 100, 1 << 20 | 3, (5 << 20) + 7):
            data = [rng.integers(0, 256, nbytes, dtype=np.uint8) for _ in range(3)]
            bufs = [to_dev(d, 1 + r) for r, d in enumerate(data)]
            streams = group3.streams
            torch.cuda.synchronize()
            for r in range(3):
                assert _LIB.RdcCommBroadcast(group3[r].handle, ptr(bufs[r], 1 + r), nbytes, root,
                                             ctypes.c_void_p(streams[r].cuda_stream)) == 0
            for r in range(3):
                group3[r].check(ctypes.c_void_p(streams[r].cuda_stream))
                assert from_dev(bufs[r], 1 + r, nbytes, O.DT_UINT8).tobytes() == data[root].tobytes()


def test_group_allgather(group3):
    """Variable-size per-rank buffers (test/allgather.cc shape, 1 B .. 3 MiB)."""
    import ctypes
    from rdc_amd._lib import _LIB
    rng = np.random.default_rng(4)
    for sizes in ([1, 2, 3], [1000, 0, 4097], [3 << 20, 5, (1 << 20) + 3], [7 << 20, 7 << 20, 1]):
        data = [rng.integers(0, 256, s, dtype=np.uint8) for s in sizes]
        # every rank allocates all n buffers (pads differ per rank and buffer)
        bufs = [[to_dev(data[c] if c == r else np.zeros(sizes[c], np.uint8), 1 + r + c) for c in range(3)]
                for r in range(3)]
        torch.cuda.synchronize()
        for r in range(3):
            ptrs = (ctypes.c_void_p * 3)(*[bufs[r][c].data_ptr() + 1 + r + c for c in range(3)])
            szs = (ctypes.c_size_t * 3)(*sizes)
            assert _LIB.RdcCommAllgather(group3[r].handle, ptrs, szs,
                                         ctypes.c_void_p(group3.streams[r].cuda_stream)) == 0, _LIB.RdcGetLastError()
        for r in range(3):
            group3[r].check(ctypes.c_void_p(group3.streams[r].cuda_stream))
            for c in range(3):
                got = from_dev(bufs[r][c], 1 + r + c, sizes[c], O.DT_UINT8)
                assert got.tobytes() == data[c].tobytes(), (sizes, r, c)


# --------------------------------------------------------------- multi-process
def run_mp(world, cases, timeout=240, env_extra=None):
    tmp = tempfile.mkdtemp(prefix="rdc_mp_")
    cf = os.path.join(tmp, "cases.json")
    with open(cf, "w") as f:
        json.dump(cases, f)
    port = free_port()
    env = dict(os.environ)
    # grids are left to the library (clamped to what stays resident with
    # `world` ranks on GPU 0) unless a test forces RDC_NBLOCKS
    env.update({"RDC_DEVICE": "0", "RDC_SCRATCH_BYTES": "64M"})
    env.update(env_extra or {})
    # every rank on GPU 0: the hardware-queue budget rdc_amd.launcher applies
    # to workers that share a GPU (8 ranks -> 2 queues each)
    from rdc_amd.launcher import hw_queues_per_process, queues_over_budget
    q = hw_queues_per_process(world)
    if (q is not None and env.get("RDC_DEVICE") != "rank" and not env.get("RDC_TEST_KEEP_QUEUES")
            and queues_over_budget(env.get("GPU_MAX_HW_QUEUES"), q)):
        env["GPU_MAX_HW_QUEUES"] = str(q)
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp_worker.py"), str(r), str(world),
                               str(port), tmp, cf], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    # RDC_TEST_MP_TIMEOUT (debug runs): a shorter limit than the test's
    if os.environ.get("RDC_TEST_MP_TIMEOUT"):
        timeout = min(timeout, float(os.environ["RDC_TEST_MP_TIMEOUT"]))
    outs = []
    deadline = time.time() + timeout
    for p in procs:
        try:
            out, _ = p.communicate(timeout=max(1.0, deadline - time.time()))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            tails = []
            for r, q in enumerate(procs):  # what every rank printed before the kill
                try:
                    o, _ = q.communicate(timeout=10)
                    tails.append("rank %d:\n%s" % (r, o.decode(errors="replace")[-1500:]))
                    if os.environ.get("RDC_TEST_MP_LOGDIR"):  # debug runs: the whole output
                        os.makedirs(os.environ["RDC_TEST_MP_LOGDIR"], exist_ok=True)
                        with open(os.path.join(os.environ["RDC_TEST_MP_LOGDIR"], "%s_rank%d_timeout.log"
                                               % (os.path.basename(tmp), r)), "wb") as f:
                            f.write(o)
                except Exception:  # noqa: BLE001
                    tails.append("rank %d: (no output)" % r)
            raise AssertionError("multi-process run timed out after %.0f s\n%s" % (timeout, "\n".join(tails)))
        outs.append(out.decode(errors="replace"))
    if os.environ.get("RDC_TEST_MP_LOGDIR"):  # debug runs: every rank's whole output
        d = os.environ["RDC_TEST_MP_LOGDIR"]
        os.makedirs(d, exist_ok=True)
        for r, o in enumerate(outs):
            with open(os.path.join(d, "%s_rank%d.log" % (os.path.basename(tmp), r)), "w") as f:
                f.write(o)
    failed = [r for r, p in enumerate(procs) if p.returncode != 0]
    assert not failed, "\n".join("rank %d failed (rc %d):\n%s" % (r, procs[r].returncode, outs[r][-1500:])
                                  for r in failed)
    return tmp


def expected_for(case, world):
    dt = case["dtype"]
    if case.get("kind") == "allgather":
        # test/allgather.cc: buffer i has i + N items, a[i][j] = i + j, gathered everywhere
        N = case["count"]
        cat = np.concatenate([np.arange(i, i + i + N, dtype=np.int32) for i in range(world)])
        return [cat] * world
    if case.get("kind") == "bcast_chain":
        acc = np.zeros(case["count"], dtype=np.int32)
        for k in range(case["steps"]):
            root = (k * 3 + 1) % world
            O.reducer(O.fill(case["count"], O.DT_INT32, case.get("seed", 0x5EED0000) + k, root), acc, O.DT_INT32,
                      O.OP_SUM)
        return [acc] * world
    esz = np.dtype(O.NP_DTYPE[dt]).itemsize
    mincount = case.get("mincount", 1)  # rdc_reduce_ring_mincount of the run (bytes)

    def reduce_all(xs, op):  # TryAllreduce: the tree's order up to mincount bytes, the ring's above
        if xs[0].size * esz <= mincount or case.get("algo") == 4:
            O.allreduce_tree(xs, dt, op)
        else:
            O.allreduce_ring(xs, dt, op)

    if case.get("kind") == "coalesced":
        per = []
        for b, k in enumerate(case["counts"]):
            xs = [O.fill(k, dt, case.get("seed", 0x5EED0000) + b, r) for r in range(world)]
            for _ in range(case.get("reps", 1)):
                reduce_all(xs, case["op"])
            per.append(xs)
        return [np.concatenate([per[b][r] for b in range(len(per))]) if per else np.zeros(0, np.uint8)
                for r in range(world)]
    inputs = [O.fill(case["count"], dt, case.get("seed", 0x5EED0000), r) for r in range(world)]
    kind = case.get("kind", "allreduce")
    if kind == "broadcast":
        return [inputs[case["root"]]] * world
    bufs = [x.copy() for x in inputs]
    for _ in range(case.get("reps", 1)):
        reduce_all(bufs, case["op"])
    return bufs


@pytest.mark.parametrize("world", [2, 3, 4])
def test_mp_allreduce(world):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cases = [
        {"count": 1, "dtype": 6, "op": 2},
        {"count": 1001, "dtype": 6, "op": 2, "algo": 2, "pad": 4},
        {"count": 1001, "dtype": 6, "op": 2, "algo": 1, "pad": 8},
        {"count": 4099, "dtype": 2, "op": 0},
        {"count": 1 << 20, "dtype": 10, "op": 2},
        {"count": 3 << 20, "dtype": 7, "op": 1, "algo": 1},
        {"count": 5 << 20, "dtype": 6, "op": 2, "algo": 2},     # 20 MiB > scratch: 2 pieces
        {"count": 5 << 20, "dtype": 6, "op": 2, "algo": 5},     # the pull-mode mesh, 2 pieces
        {"count": 1001, "dtype": 6, "op": 2, "algo": 5, "pad": 4},
        {"count": 100003, "dtype": 10, "op": 1, "algo": 5, "pad_per_rank": 2},
        {"count": 0, "dtype": 6, "op": 2, "kind": "coalesced", "counts": [1024, 7, 0, 100003, 1, 65536], "algo": 5},
        {"count": 77777, "dtype": 1, "op": 3, "comm": "second"},
        {"count": 70000, "dtype": 11, "op": 2, "reps": 3},
        {"count": 123457, "dtype": 0, "kind": "broadcast", "root": world - 1},
        {"count": (3 << 20) + 5, "dtype": 0, "kind": "broadcast", "root": 1},   # forwarded (n >= 3)
        {"count": 4096, "dtype": 6, "op": 2, "kind": "host_allreduce"},
        {"count": 25000003, "dtype": 6, "op": 2, "kind": "host_allreduce", "reps": 2},   # 7 pipelined pieces
        {"count": 3000001, "dtype": 10, "op": 0, "kind": "host_allreduce"},
        {"count": 5, "dtype": 4, "op": 2, "kind": "host_allreduce"},
        # host copies cut into parts whose floor is a 4 KiB multiple with bytes left over
        # (2 x 256 KiB + 1 B staged small path, 4 x 256 KiB + 3 B one inline piece)
        {"count": 524289, "dtype": 0, "op": 2, "kind": "host_allreduce"},
        {"count": 1048579, "dtype": 1, "op": 0, "kind": "host_allreduce"},
        {"count": 100003, "dtype": 6, "op": 2, "algo": 2, "pad_per_rank": 4},   # ranks' buffers differ mod 16
        {"count": 100003, "dtype": 10, "op": 0, "algo": 1, "pad_per_rank": 2},
        {"count": 2, "dtype": 2, "kind": "bcast_chain", "steps": 40},
        {"count": 50001, "dtype": 6, "op": 2, "algo": 3, "pad_per_rank": 4},
        {"count": 30000, "dtype": 11, "op": 2, "algo": 3, "reps": 5},
        {"count": 8191, "dtype": 6, "op": 2, "algo": 0, "reps": 7},
        {"count": 1000, "dtype": 2, "kind": "allgather"},
        {"count": 400001, "dtype": 2, "kind": "allgather"},
        {"count": 300001, "dtype": 2, "kind": "bcast_chain", "steps": 12},
        {"count": 0, "dtype": 6, "op": 2, "kind": "coalesced", "counts": [1024, 7, 0, 100003, 1, 65536], "reps": 2},
        {"count": 0, "dtype": 10, "op": 0, "kind": "coalesced", "counts": [4099] * 9, "algo": 1},
        {"count": 0, "dtype": 6, "op": 2, "kind": "coalesced", "counts": [333, 20000, 5], "algo": 3, "reps": 3},
        {"count": 0, "dtype": 2, "op": 2, "kind": "coalesced", "counts": [3, 1000, 77], "host": True},
    ]
    tmp = run_mp(world, cases)
    for i, c in enumerate(cases):
        want = expected_for(c, world)
        for r in range(world):
            got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
            exp = np.frombuffer(want[r].tobytes(), dtype=np.uint8)
            assert got.tobytes() == exp.tobytes(), (i, c, r)


@pytest.mark.parametrize("world", [3, 5, 8])
def test_mp_tree_path_ring_mincount(world):
    """rdc_reduce_ring_mincount=64K (communicator_manager.cc:140-162 key):
    buffers of <= 64 KiB take the reference's tree order, larger ones the
    ring's — device, host (RdcAllreduce) and coalesced lists mixing both,
    against the oracle (tree: oracle/tree_order.cc).  Integer cases are
    test/allreduce.cc-style known answers (order-free); every rank holds the
    root's bits (the reference's broadcast forwards stale data at n >= 4,
    SURVEY finding 6 — not reproduced)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    M = 64 << 10
    cases = [
        {"count": 1001, "dtype": 6, "op": 2, "mincount": M},
        {"count": 16384, "dtype": 6, "op": 2, "mincount": M, "pad_per_rank": 4},      # exactly 64 KiB: tree
        {"count": 16385, "dtype": 6, "op": 2, "mincount": M},                         # one more: ring
        {"count": 4099, "dtype": 2, "op": 2, "mincount": M},
        {"count": 3001, "dtype": 10, "op": 0, "mincount": M, "reps": 3},
        {"count": 777, "dtype": 7, "op": 1, "mincount": M, "algo": 2},                # algo does not change the order
        {"count": 1, "dtype": 0, "op": 2, "mincount": M},
        {"count": 4096, "dtype": 6, "op": 2, "kind": "host_allreduce", "mincount": M},
        {"count": 0, "dtype": 6, "op": 2, "kind": "coalesced", "counts": [1001, 70000, 5, 16384, 0, 20000],
         "mincount": M, "reps": 2},
        {"count": 0, "dtype": 2, "op": 0, "kind": "coalesced", "counts": [3, 1000, 77], "host": True,
         "mincount": M},
        {"count": 30011, "dtype": 6, "op": 2, "kind": "algo_chain", "algos": [0, 4, 3, 2, 1, 4, 4, 0],
         "mincount": M},
    ]
    tmp = run_mp(world, cases, env_extra={"rdc_reduce_ring_mincount": "64K"})
    for i, c in enumerate(cases):
        if c.get("kind") == "algo_chain":
            bufs = [O.fill(c["count"], 6, 0x5EED0000, r) for r in range(world)]
            for a in c["algos"]:
                (O.allreduce_tree if a == 4 else O.allreduce_ring)(bufs, 6, 2)
            want = bufs
        else:
            want = expected_for(c, world)
        for r in range(world):
            got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
            assert got.tobytes() == np.frombuffer(want[r].tobytes(), dtype=np.uint8).tobytes(), (world, i, c, r)


HOST_MIX = [(1024, 6, 2, 0), (1024, 6, 2, 0), (1, 6, 2, 0), (16384, 6, 2, 0), (3, 2, 0, 0), (4099, 10, 2, 0),
            (777, 7, 1, 5), (1024, 6, 2, 0), (8, 0, 3, 3), (5000, 11, 2, 0), (1024, 6, 2, 4), (12345, 1, 2, 0)]


def expected_host_mix(world, mincount=1):
    out = []
    for j, (cnt, dt, op, _) in enumerate(HOST_MIX):
        xs = [O.fill(cnt, dt, 0x5EED6000 + j, r) for r in range(world)]
        esz = np.dtype(O.NP_DTYPE[dt]).itemsize
        (O.allreduce_tree if cnt * esz <= mincount else O.allreduce_ring)(xs, dt, op)
        out.append([x.view(np.uint8) for x in xs])
        if j % 3 == 2:
            d = [O.fill(20011, 6, 0x5EED6500 + j, r) for r in range(world)]
            O.allreduce_ring(d, 6, 2)
            out.append([x.view(np.uint8) for x in d])
    return [np.concatenate([o[r] for o in out]) for r in range(world)]


@pytest.mark.parametrize("world,env", [(2, {}), (3, {"rdc_reduce_ring_mincount": "8K"}), (2, {"RDC_HOST_SERVICE": "0"}),
                                       (4, {"RDC_HOST_SERVICE_IDLE_US": "50"}),
                                       (2, {"RDC_HOST_SERVICE_LL_BYTES": "0"}),
                                       (3, {"RDC_HOST_SERVICE_EAGER_BYTES": "0", "rdc_reduce_ring_mincount": "8K"}),
                                       (8, {"RDC_HOST_SERVICE_SHARE_MAX": "8"}),
                                       (5, {"RDC_HOST_SERVICE_SHARE_MAX": "8"}),
                                       (7, {"RDC_HOST_SERVICE_SHARE_MAX": "8",
                                            "rdc_reduce_ring_mincount": "2K"}),
                                       (2, {"RDC_HOST_SERVICE_HX_BYTES": "32768"}),
                                       (3, {"RDC_HOST_SERVICE_HX_BYTES": "1048576", "RDC_HOST_SERVICE_HX_EAGER_BYTES": "0",
                                            "rdc_reduce_ring_mincount": "8K"}),
                                       (4, {"RDC_HOST_SERVICE_HX_BYTES": "1048576",
                                            "RDC_HOST_SERVICE_HX_EAGER_BYTES": "65536"}),
                                       (3, {"RDC_HOST_SERVICE_PIPELINE": "1"})])
def test_mp_host_small_service(world, env):
    """Small synchronous HOST allreduces (cfg1's path) through the resident
    service block (rdc_service.h): 12 calls of 1 B - 64 KiB over 8 (dtype, op)
    pairs (each switch restarts the kernel), sleeps of 3-5 ms longer than its
    idle time (it exits and is relaunched), device collectives in between,
    the tree order below rdc_reduce_ring_mincount; LL and plain input modes
    (RDC_HOST_SERVICE_LL_BYTES=0), no eager polling, 8 ranks (the 8-wide
    kernel; RDC_HOST_SERVICE_SHARE_MAX lifts the one-GPU cap); the host
    exchange (RDC_HOST_SERVICE_HX_BYTES: every rank's input from one shared
    host region) at a 32 KiB budget and up to the 16 KiB LL limit, with no and
    with whole-block eager polling; two poll rounds in flight
    (RDC_HOST_SERVICE_PIPELINE=1); and the launch path with RDC_HOST_SERVICE=0.
    Every result bit-exact against the oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cases = [{"count": 0, "dtype": 6, "op": 2, "kind": "host_mix", "ops": HOST_MIX}]
    tmp = run_mp(world, cases, env_extra=env)
    mc = env.get("rdc_reduce_ring_mincount", "1")
    mincount = int(mc[:-1]) << 10 if mc.endswith("K") else int(mc)
    want = expected_host_mix(world, mincount)
    for r in range(world):
        got = np.load(os.path.join(tmp, "case0_rank%d.npy" % r))
        assert got.shape == want[r].shape, (r, got.shape, want[r].shape)
        bad = np.nonzero(got != want[r])[0]
        assert bad.size == 0, "rank %d: %d bytes differ, first at %d" % (r, bad.size, bad[0])


def test_mp_named_communicators_share_scratch():
    """Every named communicator over the same ranks shares ONE scratch channel
    (4080 MiB by default, not 4080 MiB per communicator): two more
    communicators cost only their point-to-point regions, and allreduces on
    three communicators issued back to back on three different streams, every
    schedule, no host syncs, all come out bit-exact (the channel orders them)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cases = [{"count": 300007, "dtype": 6, "op": 2, "kind": "shared_comms", "reps": 4}]
    tmp = run_mp(3, cases, env_extra={"RDC_SCRATCH_BYTES": "4080M"})
    for r in range(3):
        info = json.load(open(os.path.join(tmp, "case0_rank%d.json" % r)))
        assert info["shares"] == [1, 1, 1], info
        assert info["bytes_used_by_two_comms"] < (512 << 20), info  # two p2p regions, no 2 x 4 GiB scratch
        got = np.load(os.path.join(tmp, "case0_rank%d.npy" % r))
        want = []
        for j in range(3):
            xs = [O.fill(300007, 6, 0x5EED4000 + j, q) for q in range(3)]
            for _ in range(4):
                O.allreduce_ring(xs, 6, 2)
            want.append(xs[r])
        assert got.tobytes() == np.concatenate(want).view(np.uint8).tobytes(), r


@pytest.mark.parametrize("world,algo", [(2, 1), (3, 0), (3, 2)])
def test_mp_shared_channel_order_violation_is_an_error(world, algo):
    """Two named communicators share one channel; rank 0 issues main then x,
    the other ranks x then main.  Launches with the same sequence number
    belong to different communicators: every rank must get an error naming
    the order violation (tagged hand-off flags, RDC_KERR_ORDER), never wrong
    bits.  Ring (n = 2), one-shot (auto at n = 3) and mesh."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cases = [{"count": 100003, "dtype": 6, "op": 2, "kind": "order_violation", "algo": algo}]
    tmp = run_mp(world, cases, timeout=120, env_extra={"RDC_TIMEOUT": "30"})
    infos = [json.load(open(os.path.join(tmp, "case0_rank%d.json" % r))) for r in range(world)]
    for info in infos:
        assert info["shares"] == [1, 1], infos
        assert "another communicator" in info["error"] and "different orders" in info["error"], infos


@pytest.mark.parametrize("world,kind", [(2, "allreduce"), (3, "allreduce"), (2, "host_allreduce")])
def test_mp_count_beyond_int32(world, kind):
    """A buffer of more than 2^31 elements (int8, 2 GiB + 4099): the
    reference's int Split (include/utils/utils.h:59-70) overflows there; the
    device path's 64-bit ranges and offsets must not.  Device buffers through
    the schedule pieces, and a host buffer through the PCIe pipeline.  Windows
    at every Split boundary, across the 2^31 element index and at both ends
    are compared with the oracle (int8 Sum wraps, order-free), and every
    rank's whole result must hash the same."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    count = (1 << 31) + 4099
    W = 4096
    starts = {0, count - W, (1 << 31) - W // 2, (1 << 31) + 4099 - W}
    for b, _ in O.split(count, world)[1:]:
        starts.add(b - W // 2)
    wins = sorted((st, W) for st in starts)
    seed = 0x5EED9000
    cases = [{"count": count, "dtype": 0, "op": 2, "kind": kind, "seed": seed, "windows": wins}]
    tmp = run_mp(world, cases, timeout=600)
    shas = [open(os.path.join(tmp, "case0_rank%d.sha" % r)).read() for r in range(world)]
    assert all(h == shas[0] for h in shas), shas
    want = np.concatenate([O.expected_window(count, st, m, world, 0, 2, seed) for st, m in wins])
    for r in range(world):
        got = np.load(os.path.join(tmp, "case0_rank%d.npy" % r))
        assert got.tobytes() == want.tobytes(), r


HOST_SWEEP_BYTES = [
    65535, 65537,                      # the resident service's 64 KiB limit
    524287, 524289, 786435,            # the copy pool's 512 KiB threshold, 2-3 parts with a remainder
    1048575, 1048577, 1048579,         # zero-copy / staged small path (1 MiB) vs one inline piece
    (3 << 20) + 7, 16777215, 16777217,  # one inline piece up to 16 MiB, the pipeline above
    (33 << 20) + 4097,                 # pipeline without the ramp (< 8 pieces of 16 MiB)
    (64 << 20) + 4095,                 # 4 pieces, ragged last piece
    (128 << 20) + 4095,                # pipeline with the ramp (>= 8 pieces), ragged last piece
]


@pytest.mark.parametrize("world,balance", [(2, "0"), (3, "0"), (3, "1"), (4, "1"), (5, "0"), (5, "1"), (5, "diag"),
                                           (5, "one_block_per_cu")])
def test_mp_host_size_sweep(world, balance):
    """Host buffers at every boundary of the host path (rdc_host.cpp: service,
    copy-pool parts, zero-copy / staged small path, inline piece, pipeline
    with and without the ramp) +-1 element, 1-byte and 4-byte elements, every
    byte of every rank's result against the oracle.  A copy cut whose parts
    did not cover the buffer (bytes % parts left over) once dropped the last
    bytes of a piece: only sizes like these see it.  RDC_HOST_BALANCE=1: the
    pieces' balanced ranges (every rank folds a part of each piece in its
    chunk's ring order; the default with one rank per GPU).  "diag": 5
    processes on one GPU at the launcher's queue budget (round 4's lost
    one-shot hand-off ran here) with poison mode and the device-side launch
    number check on (RDC_POISON_SCRATCH=1, RDC_SEQ_CHECK=1).
    "one_block_per_cu": the same with every collective held to one block per
    CU (RDC_DEBUG_LDS_PAD=96K) — at round 4's budget of 3 queues per process
    this lost a hand-off in every run; the launcher's budget is now a power of
    two (2 queues for 5 ranks)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = {"RDC_HOST_BALANCE": balance}
    if balance == "diag":
        env = {"RDC_HOST_BALANCE": "0", "RDC_POISON_SCRATCH": "1", "RDC_SEQ_CHECK": "1"}
    elif balance == "one_block_per_cu":
        env = {"RDC_HOST_BALANCE": "0", "RDC_POISON_SCRATCH": "1", "RDC_SEQ_CHECK": "1",
               "RDC_DEBUG_LDS_PAD": str(96 << 10)}
    cases = []
    for k, nb in enumerate(HOST_SWEEP_BYTES):
        cases.append({"count": nb, "dtype": 1, "op": (0, 2)[k % 2], "kind": "host_allreduce", "seed": 0x5EEDA000 + k})
        cases.append({"count": nb // 4 + 1, "dtype": 6, "op": 2, "kind": "host_allreduce", "seed": 0x5EEDB000 + k})
    tmp = run_mp(world, cases, timeout=400, env_extra=env)
    for i, c in enumerate(cases):
        want = expected_for(c, world)
        for r in range(world):
            got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
            w = np.frombuffer(want[r].tobytes(), dtype=np.uint8)
            assert got.shape == w.shape, (c, r)
            bad = np.nonzero(got != w)[0]
            assert bad.size == 0, "%r rank %d: %d bytes differ, first at byte %d" % (c, r, bad.size, bad[0])


REGISTERED_BYTES = [(1 << 20) + 4, (3 << 20) + 7, 16777217, (33 << 20) + 4097, (128 << 20) + 4095]


@pytest.mark.parametrize("world,pinned,balance,mode", [(2, True, "0", "dma"), (3, True, "0", "dma"),
                                                       (3, "even", "0", "dma"), (4, True, "1", "dma"),
                                                       (2, True, "0", "zc"), (3, "even", "1", "zc"),
                                                       (2, True, "0", "kcopy"), (3, "even", "1", "kcopy")])
# dma: RDC_HOST_REG_KCOPY=0 (the DMA engines); kcopy: the default kernel copies
def test_mp_host_registered(world, pinned, balance, mode):
    """Host buffers inside a registered RdcNewBuffer(pinned=1) range
    (rdc/buffer.py:34-38) DMA in place (HostPath::AllreduceRegistered): the
    inline piece, the pipeline with and without the ramp, ragged last pieces,
    a buffer starting 4 B into its registered range, and registered ranks
    beside staged ones in one collective ("even").  Every byte against the
    oracle; the registered ranks report that they took the in-place path."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cases = []
    for k, nb in enumerate(REGISTERED_BYTES):
        cases.append({"count": nb, "dtype": 1, "op": (0, 2)[k % 2], "kind": "host_allreduce", "pinned": pinned,
                      "seed": 0x5EEDC000 + k})
        cases.append({"count": nb // 4 + 1, "dtype": 6, "op": 2, "kind": "host_allreduce", "pinned": pinned,
                      "host_offset": 4 * (k % 2), "seed": 0x5EEDD000 + k})
    # zc: RDC_HOST_REG_ZC=1, the registered ranks' pieces reduced in place over PCIe; kcopy:
    # RDC_HOST_REG_KCOPY=1, their H2D / D2H copies done by kernels ("even": beside staged ranks in one
    # call, pieces and collectives identical)
    tmp = run_mp(world, cases, timeout=400, env_extra={"RDC_HOST_BALANCE": balance,
                                                       "RDC_HOST_REG_ZC": "1" if mode == "zc" else "0",
                                                       "RDC_HOST_REG_KCOPY": "0" if mode == "dma" else "1"})
    for i, c in enumerate(cases):
        want = expected_for(c, world)
        for r in range(world):
            got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
            w = np.frombuffer(want[r].tobytes(), dtype=np.uint8)
            assert got.shape == w.shape, (c, r)
            bad = np.nonzero(got != w)[0]
            assert bad.size == 0, "%r rank %d: %d bytes differ, first at byte %d" % (c, r, bad.size, bad[0])
            reg = os.path.join(tmp, "case%d_rank%d.reg" % (i, r))
            if pinned is True or r % 2 == 0:
                assert open(reg).read() == "1", (c, r)
            else:
                assert not os.path.exists(reg)


def fuzz_cases(seed, world, n=40):
    """Seeded random sizes (log-uniform, 1 element .. 24 Mi elements), (dtype,
    op) pairs with reference semantics, schedules, per-rank misalignment,
    host buffers (service, zero-copy, inline piece, pipeline; pageable or
    in registered ranges on all or some ranks), broadcasts
    from random roots and coalesced lists of random buckets."""
    import random
    rng = random.Random(seed)
    pairs = [(6, 2), (6, 0), (7, 2), (7, 1), (2, 2), (2, 3), (3, 0), (0, 2), (1, 3), (4, 2), (5, 1), (10, 2),
             (11, 2), (10, 0)]
    esz = {0: 1, 1: 1, 2: 4, 3: 4, 4: 8, 5: 8, 6: 4, 7: 8, 10: 2, 11: 2}
    cases = []
    for k in range(n):
        sd = seed * 1000 + k
        kind = rng.choice(["allreduce"] * 5 + ["broadcast", "coalesced", "host_allreduce"])
        if kind == "host_allreduce":
            dt, op = rng.choice(pairs)
            cases.append({"count": max(1, int(2 ** rng.uniform(0, 24))), "dtype": dt, "op": op,
                          "kind": "host_allreduce", "seed": 0x5EED0000 + sd,
                          "host_offset": esz[dt] * rng.choice([0, 0, 1, 3]),
                          # registered ranges (all / even ranks), drawn from a
                          # separate stream so the other cases stay as they were
                          "pinned": random.Random(sd).choice([None, None, True, "even"])})
        elif kind == "allreduce":
            dt, op = rng.choice(pairs)
            count = max(1, int(2 ** rng.uniform(0, 24.6)))
            c = {"count": count, "dtype": dt, "op": op, "algo": rng.choice([0, 1, 2, 3, 5]), "seed": 0x5EED0000 + sd}
            if rng.random() < 0.5:  # the ranks' buffers differ mod 16 (element-aligned)
                c["pad_per_rank"] = esz[dt] * rng.choice([1, 2, 3])
            if random.Random(sd ^ 0xD1EC7).random() < 0.3:  # the direct schedule (separate stream: the
                c["algo"] = 6                                # other draws stay as they were)
            cases.append(c)
        elif kind == "broadcast":
            cases.append({"count": max(1, int(2 ** rng.uniform(0, 24))), "dtype": 0, "kind": "broadcast",
                          "root": rng.randrange(world), "seed": 0x5EED0000 + sd, "pad": rng.choice([0, 1, 5])})
        else:
            dt, op = rng.choice([(6, 2), (2, 0), (10, 2), (7, 1)])
            counts = [max(0, int(2 ** rng.uniform(-1, 19))) for _ in range(rng.randint(1, 12))]
            c = {"count": 0, "dtype": dt, "op": op, "kind": "coalesced", "counts": counts,
                 "algo": rng.choice([0, 1, 2, 3, 5]), "seed": 0x5EED0000 + sd}
            if random.Random(sd ^ 0xD1EC7).random() < 0.3:  # one direct launch over the list
                c.update({"algo": 6, "same_pads": True})
            cases.append(c)
    return cases


@pytest.mark.parametrize("world,seed,env", [
    (2, 21, {}),
    (3, 22, {"RDC_SCRATCH_BYTES": "8M", "RDC_TILE_BYTES": "16K"}),   # many pieces and tiles per call
    (2, 23, {"RDC_SCRATCH_BYTES": "4M", "RDC_NBLOCKS": "7"}),        # odd grid, tiny scratch
    (4, 24, {"RDC_HOST_BALANCE": "1"}),     # host pieces as balanced ranges (one-rank-per-GPU default)
    (3, 25, {"RDC_ALGO": "ring"}),          # host pipeline pieces and auto calls on the ring
    (5, 26, {"RDC_SCRATCH_BYTES": "16M"}),
])
def test_mp_random_sizes_fuzz(world, seed, env):
    """Seeded fuzz over sizes, types, ops, schedules, misalignment, scratch
    and tile sizes (fuzz_cases): every byte of every rank's result against
    the oracle (the reference's ring order; broadcast = the root's bytes).
    Fixed size lists can miss a boundary a random size lands on."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cases = fuzz_cases(seed, world)
    tmp = run_mp(world, cases, timeout=400, env_extra=env)
    for i, c in enumerate(cases):
        want = expected_for(c, world)
        for r in range(world):
            got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
            w = np.frombuffer(want[r].tobytes(), dtype=np.uint8)
            assert got.shape == w.shape, (i, c, r)
            bad = np.nonzero(got != w)[0]
            assert bad.size == 0, "case %d %r rank %d: %d bytes differ, first at byte %d" % (
                i, c, r, bad.size, bad[0])


@pytest.mark.parametrize("world", [2, 4, 8])
def test_mp_across_devices(world):
    """One rank per GPU when the box has several (rank r on GPU r % #GPUs):
    the hand-offs then cross xGMI instead of landing in one HBM.  Fixed
    cases at every schedule plus a seeded fuzz, every byte against the
    oracle.  Skipped on a 1-GPU box (the driver's 8-GPU bench checks the same
    hand-offs after its timed region)."""
    if not torch.cuda.is_available() or torch.cuda.device_count() < 2:
        pytest.skip("needs 2 or more GPUs")
    cases = [{"count": 1001, "dtype": 6, "op": 2, "algo": a} for a in (0, 1, 2, 3, 5, 6)]
    cases += [{"count": (16 << 20) + 5, "dtype": 6, "op": 2, "algo": a} for a in (1, 2, 5, 6)]
    cases += [{"count": 0, "dtype": 6, "op": 2, "kind": "coalesced", "counts": [1024, 70001, 333] * 3, "algo": 6,
               "same_pads": True}]
    # the direct schedule's result hand-off across GPUs: every line of the buffer in this
    # GPU's L2s (a read kernel before each call) when remote owners overwrite it, read back
    # by a kernel (DESIGN.md §4.2 "what the second row rests on")
    cases += [{"count": c, "dtype": 6, "op": 2, "algo": 6, "reps": 3, "warm_l2": True, "seed": 0x5EEDF000 + c}
              for c in (16384, 262147, 1 << 20)]
    # the untuned default on a buffer above the threshold (the direct schedule where the check passed)
    cases += [{"count": (64 << 20) // 4 + 7, "dtype": 6, "op": 2, "algo": 0}]
    cases += [{"count": 4096, "dtype": 6, "op": 2, "kind": "host_allreduce"},
              {"count": (40 << 20) + 3, "dtype": 1, "op": 0, "kind": "host_allreduce"},
              {"count": (3 << 20) + 5, "dtype": 0, "kind": "broadcast", "root": world - 1}]
    cases += fuzz_cases(30 + world, world, n=24)
    tmp = run_mp(world, cases, timeout=400, env_extra={"RDC_DEVICE": "rank"})
    for i, c in enumerate(cases):
        want = expected_for(c, world)
        for r in range(world):
            got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
            w = np.frombuffer(want[r].tobytes(), dtype=np.uint8)
            assert got.tobytes() == w.tobytes(), (i, c, r)


def test_mp_full_size_cfg2():
    """BASELINE cfg2 at full size: fp32 256 MiB allreduce over 2 ranks, both
    schedules, checked bit-exact (sha256) against the oracle's ring."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import hashlib
    count = (256 << 20) // 4
    cases = [{"count": count, "dtype": 6, "op": 2, "algo": 2, "digest": True},
             {"count": count, "dtype": 6, "op": 2, "algo": 1, "digest": True},
             {"count": count, "dtype": 6, "op": 2, "algo": 6, "digest": True}]
    tmp = run_mp(2, cases, timeout=400, env_extra={"RDC_SCRATCH_BYTES": "4080M", "RDC_NBLOCKS": "64"})
    want = expected_for(cases[0], 2)
    h = hashlib.sha256(np.frombuffer(want[0].tobytes(), dtype=np.uint8).tobytes()).hexdigest()
    for i in range(len(cases)):
        for r in range(2):
            assert open(os.path.join(tmp, "case%d_rank%d.sha" % (i, r))).read() == h, (i, r)


def full_digest(count, dt, world, seed=0x5EED0000):
    import hashlib
    want = expected_for({"count": count, "dtype": dt, "op": 2, "seed": seed}, world)
    h = hashlib.sha256(np.frombuffer(want[0].tobytes(), dtype=np.uint8).tobytes()).hexdigest()
    del want
    return h


def test_mp_full_size_cfg3_cfg4_eight_ranks():
    """BASELINE cfg3 / cfg4 at full size and rank count: 1 GiB fp32 (mesh AND
    the reference's ring schedule, k_ring) and 1 GiB fp16 allreduces over 8
    processes (sharing GPU 0 here; automatic grids, clamped so all 8 grids
    stay resident), each rank's result checked bit-exact (sha256) against the
    oracle's ring — the 8-GPU run's launch plan (NMAX = 8 kernels, one launch
    per call), only the grid is smaller."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cases = [{"count": (1 << 30) // 4, "dtype": 6, "op": 2, "algo": 2, "digest": True},
             {"count": (1 << 30) // 4, "dtype": 6, "op": 2, "algo": 1, "digest": True, "last_launch": True},
             {"count": (1 << 30) // 2, "dtype": 10, "op": 2, "algo": 2, "digest": True},
             {"count": (1 << 30) // 4, "dtype": 6, "op": 2, "algo": 5, "digest": True},
             # the direct schedule (registered user buffers) on both dtypes
             {"count": (1 << 30) // 4, "dtype": 6, "op": 2, "algo": 6, "digest": True},
             {"count": (1 << 30) // 2, "dtype": 10, "op": 2, "algo": 6, "digest": True, "last_launch": True}]
    tmp = run_mp(8, cases, timeout=600, env_extra={"RDC_SCRATCH_BYTES": "4080M"})
    want = {6: full_digest((1 << 30) // 4, 6, 8), 10: full_digest((1 << 30) // 2, 10, 8)}
    for i, c in enumerate(cases):
        for r in range(8):
            assert open(os.path.join(tmp, "case%d_rank%d.sha" % (i, r))).read() == want[c["dtype"]], (i, r)
    # the ring ran as ONE launch per call with one tile per block
    grid = json.load(open(os.path.join(tmp, "case1_rank0.launch")))
    assert grid[5] == 1 and grid[0] >= 1, grid
    assert json.load(open(os.path.join(tmp, "case5_rank0.launch")))[5] == 6  # the direct schedule ran


def test_mp_cfg5_exact_shape_eight_ranks():
    """BASELINE cfg5 at its exact shape: 1024 x 1 MiB fp32 buckets (separate
    allocations, per-bucket misalignment) in ONE RdcCommAllreduceCoalesced
    call over 8 processes — the unit-table mesh with NMAX = 8 — twice with
    the cached unit table; every rank's 1 GiB of results checked (sha256)
    against 1024 oracle rings (test/mallreduce.cc:17-53 shape)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import hashlib
    K, per = 1024, 1 << 18
    cases = [{"count": 0, "dtype": 6, "op": 2, "kind": "coalesced", "counts": [per] * K, "reps": 2,
              "digest": True},
             {"count": 0, "dtype": 6, "op": 2, "kind": "coalesced", "counts": [per] * K, "reps": 2,
              "digest": True, "algo": 5},   # the pull-mode mesh over the same unit table
             # one direct launch over the list (buckets congruent mod 16 across ranks)
             {"count": 0, "dtype": 6, "op": 2, "kind": "coalesced", "counts": [per] * K, "reps": 2,
              "digest": True, "algo": 6, "same_pads": True, "last_launch": True}]
    tmp = run_mp(8, cases, timeout=600, env_extra={"RDC_SCRATCH_BYTES": "4080M"})
    h = hashlib.sha256()
    for b in range(K):
        xs = [O.fill(per, 6, 0x5EED0000 + b, r) for r in range(8)]
        for _ in range(2):
            O.allreduce_ring(xs, 6, 2)
        h.update(xs[0].tobytes())
    for i in range(len(cases)):
        for r in range(8):
            assert open(os.path.join(tmp, "case%d_rank%d.sha" % (i, r))).read() == h.hexdigest(), (i, r)
    assert json.load(open(os.path.join(tmp, "case2_rank0.launch")))[5] == 6  # the direct schedule ran


def test_mp_forced_oversized_grid_four_ranks():
    """RDC_NBLOCKS=4096 (4x what one GPU holds) on 4 processes sharing GPU 0:
    every waiting launch is clamped to the resident share (ResidentGrid, per
    XCD since round 4: a multiple of the 8 XCDs), so the ring (>= 256 tiles
    per chunk), mesh, one-shot, broadcast and allgather all complete bit-exact
    instead of timing out (round 1: k_ring at 768 blocks x 4 ranks on one GPU
    hit the device timeout)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cases = [{"count": 16 << 20, "dtype": 6, "op": 2, "algo": 1, "last_launch": True, "reps": 2},
             {"count": 16 << 20, "dtype": 6, "op": 2, "algo": 2, "last_launch": True},
             {"count": 100003, "dtype": 6, "op": 2, "algo": 3},
             {"count": (5 << 20) + 3, "dtype": 0, "kind": "broadcast", "root": 2},
             {"count": 200001, "dtype": 2, "kind": "allgather"}]
    tmp = run_mp(4, cases, timeout=400, env_extra={"RDC_NBLOCKS": "4096", "RDC_SCRATCH_BYTES": "512M",
                                                   "RDC_TILE_BYTES": "16K"})
    for i, c in enumerate(cases):
        want = expected_for(c, 4)
        for r in range(4):
            got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
            assert got.tobytes() == np.frombuffer(want[r].tobytes(), dtype=np.uint8).tobytes(), (i, r)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for i in (0, 1):
        ll = json.load(open(os.path.join(tmp, "case%d_rank0.launch" % i)))
        assert ll[0] < 4096 and ll[0] <= 8 * cus // 4, ll  # clamped (8 blocks per CU is the hardware ceiling)
    ll = json.load(open(os.path.join(tmp, "case0_rank0.launch")))
    assert (16 << 20) * 4 // 4 // ll[4] >= 256, ll  # ring: >= 256 tiles per chunk
    if cus % 8 == 0:  # 8 XCDs: the clamp gives every XCD the same share of each rank's grid
        assert ll[0] % 8 == 0, ll


def test_mp_full_grid_beside_resident_service():
    """The small-allreduce service keeps one persistent block per rank resident
    (a host allreduce starts it); a collective forced to the largest grid
    (RDC_NBLOCKS=4096 -> clamped to 4 blocks per CU) must still be wholly
    co-resident beside it, so LaunchGrid leaves one CU per rank out of the
    budget.  Host calls, full-grid mesh / ring / broadcast launches and host
    calls again, interleaved, all bit-exact."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cases = [{"count": 1024, "dtype": 6, "op": 2, "kind": "host_allreduce"},
             {"count": 4 << 20, "dtype": 6, "op": 2, "algo": 2, "last_launch": True},
             {"count": 1000, "dtype": 2, "op": 2, "kind": "host_allreduce"},
             {"count": 4 << 20, "dtype": 6, "op": 2, "algo": 1},
             {"count": 999, "dtype": 6, "op": 0, "kind": "host_allreduce"},
             {"count": (3 << 20) + 1, "dtype": 0, "kind": "broadcast", "root": 1},
             {"count": 16, "dtype": 7, "op": 2, "kind": "host_allreduce"}]
    # the service stays resident for 30 s after its last request (default 1 ms)
    tmp = run_mp(2, cases, timeout=300, env_extra={"RDC_NBLOCKS": "4096", "RDC_TIMEOUT": "20",
                                                   "RDC_HOST_SERVICE_IDLE_US": "30000000"})
    for i, c in enumerate(cases):
        want = expected_for(c, 2)
        for r in range(2):
            got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
            assert got.tobytes() == np.frombuffer(want[r].tobytes(), dtype=np.uint8).tobytes(), (i, r)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    ll = json.load(open(os.path.join(tmp, "case1_rank0.launch")))
    assert ll[0] <= 4 * (cus - 2) // 2, ll


@pytest.mark.parametrize("world", [2, 3])
def test_mp_autotune_agrees_and_stays_bit_exact(world):
    """RdcCommAutotune (bench.py runs it before the timed region at N > 1):
    every rank keeps the same winner (times agreed by a MAX allreduce), the
    stages cover the schedules (ring, mesh, pull-mode mesh, one-shot where it fits, direct) and
    then the winner's shape (mesh split / grid / tiles per reduce block, ring
    grid / tiles per block, or direct grid),
    and the allreduces on the chosen shape stay bit-exact."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    big = 8 << 20  # fp32 elements: 32 MiB
    cases = [{"count": 16384, "dtype": 6, "op": 2, "autotune": 65536},
             {"count": big, "dtype": 6, "op": 2, "autotune": big * 4, "reps": 2},
             {"count": 100003, "dtype": 11, "op": 2, "algo": 2},
             # the tuned schedule / shape serve every dtype and op of the size class
             {"count": 2 * big, "dtype": 10, "op": 2},
             {"count": big + 12345, "dtype": 2, "op": 0},
             {"count": big // 2 - 7, "dtype": 7, "op": 1},
             # a coalesced list of the tuned size class takes the schedule and shape that won (unit table)
             {"count": 0, "dtype": 6, "op": 2, "kind": "coalesced", "counts": [1 << 20] * 8}]
    tmp = run_mp(world, cases, timeout=400)
    for i, c in enumerate(cases):
        want = expected_for(c, world)
        for r in range(world):
            got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
            assert got.tobytes() == np.frombuffer(want[r].tobytes(), dtype=np.uint8).tobytes(), (i, r)
    small = [json.load(open(os.path.join(tmp, "case0_rank%d.tune" % r))) for r in range(world)]
    assert all(t == small[0] for t in small), small
    # the direct schedule passed its self-check (direct vs ring, read back by a kernel) before it was timed
    assert small[0]["direct_check"] == 1, small[0]
    # a one-shot size: the rule's schedule (the one-shot) first, then ring, mesh, the
    # pull-mode mesh and the direct schedule; the winner's shape if it has one
    sched = [c["schedule"] for c in small[0]["candidates"][:5]]
    assert sched[0] == "oneshot" and sorted(sched) == ["direct", "mesh", "mesh_pull", "oneshot", "ring"], small[0]
    if small[0]["chosen"]["schedule"] == "oneshot":
        assert len(small[0]["candidates"]) == 5, small[0]
    tunes = [json.load(open(os.path.join(tmp, "case1_rank%d.tune" % r))) for r in range(world)]
    assert all(t == tunes[0] for t in tunes), tunes  # identical bits on every rank
    t = tunes[0]
    cands = t["candidates"]
    assert t["chosen"] is not None and t["chosen"] in cands, t
    # every candidate timed in 3 rounds: median inside its spread
    assert all(c["spread_ms"][0] <= c["ms"] <= c["spread_ms"][1] for c in cands), t
    # stage 0: the rule's schedule first (ring at n = 2, mesh from n = 3), the other two of
    # ring / mesh / pull-mode mesh, the one-shot where it fits, the direct schedule; then
    # (either mesh) 7 splits, 4 grids, 4 tilings, (ring) 2 grids, 5 tilings or (direct)
    # 4 grids, each later stage re-timing its predecessor's winner first
    rule = "ring" if world == 2 else "mesh"
    s0 = 5 if cands[3]["schedule"] == "oneshot" else 4
    assert cands[0]["schedule"] == rule and {c["schedule"] for c in cands[:3]} == {"ring", "mesh", "mesh_pull"}, t
    assert cands[s0 - 1]["schedule"] == "direct", t
    if t["chosen"]["schedule"] != "oneshot":
        chosen = t["chosen"]["schedule"]
        last = 4 if chosen != "ring" else 5
        assert len(cands) == s0 + {"mesh": 15, "mesh_pull": 15, "ring": 7, "direct": 4}[chosen], t
        assert all(c["schedule"] == t["chosen"]["schedule"] for c in cands[s0:]), t
        # the last stage's incumbent stays unless another beats it by more than 3 %
        fin = cands[-last:]
        assert t["chosen"] in fin and t["chosen"]["ms"] <= min(c["ms"] for c in fin) / 0.97 + 1e-9, t


def test_mp_tune_file_persists_autotune():
    """RDC_TUNE_FILE: rank 0 appends the winner of RdcCommAutotune; a later
    job on the same node (new processes, no autotune) loads it at
    communicator creation and launches the same schedule and shape, still
    bit-exact."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    big = 8 << 20
    path = os.path.join(tempfile.mkdtemp(prefix="rdc_tune_"), "tune.txt")
    env = {"RDC_TUNE_FILE": path}
    first = run_mp(2, [{"count": big, "dtype": 6, "op": 2, "autotune": big * 4, "last_launch": True}],
                   timeout=400, env_extra=env)
    lines = open(path).read().splitlines()
    assert len(lines) == 1 and lines[0].startswith("rdc-tune 2 2 "), lines
    second = run_mp(2, [{"count": big, "dtype": 6, "op": 2, "last_launch": True},
                        {"count": big + 3, "dtype": 10, "op": 2, "last_launch": True}], env_extra=env)
    tuned = json.load(open(os.path.join(first, "case0_rank0.tune")))
    for r in range(2):
        a = json.load(open(os.path.join(first, "case0_rank%d.launch" % r)))
        b = json.load(open(os.path.join(second, "case0_rank%d.launch" % r)))
        assert a == b, (a, b, tuned)
        assert {1: "ring", 2: "mesh", 3: "oneshot", 5: "mesh_pull", 6: "direct"}[b[5]] == tuned["chosen"]["schedule"], (b, tuned)
    for tmp, cases in ((first, [{"count": big, "dtype": 6, "op": 2}]),
                       (second, [{"count": big, "dtype": 6, "op": 2}, {"count": big + 3, "dtype": 10, "op": 2}])):
        for i, c in enumerate(cases):
            want = expected_for(c, 2)
            for r in range(2):
                got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
                assert got.tobytes() == np.frombuffer(want[r].tobytes(), dtype=np.uint8).tobytes(), (tmp, i, r)


def test_mp_many_small_buckets_cfg5_shape():
    """test/mallreduce.cc shape: back-to-back 1 MiB fp32 allreduces on one buffer."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cases = [{"count": 1 << 18, "dtype": 6, "op": 2, "reps": 64},
             {"count": 1 << 18, "dtype": 2, "op": 0, "reps": 64, "algo": 1}]
    tmp = run_mp(4, cases)
    for i, c in enumerate(cases):
        want = expected_for(c, 4)
        for r in range(4):
            got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
            assert got.tobytes() == np.frombuffer(want[r].tobytes(), dtype=np.uint8).tobytes(), (i, r)


@pytest.mark.parametrize("world", [8, 12])
def test_mp_many_ranks(world):
    """n = 8 (the node size; k_mesh NMAX = 8) and n = 12 (NMAX = 16) as processes
    sharing GPU 0: every schedule, odd counts, a broadcast and an allgather."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cases = [
        {"count": 1, "dtype": 6, "op": 2},
        {"count": 7, "dtype": 6, "op": 2, "algo": 1},
        {"count": 100003, "dtype": 6, "op": 2, "algo": 2},
        {"count": 100003, "dtype": 6, "op": 2, "algo": 1, "pad_per_rank": 4},
        {"count": 65537, "dtype": 10, "op": 1},
        {"count": 3001, "dtype": 4, "op": 2, "reps": 2},
        {"count": 4099, "dtype": 0, "kind": "broadcast", "root": world // 2},
        {"count": 333, "dtype": 2, "kind": "allgather"},
    ]
    tmp = run_mp(world, cases, timeout=400, env_extra={"RDC_NBLOCKS": "8", "RDC_SCRATCH_BYTES": "16M"})
    for i, c in enumerate(cases):
        want = expected_for(c, world)
        for r in range(world):
            got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
            assert got.tobytes() == np.frombuffer(want[r].tobytes(), dtype=np.uint8).tobytes(), (world, i, c, r)


def test_mp_mixed_schedule_chain():
    """Stream-ordered chains without host syncs mixing every schedule on one
    communicator: exercises the parity halves and the post-one-shot gates
    across processes."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cases = [{"count": 20011, "dtype": 6, "op": 2, "kind": "algo_chain", "algos": [3, 3, 2, 3, 1, 3, 3, 2, 2, 1, 3]},
             # the pull-mode mesh between every other schedule, back to back
             {"count": 300007, "dtype": 6, "op": 2, "kind": "algo_chain", "algos": [5, 5, 3, 5, 1, 5, 2, 5, 3, 3, 5]}]
    tmp = run_mp(3, cases)
    for i, c in enumerate(cases):
        inputs = [O.fill(c["count"], 6, 0x5EED0000, r) for r in range(3)]
        bufs = [x.copy() for x in inputs]
        for _ in c["algos"]:
            O.allreduce_ring(bufs, 6, 2)
        for r in range(3):
            got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
            assert got.tobytes() == np.frombuffer(bufs[r].tobytes(), dtype=np.uint8).tobytes(), (i, r)


# ------------------------------------------------------- coalesced (buckets)
def run_group_coalesced(comms, bufsets, dtype, op, algo, pads):
    """bufsets[r][b]: rank r's input of bucket b.  One fused call per rank."""
    import ctypes
    from rdc_amd._lib import _LIB
    n = len(comms)
    nb = len(bufsets[0])
    esz = np.dtype(O.NP_DTYPE[dtype]).itemsize
    devs = [[to_dev(bufsets[r][b], pads[r][b] * esz) for b in range(nb)] for r in range(n)]
    torch.cuda.synchronize()
    for r in range(n):
        arr = (ctypes.c_void_p * nb)(*[devs[r][b].data_ptr() + pads[r][b] * esz for b in range(nb)])
        cnt = (ctypes.c_size_t * nb)(*[bufsets[r][b].size for b in range(nb)])
        rc = _LIB.RdcCommAllreduceCoalesced(comms[r].handle, arr, cnt, nb, dtype, op, algo,
                                            ctypes.c_void_p(comms.streams[r].cuda_stream))
        assert rc == 0, _LIB.RdcGetLastError()
    for r in range(n):
        comms[r].check(ctypes.c_void_p(comms.streams[r].cuda_stream))
    return [[from_dev(devs[r][b], pads[r][b] * esz, bufsets[r][b].size, dtype) for b in range(nb)]
            for r in range(n)]


BUCKETS = [[1024] * 6, [1, 2, 3, 1001, 0, 7], [4099, 1 << 16, 3], [0, 0, 5], [17, 100003, 1, 2]]


@pytest.mark.parametrize("algo", [0, 1, 2, 3, 5])
@pytest.mark.parametrize("dtype,op", [(6, 2), (10, 2), (11, 2), (7, 1), (2, 0), (0, 3), (4, 2)])
def test_group3_coalesced(group3, dtype, op, algo):
    """Coalesced allreduce == one reference allreduce per bucket, bit for bit:
    ragged bucket sizes (incl. empty buckets and buckets shorter than n),
    every bucket its own allocation at a per-rank, per-bucket misalignment."""
    rng = np.random.default_rng(1000 + dtype * 8 + op)
    for counts in BUCKETS:
        sets = [[rand_input(rng, k, dtype) for k in counts] for _ in range(3)]
        pads = [[(r + 2 * b) % 4 for b in range(len(counts))] for r in range(3)]
        got = run_group_coalesced(group3, sets, dtype, op, algo, pads)
        for b, k in enumerate(counts):
            want = O.expected_allreduce([sets[r][b] for r in range(3)], dtype, op)
            for r in range(3):
                assert same_bits(got[r][b], want, dtype), (counts, algo, b, r)


@pytest.mark.parametrize("algo", [2, 1, 5])
@pytest.mark.parametrize("fused,tile", [("1", "16K"), ("1", "0"), ("0", "16K")])
def test_group_coalesced_mesh_unit_table(fused, tile, algo):
    """The mesh (algo 2) and the ring (algo 1) on a coalesced list move bytes
    straight between the user buffers and the peers' scratch through the unit
    table (no staging image); small tiles make tiles start and end inside
    units and span several.  RDC_COALESCE_FUSED=0 keeps the pack / schedule /
    unpack path.  Bit-exact."""
    from rdc_amd._lib import _LIB
    assert _LIB.RdcSetParam(b"RDC_COALESCE_FUSED", fused.encode()) == 0
    assert _LIB.RdcSetParam(b"RDC_TILE_BYTES", tile.encode()) == 0
    try:
        g = make_group(2, 32 << 20)
    finally:
        assert _LIB.RdcSetParam(b"RDC_COALESCE_FUSED", b"1") == 0
        assert _LIB.RdcSetParam(b"RDC_TILE_BYTES", b"0") == 0
    try:
        rng = np.random.default_rng(77)
        for dtype, op, counts in [(6, 2, [300000, 5, 70001, 1 << 20, 33, 0, 4096]),
                                  (10, 2, [65537, 3, 200003]), (2, 0, [1, 99999, 12345, 7]),
                                  (7, 2, [40000, 40001, 2])]:
            sets = [[rand_input(rng, k, dtype) for k in counts] for _ in range(2)]
            pads = [[(r + b) % 3 for b in range(len(counts))] for r in range(2)]
            got = run_group_coalesced(g, sets, dtype, op, algo, pads)
            for b, k in enumerate(counts):
                want = O.expected_allreduce([sets[r][b] for r in range(2)], dtype, op)
                for r in range(2):
                    assert same_bits(got[r][b], want, dtype), (dtype, counts, algo, b, r)
    finally:
        for c in g:
            c.destroy()


def test_group_coalesced_fusion_groups_and_cache(group2):
    """Small fuse groups (RDC_FUSE_BYTES) split the list into several fused
    launch sequences; repeated calls with the same buffers reuse the cached
    unit table and still produce fresh results."""
    import ctypes
    import rdc_amd
    from rdc_amd._lib import _LIB
    rng = np.random.default_rng(11)
    assert _LIB.RdcSetParam(b"RDC_FUSE_BYTES", b"64K") == 0
    try:
        g = make_group(2, 16 << 20)
    finally:
        assert _LIB.RdcSetParam(b"RDC_FUSE_BYTES", b"256M") == 0
    try:
        counts = [5000, 9000, 30000, 1, 16384, 2000]      # 20 KB .. 120 KB fp32 -> several groups
        ts = [[torch.zeros(k, dtype=torch.float32, device="cuda") for k in counts] for _ in range(2)]
        for it in range(3):
            xs = [[rng.standard_normal(k).astype(np.float32) for k in counts] for _ in range(2)]
            for r in range(2):
                for b in range(len(counts)):
                    ts[r][b].copy_(torch.from_numpy(xs[r][b]))
            torch.cuda.synchronize()
            for r in range(2):
                g[r].allreduce_coalesced(ts[r], rdc_amd.Op.SUM, stream=ctypes.c_void_p(g.streams[r].cuda_stream))
            for r in range(2):
                g[r].check(ctypes.c_void_p(g.streams[r].cuda_stream))
            for b in range(len(counts)):
                want = O.expected_allreduce([xs[0][b], xs[1][b]], O.DT_FLOAT32, O.OP_SUM)
                for r in range(2):
                    assert ts[r][b].cpu().numpy().tobytes() == want.tobytes(), (it, b, r)
    finally:
        for c in g:
            c.destroy()


def test_group_coalesced_graph_capture(group2):
    """After a warm-up call (unit table cached), a coalesced allreduce is
    capturable in a hipGraph and replays with fresh inputs."""
    import ctypes
    import rdc_amd
    rng = np.random.default_rng(12)
    counts = [4096, 333, 70001, 8]
    ts = [[torch.zeros(k, dtype=torch.float32, device="cuda") for k in counts] for _ in range(2)]
    sp = [ctypes.c_void_p(group2.streams[r].cuda_stream) for r in range(2)]
    torch.cuda.synchronize()
    for r in range(2):
        group2[r].allreduce_coalesced(ts[r], rdc_amd.Op.SUM, stream=sp[r])
    for r in range(2):
        group2[r].check(sp[r])
    graphs = []
    for r in range(2):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=group2.streams[r], capture_error_mode="thread_local"):
            group2[r].allreduce_coalesced(ts[r], rdc_amd.Op.SUM, stream=sp[r])
        graphs.append(gr)
    torch.cuda.synchronize()
    for it in range(3):
        xs = [[rng.standard_normal(k).astype(np.float32) for k in counts] for _ in range(2)]
        for r in range(2):
            for b in range(len(counts)):
                ts[r][b].copy_(torch.from_numpy(xs[r][b]))
        torch.cuda.synchronize()
        for r in range(2):
            with torch.cuda.stream(group2.streams[r]):
                graphs[r].replay()
        for r in range(2):
            group2[r].check(sp[r])
        for b in range(len(counts)):
            want = O.expected_allreduce([xs[0][b], xs[1][b]], O.DT_FLOAT32, O.OP_SUM)
            for r in range(2):
                assert ts[r][b].cpu().numpy().tobytes() == want.tobytes(), (it, b, r)


def test_mp_coalesced_cfg5_shape():
    """BASELINE cfg5 shape (scaled): 64 x 1 MiB fp32 buckets in one coalesced
    call on 4 processes, twice (cached unit table), vs one oracle ring per bucket."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cases = [{"count": 0, "dtype": 6, "op": 2, "kind": "coalesced", "counts": [1 << 18] * 64, "reps": 2}]
    tmp = run_mp(4, cases, env_extra={"RDC_SCRATCH_BYTES": "256M"})
    want = expected_for(cases[0], 4)
    for r in range(4):
        got = np.load(os.path.join(tmp, "case0_rank%d.npy" % r))
        assert got.tobytes() == np.frombuffer(want[r].tobytes(), dtype=np.uint8).tobytes(), r


@pytest.mark.parametrize("algo", ["mesh", "ring", "oneshot"])
def test_missing_peer_times_out_instead_of_hanging(algo):
    """Rank 1 never joins: rank 0's launch gives up after RDC_TIMEOUT (device
    wall clock), every block drains, and RdcCommCheck reports the failure
    (the reference's TCP ring can hang forever, SURVEY finding 4)."""
    import ctypes
    import time
    import rdc_amd
    from rdc_amd._lib import _LIB, RdcError
    assert _LIB.RdcSetParam(b"RDC_TIMEOUT", b"1") == 0
    try:
        g = make_group(2, 8 << 20)
    finally:
        assert _LIB.RdcSetParam(b"RDC_TIMEOUT", b"30") == 0
    try:
        t = torch.ones(100003, dtype=torch.float32, device="cuda")
        sp = ctypes.c_void_p(g.streams[0].cuda_stream)
        torch.cuda.synchronize()
        t0 = time.time()
        g[0].allreduce(t, rdc_amd.Op.SUM, algo=algo, stream=sp)
        with pytest.raises(RdcError, match="timed out"):
            g[0].check(sp)
        assert time.time() - t0 < 20
    finally:
        for c in g:
            c.destroy()


_PLAN_SNIPPET = r"""
import os, sys
sys.path.insert(0, %r)
import rdc_amd
rank, world, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
rdc_amd.init(["RDC_RANK=%%d" %% rank, "RDC_WORLD_SIZE=%%d" %% world, "RDC_TRACKER_PORT=%%d" %% port,
              "RDC_TRACKER_URI=127.0.0.1"])
try:
    rdc_amd.get_comm("main")
    print("NOERROR", flush=True)
except Exception as e:  # the expected path
    print("ERR:", e, flush=True)
"""


@pytest.mark.parametrize("key,value", [("RDC_TILE_BYTES", "1M"), ("RDC_HOST_SERVICE", "0"),
                                       ("RDC_HOST_SERVICE_SHARE_MAX", "2"), ("RDC_HOST_PIECE_BYTES", "4194304"),
                                       ("RDC_HOST_BALANCE", "1"), ("RDC_HOST_SERVICE_HX_BYTES", "32768")])
def test_mp_plan_disagreement_is_refused(key, value):
    """Ranks whose launch-plan parameters differ (one rank's env) are refused
    at communicator creation with the parameter named, on every rank: a
    mismatch would otherwise read contributions that never landed, or leave a
    rank waiting in the small-allreduce service while its peer launched a
    kernel (rdc_comm.cpp PlanKey)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    port = free_port()
    base = dict(os.environ, RDC_DEVICE="0", RDC_SCRATCH_BYTES="64M")
    procs = []
    for r in range(2):
        env = dict(base)
        if r == 1:
            env[key] = value
        procs.append(subprocess.Popen([sys.executable, "-c", _PLAN_SNIPPET % ROOT, str(r), "2", str(port)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = [p.communicate(timeout=120)[0].decode(errors="replace") for p in procs]
    for r, o in enumerate(outs):
        assert "ERR:" in o and ("disagree on " + key) in o, "rank %d:\n%s" % (r, o[-2000:])


@pytest.mark.parametrize("vmem", [False, True], ids=["ipc", "vmem"])
@pytest.mark.parametrize("world", [2, 3])
def test_mp_direct_after_free(world, vmem):
    """The direct schedule across freed and re-allocated buffers (each case
    allocates after torch.cuda.empty_cache, so HIP hands the same or
    overlapping address ranges to new allocations, of the same or another
    size — round 5's fault pattern: a 64 MiB mapping over two closed 16 MiB
    ones).  A HIP IPC handle names (process, base address), so a peer still
    mapping the freed allocation would get that stale mapping back for the
    new one: the exporter retires the dead allocation in its rendezvous slot
    and every peer closes its mapping (after its previous direct launch
    finished) before opening the new handle; a new mapping that lands partly
    over ranges the process unmapped is closed unused and that call falls
    back (the fault's trigger).  Round 6: every other call
    takes the direct schedule (round 5's rule made these fall back), every
    result bit-exact against the oracle's ring, and mappings are closed as
    allocations die.  vmem: the same with RDC_DIRECT_IMPORT=vmem (peers'
    allocations mapped at addresses each process chooses, rdc_vmem.h), which
    never meets the placement refusal."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cases = []
    for k, (mib, dt) in enumerate(((16, 6), (16, 6), (16, 10), (64, 10), (64, 6), (16, 6), (128, 10), (64, 6),
                                   (16, 6), (16, 6), (256, 6), (16, 10))):
        esz = 4 if dt == 6 else 2
        cases.append({"count": (mib << 20) // esz, "dtype": dt, "op": 2, "algo": 6, "empty_cache": k > 0,
                      "seed": 0x5EEDE000 + k, "last_launch": True, "direct_stats": True})
    tmp = run_mp(world, cases, timeout=300, env_extra={"RDC_DIRECT_IMPORT": "vmem"} if vmem else None)
    for i, c in enumerate(cases):
        want = expected_for(c, world)
        for r in range(world):
            got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
            assert got.tobytes() == np.frombuffer(want[r].tobytes(), dtype=np.uint8).tobytes(), (i, c, r)
    st = [[json.load(open(os.path.join(tmp, "case%d_rank%d.stats" % (i, r)))) for i in range(len(cases))]
          for r in range(world)]
    ll = [[json.load(open(os.path.join(tmp, "case%d_rank%d.launch" % (i, r)))) for i in range(len(cases))]
          for r in range(world)]
    def grew(key, i, r):
        return st[r][i][key] - (st[r][i - 1][key] if i else 0)

    for i in range(len(cases)):
        # the direct schedule on every call, except where some rank could not
        # map a peer's new allocation (in this test: its mapping landed partly
        # over ranges the process had unmapped, refused) — then every rank
        # takes the scratch schedules for that call
        # or HIP refused to export a rank's new allocation (hipIpcGetMemHandle:
        # hipErrorInvalidValue for an 18 MiB allocation at a base exported four
        # times before, also after every peer had closed those:
        # profiles/r06/remap/export_refused/)
        why = [(r, grew("direct_map_failed", i, r), st[r][i]["direct_fail_reason"],
                grew("direct_export_failed", i, r), st[r][i]["direct_export_error"]) for r in range(world)]
        export_failed = any(w[3] > 0 for w in why)
        explained = any(w[1] > 0 for w in why) or export_failed
        fell = [grew("direct_fallback", i, r) for r in range(world)]
        assert len(set(fell)) == 1, (i, "ranks disagree", fell, why)   # all ranks alike
        for r in range(world):
            # every list here can run direct, unless an export failed
            assert grew("direct_unusable", i, r) == 0 or export_failed, (i, r, why, st[r][i])
            assert (ll[r][i][5] == 6) == (fell[r] == 0), (i, r, ll[r][i], fell, why)
            assert ll[r][i][5] == 6 or (explained and ll[r][i][5] in (1, 2, 5)), (i, r, ll[r][i], why, st[r][i])
            # RDC_DIRECT_IMPORT=vmem: peers mapped at addresses this process
            # chose (rdc_vmem.h): no placement to refuse (reason 5) — what can
            # remain is the runtime naming an earlier buffer object for a
            # reused base (export refused, or its import refused: reason 3)
            assert st[r][i]["direct_import"] == (1 if vmem else 0), st[r][i]
            if vmem:
                assert all(w[2] != 5 or w[1] == 0 for w in why), (i, why)
    for r in range(world):
        # dead allocations are retired and their peer mappings closed as the run goes
        assert st[r][-1]["direct_retired"] >= 1 and st[r][-1]["direct_closed"] >= 1, (r, st[r][-1])
        # every new peer mapping was checked by its exporter's canary before any launch used it
        assert st[r][-1]["direct_canary"] >= len(cases) * (world - 1) // 2, (r, st[r][-1])
        assert st[r][-1]["direct_maps"] <= 4 * (world - 1), (r, st[r][-1])
    # HIP IPC: about a third of these calls refused (placement); vmem: at most
    # a few calls that met the runtime's earlier-buffer-object defect
    assert sum(x[5] == 6 for x in ll[0]) >= (len(cases) - 3 if vmem else len(cases) // 2), ll[0]


@pytest.mark.parametrize("world", [2, 3])
def test_mp_direct_is_the_untuned_default(world):
    """Round 6: without RdcCommAutotune, an automatic
    allreduce (algo 0, what rdc::Allreduce / rdc.allreduce issue) of a device
    buffer above the one-shot sizes and the default threshold (16 MiB; 32 MiB
    at n = 2) takes the direct schedule, because the
    channel ran its self-check at creation (direct_check 1); smaller buffers
    keep the one-shot; a coalesced list above the threshold is one direct
    launch; RDC_DIRECT_BYTES=0 restores the scratch schedules.  Every result
    bit-exact against the oracle's ring."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    big = (16 << 20) + 5
    cases = [{"count": big, "dtype": 6, "op": 2, "last_launch": True, "direct_stats": True},
             {"count": big, "dtype": 10, "op": 2, "last_launch": True, "reps": 2},
             {"count": 70001, "dtype": 6, "op": 2, "last_launch": True},
             {"count": 0, "dtype": 6, "op": 2, "kind": "coalesced", "counts": [1 << 18] * 40 + [12345],
              "same_pads": True, "last_launch": True}]
    for env, want_direct in (({}, True), ({"RDC_DIRECT_BYTES": "0"}, False)):
        tmp = run_mp(world, cases, timeout=300, env_extra=env)
        for i, c in enumerate(cases):
            want = expected_for(c, world)
            for r in range(world):
                got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
                assert got.tobytes() == np.frombuffer(want[r].tobytes(), dtype=np.uint8).tobytes(), (env, i, r)
        ll = [json.load(open(os.path.join(tmp, "case%d_rank0.launch" % i))) for i in range(len(cases))]
        st = json.load(open(os.path.join(tmp, "case0_rank0.stats")))
        # round 6: the flag words of a multi-process channel are HSA-uncached (MTYPE UC), not
        # hipDeviceMallocUncached (MTYPE CC on gfx950: profiles/r06/mtype/)
        assert st["flags_kind"] == 3, st
        assert st["direct_import"] == 0, st  # HIP IPC unless RDC_DIRECT_IMPORT=vmem
        if want_direct:
            assert st["direct_check"] == 1, st  # checked at creation, no autotune ran
            assert ll[0][5] == 6 and ll[1][5] == 6 and ll[3][5] == 6, ll
            assert ll[2][5] == 3, ll  # 280 KB: the one-shot
        else:
            assert st["direct_check"] == 0 and st["direct_calls"] == 0, st  # no self-check, no rendezvous
            assert all(x[5] != 6 for x in ll), ll


def test_mp_uncached_flags_fall_back_together():
    """The flag words and service slots of a multi-process channel are
    HSA-uncached (MTYPE UC, attached through HSA IPC).  If any rank cannot
    attach a peer's region, every rank replaces its HSA-uncached regions with
    hipDeviceMallocUncached ones and the regions are exchanged again
    (RDC_TEST_FAIL_HSA_ATTACH=1 makes rank 1's attaches fail): flags kind 0 on
    every rank, every schedule still bit-exact."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cases = [{"count": 100003, "dtype": 6, "op": 2, "algo": a, "direct_stats": True} for a in (1, 2, 3, 5, 6)]
    cases.append({"count": 4096, "dtype": 6, "op": 2, "kind": "host_allreduce"})
    # RDC_DEBUG: the creation's steps on stderr (the tail of a timed-out run
    # names the step; this test timed out once in 11 runs: profiles/r06/final/gpu_suite_fallback_timeout.txt)
    tmp = run_mp(3, cases, timeout=300, env_extra={"RDC_TEST_FAIL_HSA_ATTACH": "1", "RDC_DEBUG": "1"})
    for i, c in enumerate(cases):
        want = expected_for(c, 3)
        for r in range(3):
            got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
            assert got.tobytes() == np.frombuffer(want[r].tobytes(), dtype=np.uint8).tobytes(), (i, r)
            if c.get("direct_stats"):
                assert json.load(open(os.path.join(tmp, "case%d_rank%d.stats" % (i, r))))["flags_kind"] == 0


@pytest.mark.parametrize("world,second_pad", [(2, False), (3, False), (3, True)])
def test_mp_direct_freed_memory_returned(world, second_pad):
    """A 512 MiB buffer through the direct schedule, freed back to HIP: the
    next direct call makes every peer close its mapping, and the device's
    free memory grows by at least this rank's 512 MiB (round 5 never closed a
    peer mapping, so every freed allocation stayed alive in n-1 processes).
    second_pad: that next call cannot run direct (buffers differ mod 16
    between ranks), and the retired allocation is closed in its rendezvous
    all the same."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    count = (512 << 20) // 4
    cases = [{"count": count, "dtype": 6, "op": 2, "kind": "mem_return", "small": (4 << 20) + 3,
              "seed": 0x5EEDA000, "second_pad": second_pad}]
    tmp = run_mp(world, cases, timeout=300)
    second = expected_for({"count": (4 << 20) + 3, "dtype": 6, "op": 2, "seed": 0x5EEDB000}, world)
    for r in range(world):
        got = np.load(os.path.join(tmp, "case0_rank%d.npy" % r))
        info = json.load(open(os.path.join(tmp, "case0_rank%d.json" % r)))
        # the second call maps a fresh 16 MiB buffer: direct, or — where the runtime placed a peer
        # mapping partly over the freed big buffer's range — refused and run on the scratch schedules
        if second_pad:  # the ranks' buffers differ mod 16: the scratch schedules, closes all the same
            assert info["first_algo"] == 6 and info["second_algo"] != 6, info
        else:
            assert info["first_algo"] == 6 and (info["second_algo"] == 6 or info["refused"] > 0), info
        assert info["closed"] >= world - 1, info
        # hipMemGetInfo's free bytes (device-wide): the peers' closes released this rank's 512 MiB
        # (round 6 first run: +988 MiB at n = 2, both ranks' buffers; the sysfs vram counter seen
        # from the box's container did not track this GPU and is only recorded)
        assert info["free_after"] - info["free_before"] >= (512 << 20) - (64 << 20), info
        assert got[4096:].tobytes() == np.frombuffer(second[r].tobytes(), dtype=np.uint8).tobytes(), r
    # the big buffer's head (its first 4 KiB) against the full-size oracle
    want_big = expected_for({"count": count, "dtype": 6, "op": 2, "seed": 0x5EEDA000}, world)
    for r in range(world):
        got = np.load(os.path.join(tmp, "case0_rank%d.npy" % r))
        assert got[:4096].tobytes() == np.frombuffer(want_big[r].tobytes(), dtype=np.uint8).tobytes()[:4096], r


@pytest.mark.parametrize("world", [2, 3, 5])
def test_mp_direct_registered_buffers(world):
    """RDC_ALGO_DIRECT (k_direct): every rank's user buffer is mapped into
    every peer (HIP IPC, once per allocation, agreed by a per-call host
    rendezvous), owner r folds chunk r straight out of the n buffers in chunk
    r's ring order and writes the result back into all of them.  Every
    (dtype, op) family, sizes from one element to 16 Mi + 5, repeated calls on
    one buffer (the mapping cache), chains mixing the direct schedule with the
    scratch schedules on one buffer, and buffers whose addresses differ mod 16
    between ranks (the rendezvous then falls back to the scratch schedules on
    every rank) — every byte against the oracle's ring."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cases = []
    for dt, op in ((6, 2), (0, 2), (10, 2), (7, 0), (1, 3), (11, 2), (4, 1)):
        for count in (1, 1001, 70001):
            cases.append({"count": count, "dtype": dt, "op": op, "algo": 6, "last_launch": True})
    cases.append({"count": (16 << 20) + 5, "dtype": 6, "op": 2, "algo": 6, "reps": 3, "last_launch": True})
    cases.append({"count": (3 << 20) + 1, "dtype": 6, "op": 2, "kind": "algo_chain", "algos": [6, 2, 6, 5, 1, 6, 3, 6]})
    cases.append({"count": 70001, "dtype": 6, "op": 2, "algo": 6, "pad_per_rank": 4, "last_launch": True})
    # results written by other processes' blocks into lines this rank's L2s
    # hold (a read kernel before every call), read back by a copy kernel
    for count in (16384, 262147, 1 << 20):
        cases.append({"count": count, "dtype": 6, "op": 2, "algo": 6, "reps": 3, "warm_l2": True,
                      "seed": 0x5EEDF000 + count, "last_launch": True})
    # coalesced lists as ONE direct launch (buffers in separate allocations
    # and sub-allocated, odd sizes, an empty bucket); a list whose buffers sit
    # at rank-dependent offsets mod 16 falls back to the scratch schedules
    for dt, counts in ((6, [1024, 7, 0, 100003, 1, 65536]), (10, [4099] * 9), (2, [(1 << 18) + 3] * 40)):
        cases.append({"count": 0, "dtype": dt, "op": 2, "kind": "coalesced", "counts": counts, "algo": 6,
                      "same_pads": True, "last_launch": True, "reps": 2})
    cases.append({"count": 0, "dtype": 6, "op": 2, "kind": "coalesced", "counts": [1024, 70001, 333], "algo": 6,
                  "last_launch": True, "coalesced_fallback": True})
    # RdcCommDirectRelease on every rank: later algo-6 calls take the scratch schedules
    cases.append({"count": 70001, "dtype": 6, "op": 2, "algo": 6, "direct_release": True, "reps": 2,
                  "last_launch": True})
    tmp = run_mp(world, cases, timeout=300)
    for i, c in enumerate(cases):
        if c.get("kind") == "algo_chain":  # every schedule gives the ring's bits
            want = [O.fill(c["count"], 6, 0x5EED0000, r) for r in range(world)]
            for _ in c["algos"]:
                O.allreduce_ring(want, 6, 2)
        else:
            want = expected_for(c, world)
        for r in range(world):
            got = np.load(os.path.join(tmp, "case%d_rank%d.npy" % (i, r)))
            assert got.tobytes() == np.frombuffer(want[r].tobytes(), dtype=np.uint8).tobytes(), (i, c, r)
        if c.get("last_launch"):
            ll = json.load(open(os.path.join(tmp, "case%d_rank0.launch" % i)))
            # aligned buffers take the direct schedule (LastLaunch algo 6);
            # buffers 4 B apart per rank fall back (every rank alike); a
            # buffer of at most rdc_reduce_ring_mincount (1 B) takes the tree
            esz = np.dtype(O.NP_DTYPE[c["dtype"]]).itemsize
            if c.get("kind") == "coalesced":
                assert (ll[5] == 6) == (not c.get("coalesced_fallback")), (i, c, ll)
                continue
            assert (ll[5] == 6) == ("pad_per_rank" not in c and "direct_release" not in c and c["count"] * esz > 1), \
                (i, c, ll)
