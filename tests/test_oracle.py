"""CPU: pin the oracle before trusting it.

* golden vectors (tests/golden/ring_allreduce.npz, made by make_golden.py from
  the reference's own op::Reducer + utils::Split build);
* the reference's known-answer tests test/allreduce.cc:17-55 and
  test/mallreduce.cc:17-53 (integer Max/Sum, a[i] = rank + N (+k) + i);
* oracle/_ref (the reference's headers compiled) on random cases, when built;
* the ring schedule (which chunk each rank sends / receives per step) and
  IEEE binary16 / bfloat16 conversions against numpy.
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.conftest import ROOT

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ring_allreduce.npz")


def test_golden_vectors(oracle):
    g = np.load(GOLDEN, allow_pickle=False)
    meta = g["meta"]
    assert len(meta) >= 20
    for k, (n, count, dt, op, _oracle_only) in enumerate(meta):
        xs = list(g["c%d_in" % k])
        want = g["c%d_out" % k]
        bufs = [x.copy() for x in xs]
        O.allreduce_ring(bufs, int(dt), int(op))
        for r in range(n):
            assert bufs[r].tobytes() == want.tobytes(), (k, n, count, dt, op, r)
        assert O.allreduce_closed_form(xs, int(dt), int(op)).tobytes() == want.tobytes(), k


def test_golden_order_sensitive(oracle):
    """The fixtures do pin the accumulation order: a rank-order sum differs."""
    g = np.load(GOLDEN, allow_pickle=False)
    differs = 0
    for k, (n, count, dt, op, _) in enumerate(g["meta"]):
        if dt != O.DT_FLOAT32 or op != O.OP_SUM or n < 5 or count < 1000:
            continue
        xs = g["c%d_in" % k]
        naive = xs[0].copy()
        for x in xs[1:]:
            naive = naive + x
        differs += int((naive != g["c%d_out" % k]).sum())
    assert differs > 100


@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize("N", [1, 3, 1024, 4099])
def test_known_answer_allreduce_cc(oracle, world, N):
    """test/allreduce.cc:17-55: a[i] = rank + N + i; Max then Sum."""
    a = [np.array([r + N + i for i in range(N)], dtype=np.int32) for r in range(world)]
    O.allreduce_ring(a, O.DT_INT32, O.OP_MAX)
    want_max = np.array([max(j + N + i for j in range(world)) for i in range(N)], dtype=np.int32)
    for r in range(world):
        assert np.array_equal(a[r], want_max)
    a = [np.array([r + N + i for i in range(N)], dtype=np.int32) for r in range(world)]
    O.allreduce_ring(a, O.DT_INT32, O.OP_SUM)
    want_sum = np.array([sum(j + N + i for j in range(world)) for i in range(N)], dtype=np.int32)
    for r in range(world):
        assert np.array_equal(a[r], want_sum)


def test_known_answer_mallreduce_cc(oracle):
    """test/mallreduce.cc:17-53: iter rounds of Max+Sum with a[i] = rank + N + k + i."""
    world, N, iters = 8, 777, 5
    for k in range(iters):
        a = [np.array([r + N + k + i for i in range(N)], dtype=np.int32) for r in range(world)]
        O.allreduce_ring(a, O.DT_INT32, O.OP_MAX)
        assert all(np.array_equal(x, np.arange(N, dtype=np.int32) + (world - 1) + N + k) for x in a)
        a = [np.array([r + N + k + i for i in range(N)], dtype=np.int32) for r in range(world)]
        O.allreduce_ring(a, O.DT_INT32, O.OP_SUM)
        want = np.array([sum(j + N + k + i for j in range(world)) for i in range(N)], dtype=np.int32)
        assert all(np.array_equal(x, want) for x in a)


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built (needs /root/reference)")
def test_oracle_matches_reference_build(oracle):
    rng = np.random.default_rng(11)
    for n in (2, 3, 5, 8, 13):
        for count in (0, 1, n - 1, n, 999, 4097):
            for dt, op in ((6, 2), (6, 0), (6, 1), (7, 2), (2, 2), (0, 2), (1, 3), (4, 0), (5, 1), (9, 2)):
                npd = O.NP_DTYPE[dt]
                if dt in (6, 7):
                    xs = [(rng.standard_normal(count) * 10).astype(npd) for _ in range(n)]
                else:
                    info = np.iinfo(npd)
                    xs = [rng.integers(info.min, info.max, count, dtype=npd, endpoint=True) for _ in range(n)]
                a = [x.copy() for x in xs]
                b = [x.copy() for x in xs]
                O.allreduce_ring(a, dt, op)
                O.ref_allreduce_ring(b, dt, op)
                for r in range(n):
                    assert a[r].tobytes() == b[r].tobytes(), (n, count, dt, op, r)


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built (needs /root/reference)")
def test_split_matches_reference(oracle):
    import ctypes
    R = O.ref()
    for count in (0, 1, 7, 1001, 1 << 20, (1 << 31) - 1):
        for n in (1, 2, 3, 5, 8, 16):
            b = (ctypes.c_int * n)()
            e = (ctypes.c_int * n)()
            R.ref_split(0, count, n, b, e)
            assert [(b[i], e[i]) for i in range(n)] == O.split(count, n)


def test_split_rule(oracle):
    for count in (0, 1, 5, 1001, 4099, 10 ** 10):
        for n in (1, 2, 3, 8, 16):
            rs = O.split(count, n)
            assert rs[0][0] == 0 and rs[-1][1] == count
            lens = [e - b for b, e in rs]
            assert max(lens) - min(lens) <= 1 and lens == sorted(lens, reverse=True)
            assert all(rs[i][1] == rs[i + 1][0] for i in range(n - 1))


@pytest.mark.parametrize("n", [2, 3, 4, 5, 8, 16])
def test_ring_schedule(oracle, n):
    """TryReduceScatterRing / TryAllgatherRing index loops (communicator_collective.cc:79-182)."""
    for r in range(n):
        rs_send, rs_recv, ag_send, ag_recv = O.ring_schedule(n, r)
        assert rs_send == [(r + 1 + j) % n for j in range(n - 1)]
        assert rs_recv == [(r + 2 + j) % n for j in range(n - 1)]
        assert ag_send == [(r + j) % n for j in range(n - 1)]
        assert ag_recv == [(r + 1 + j) % n for j in range(n - 1)]
        # rank r ends the reduce-scatter owning chunk r
        assert rs_recv[-1] == r


def test_reducer_semantics(oracle):
    """op::Max/Min keep dst unless (dst < src) / (dst > src): NaN in dst sticks,
    NaN in src is ignored, -0 vs +0 keeps dst (include/core/mpi.h:85-98)."""
    nan = np.float32("nan")
    d = np.array([nan, 1.0, -0.0, 0.0], dtype=np.float32)
    s = np.array([1.0, nan, 0.0, -0.0], dtype=np.float32)
    out = O.reducer(s, d.copy(), O.DT_FLOAT32, O.OP_MAX)
    assert np.isnan(out[0]) and out[1] == 1.0
    assert np.signbit(out[2]) and not np.signbit(out[3])
    with pytest.raises(ValueError):
        O.reducer(s, d.copy(), O.DT_FLOAT32, O.OP_BITOR)
    a = np.array([127, -128], dtype=np.int8)
    assert O.reducer(np.array([1, -1], dtype=np.int8), a, O.DT_INT8, O.OP_SUM).tolist() == [-128, 127]


def test_half_conversions(oracle):
    L = O.lib()
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.standard_normal(20000) * s for s in (1e-7, 1e-5, 1e-2, 1.0, 1e3, 7e4)]).astype(np.float32)
    x = np.concatenate([x, np.array([65504, 65519, 65520, 2.0 ** -24, 2.0 ** -25, 3 * 2.0 ** -26, np.inf, -np.inf],
                                    dtype=np.float32)])
    want = x.astype(np.float16).view(np.uint16)
    got = np.array([L.rdc_oracle_f32_to_f16(float(v)) for v in x], dtype=np.uint16)
    assert np.array_equal(got, want)
    h = np.arange(65536, dtype=np.uint16)
    f = h.view(np.float16).astype(np.float32)
    back = np.array([L.rdc_oracle_f16_to_f32(int(v)) for v in h], dtype=np.float32)
    ok = ~np.isnan(f)
    assert np.array_equal(back[ok].view(np.uint32), f[ok].view(np.uint32))


def test_f16_sum_is_correctly_rounded(oracle):
    """Per-hop f32 add + RNE to binary16 equals numpy's float16 add."""
    rng = np.random.default_rng(2)
    a = (rng.standard_normal(50000) * 100).astype(np.float16)
    b = (rng.standard_normal(50000) * 0.01).astype(np.float16)
    got = O.reducer(b, a.copy(), O.DT_FLOAT16, O.OP_SUM)
    assert np.array_equal(got.view(np.uint16), (a + b).view(np.uint16))


def test_generator(oracle):
    assert O.lib().rdc_oracle_splitmix64(0) == 0xE220A8397B1DCDAF
    a = O.fill(1000, O.DT_FLOAT32, 0x5EED0000, 0)
    b = O.fill(1000, O.DT_FLOAT32, 0x5EED0000, 1)
    assert a.tobytes() != b.tobytes() and np.all(np.abs(a) <= 1.0)
    assert len(np.unique(a)) > 990
    assert O.fill(10, O.DT_FLOAT32, 0x5EED0000, 0).tobytes() == a[:10].tobytes()


# ----------------------------------------------- CPU TCP ring (baseline port)
@pytest.mark.parametrize("n,count,dtype,op", [(2, 1024, 6, 2), (3, 1001, 6, 2), (5, 4099, 10, 2),
                                              (8, 100003, 6, 2), (4, 777, 2, 0), (3, 5, 7, 1), (2, 1, 6, 2)])
def test_tcp_ring_port_matches_oracle(oracle, tmp_path, n, count, dtype, op):
    """oracle/tcp_ring (the reference's CPU ring over loopback TCP, restated as
    n processes) produces exactly the oracle ring's bytes on every rank."""
    import subprocess
    exe = os.path.join(ROOT, "oracle", "tcp_ring")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    out = subprocess.run([exe, "-n", str(n), "-c", str(count), "-t", str(dtype), "-o", str(op), "-i", "2", "-w", "1",
                          "-d", str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    assert rec["n"] == n and rec["iters"] == 2
    bufs = [oracle.fill(count, dtype, 0x5EED0000, r) for r in range(n)]
    oracle.allreduce_ring(bufs, dtype, op)
    for r in range(n):
        got = open(os.path.join(str(tmp_path), "rank%d.bin" % r), "rb").read()
        assert got == bufs[r].tobytes(), (n, count, dtype, op, r)


# ------------------------------------------------ tree (ring_mincount) path
def test_tree_shapes_follow_get_link_map():
    """The tree is GetLinkMap's heap tree relabelled to ring positions
    (src/utils/topo.cc:3-115): parent/children consistent, rooted at 0, every
    rank reached, depth = the heap depth."""
    import math
    from oracle import oracle as O
    for n in range(1, 17):
        kids, parent, depth = O.tree(n)
        assert parent[0] == -1 and depth[0] == 0
        seen = {0}
        for r in range(n):
            for c in kids[r]:
                assert parent[c] == r and depth[c] == depth[r] + 1
                seen.add(c)
        assert seen == set(range(n))
        assert max(depth) == (int(math.log2(n)) if n > 1 else 0)
        prog = O.tree_program(n)
        assert len(prog) == max(0, n - 1)
        assert sorted(s for _, s in prog) == list(range(1, n))  # every rank folded exactly once


def test_tree_program_matches_library_plan():
    """The product's own tree planner (rdc_plan.cpp PlanTreeProgram, exported
    as RdcPlanTree) gives the oracle's fold program for every n = 1..16."""
    import ctypes
    from oracle import oracle as O
    from rdc_amd._lib import _LIB
    for n in range(1, 17):
        d, s = (ctypes.c_int * 16)(), (ctypes.c_int * 16)()
        k = _LIB.RdcPlanTree(n, d, s)
        assert [(d[i], s[i]) for i in range(k)] == O.tree_program(n), n


def test_tree_fold_order_known_cases():
    """Spot values of the fold (restated libstdc++ unordered_set order): the
    n = 8 root folds subtree 1 then subtree 7; rank 7 folds 6 then 5."""
    from oracle import oracle as O
    kids, _, _ = O.tree(8)
    assert kids[0] == [1, 7] and kids[7] == [6, 5] and kids[1] == [2, 4] and kids[2] == [3]
    assert O.tree_program(3) == [(0, 1), (0, 2)]


@pytest.mark.parametrize("n", [2, 3, 4, 5, 8, 13, 16])
def test_tree_allreduce_integer_known_answers(n):
    """test/allreduce.cc's known answers hold on the tree path too (integer
    Max/Sum are order-free): a[i] = rank + N + i."""
    from oracle import oracle as O
    N = 37
    for op, want in ((O.OP_MAX, lambda i: (n - 1) + N + i), (O.OP_SUM, lambda i: sum(r + N + i for r in range(n)))):
        bufs = [np.arange(r + N, r + N + N, dtype=np.int32) for r in range(n)]
        O.allreduce_tree(bufs, O.DT_INT32, op)
        for b in bufs:
            assert b.tolist() == [want(i) for i in range(N)]


def test_tree_order_differs_from_ring_for_floats():
    """fp32 Sum: the tree's association differs from the ring's (so the path
    must be taken by size, like the reference), and from a rank-order sum."""
    from oracle import oracle as O
    rng = np.random.default_rng(8)
    xs = [rng.standard_normal(4001).astype(np.float32) for _ in range(8)]
    t = O.expected_tree(xs, O.DT_FLOAT32, O.OP_SUM)
    r = O.expected_allreduce(xs, O.DT_FLOAT32, O.OP_SUM)
    assert (t != r).sum() > 0
    # manual evaluation of the n = 8 tree: ((x0 + ((x1 + (x2 + x3)) + x4)) + ((x7 + x6) + x5))
    a1 = (xs[1] + (xs[2] + xs[3])) + xs[4]
    a7 = (xs[7] + xs[6]) + xs[5]
    assert t.tobytes() == ((xs[0] + a1) + a7).tobytes()
