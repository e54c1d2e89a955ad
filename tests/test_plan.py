"""CPU: host-side planning of device collectives (rdc_amd/csrc/rdc_plan.cpp via
RdcPlanAllreduce / RdcPlanLayout) — the exact logic the launches use.

Checks that for every (n, count, dtype, scratch) the launches cover each
Split chunk (include/utils/utils.h:59-70) exactly once, in order, that every
piece fits its scratch slot, tiles and flag indices stay in range, and the
scratch placement is rank-independent (off % 16)."""
import ctypes
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.conftest import ROOT

WORDS = 68


def plan(n, count, dtype, scratch, algo=2, tile=0, max_blocks=256):
    from rdc_amd._lib import _LIB
    npieces = ctypes.c_int()
    rc = _LIB.RdcPlanAllreduce(n, count, dtype, scratch, algo, tile, max_blocks, None, 0, ctypes.byref(npieces))
    assert rc == 0, _LIB.RdcGetLastError()
    k = npieces.value
    buf = (ctypes.c_uint64 * (WORDS * max(1, k)))()
    assert _LIB.RdcPlanAllreduce(n, count, dtype, scratch, algo, tile, max_blocks, buf, k, ctypes.byref(npieces)) == 0
    arr = np.frombuffer(buf, dtype=np.uint64).reshape(max(1, k), WORDS)[:k]
    out = []
    for row in arr:
        out.append(dict(tile=int(row[0]), nb=(int(row[1]), int(row[2]), int(row[3])),
                        off=[int(x) for x in row[4:4 + n]], len=[int(x) for x in row[20:20 + n]],
                        mis=[int(x) for x in row[36:36 + n]], tiles=[int(x) for x in row[52:52 + n]]))
    return out


def layout(n, scratch):
    from rdc_amd._lib import _LIB
    out = (ctypes.c_uint64 * 4)()
    assert _LIB.RdcPlanLayout(n, scratch, out) == 0
    return dict(slot=out[0], region=out[1], max_tiles=out[2], flag_bytes=out[3])


CASES = [(n, count, dt, scratch)
         for n in (2, 3, 5, 8, 16)
         for count in (1, 2, 15, 1001, 4099, 1 << 20, (3 << 22) + 7)
         for dt in (O.DT_INT8, O.DT_FLOAT16, O.DT_FLOAT32, O.DT_FLOAT64)
         for scratch in (1 << 20, 24 << 20, 0)]


@pytest.mark.parametrize("n,count,dt,scratch", CASES[::3])
@pytest.mark.parametrize("algo", [1, 2])
def test_plan_covers_chunks(n, count, dt, scratch, algo):
    esz = np.dtype(O.NP_DTYPE[dt]).itemsize
    L = layout(n, scratch)
    pieces = plan(n, count, dt, scratch, algo)
    ranges = O.split(count, n)
    nxt = [b * esz for b, _ in ranges]
    for p in pieces:
        t = p["tile"]
        assert t % 256 == 0 and t >= 16 << 10
        nb_s, nb_r, nb_g = p["nb"]
        if algo == 2:
            assert min(nb_s, nb_r, nb_g) >= 1 and nb_s + nb_r + nb_g <= 256
        else:
            assert nb_s >= 1
        for c in range(n):
            ln = p["len"][c]
            assert p["mis"][c] == (p["off"][c] % 16)
            assert p["mis"][c] + ln <= L["slot"]           # fits its scratch slot
            assert p["tiles"][c] == -(-ln // t)
            assert p["tiles"][c] <= L["max_tiles"]         # flag index in range
            if ln:
                assert p["off"][c] == nxt[c]               # contiguous, in order
                nxt[c] += ln
    for c in range(n):
        assert nxt[c] == ranges[c][1] * esz                # each chunk covered exactly once


def test_layout_regions_below_2gib():
    for n in (1, 2, 8, 16):
        for scratch in (1 << 20, 4080 << 20, 16 << 30):
            L = layout(n, scratch)
            assert L["region"] < (2 << 30)                   # hipIpcOpenMemHandle limit
            assert L["slot"] * n == L["region"]
            assert L["flag_bytes"] >= (2 * n * L["max_tiles"] + n) * 8  # uint64 sequence words


def test_default_scratch_fits_cfg3_in_one_launch():
    """1 GiB fp32 over 8 ranks: one launch per allreduce with the default scratch."""
    assert len(plan(8, (1 << 30) // 4, O.DT_FLOAT32, 0)) == 1
    assert len(plan(2, (256 << 20) // 4, O.DT_FLOAT32, 0)) == 1


def test_empty_and_world1():
    assert plan(4, 0, O.DT_FLOAT32, 0) == []
    assert plan(1, 100, O.DT_FLOAT32, 0) == []


# ------------------------------------------------------------ coalesced ---
def plan_coalesced(n, counts, dtype):
    from rdc_amd._lib import _LIB
    nb = len(counts)
    cnt = (ctypes.c_size_t * max(1, nb))(*counts)
    chunk = (ctypes.c_uint64 * 33)()
    nu = ctypes.c_int()
    assert _LIB.RdcPlanCoalesced(n, cnt, nb, dtype, chunk, None, 0, ctypes.byref(nu)) == 0, _LIB.RdcGetLastError()
    units = (ctypes.c_uint64 * (4 * max(1, nu.value)))()
    assert _LIB.RdcPlanCoalesced(n, cnt, nb, dtype, chunk, units, nu.value, ctypes.byref(nu)) == 0
    u = np.frombuffer(units, dtype=np.uint64).reshape(-1, 4)[: nu.value].astype(np.int64)
    return [int(x) for x in chunk[:n]], [int(x) for x in chunk[16:16 + n]], int(chunk[32]), u


COALESCED = [
    (2, [1024] * 8), (3, [1, 2, 3, 1001, 0, 7]), (5, [4099, 1 << 16, 3]), (8, [(1 << 20) // 4] * 16),
    (8, [0, 0, 5]), (16, [17, 100003, 1]), (4, [(1 << 18) + 5]),
]


@pytest.mark.parametrize("n,counts", COALESCED)
@pytest.mark.parametrize("dt", [O.DT_INT8, O.DT_FLOAT16, O.DT_FLOAT32, O.DT_FLOAT64])
def test_coalesced_plan_packs_chunk_major(n, counts, dt):
    """Every (buffer, Split chunk c) segment lands once, congruent mod 16 with
    its offset in the buffer, inside
    packed chunk c's range; chunk ranges are disjoint, 256-B aligned and in
    order; copy units cover each segment contiguously."""
    esz = np.dtype(O.NP_DTYPE[dt]).itemsize
    off, ln, total, units = plan_coalesced(n, counts, dt)
    prev_end = 0
    for c in range(n):
        if ln[c]:
            assert off[c] % 256 == 0 and off[c] >= prev_end and ln[c] % esz == 0
            prev_end = off[c] + ln[c]
    assert total == prev_end
    covered = {}
    for b, boff, packed, l in units:
        assert 0 < l <= 128 << 10 and packed + l <= total
        covered.setdefault(int(b), []).append((int(boff), int(packed), int(l)))
    for b, cnt in enumerate(counts):
        segs = sorted(covered.get(b, []))
        pos = 0
        for c, (s0, s1) in enumerate(O.split(cnt, n)):
            lo, hi = s0 * esz, s1 * esz
            while pos < len(segs) and segs[pos][0] < hi:
                boff, packed, l = segs[pos]
                assert lo <= boff and boff + l <= hi           # inside buffer b's chunk c
                assert off[c] <= packed and packed + l <= off[c] + ln[c]  # inside packed chunk c
                if boff == lo:
                    assert packed % 16 == boff % 16            # congruent with its bytes in a 16-B aligned buffer
                pos += 1
        assert sum(s[2] for s in segs) == cnt * esz           # every byte exactly once
    # image ranges of distinct units never overlap
    spans = sorted((int(p), int(p + l)) for _, _, p, l in units)
    for (a0, a1), (b0, _) in zip(spans, spans[1:]):
        assert a1 <= b0


def fuse_groups(counts, dt, fuse):
    from rdc_amd._lib import _LIB
    nb = len(counts)
    cnt = (ctypes.c_size_t * max(1, nb))(*counts)
    out = (ctypes.c_int * (nb + 2))()
    k = ctypes.c_int()
    assert _LIB.RdcPlanFuseGroups(cnt, nb, dt, fuse, out, nb + 2, ctypes.byref(k)) == 0
    return list(out[: k.value])


def test_fuse_groups():
    f32 = O.DT_FLOAT32
    assert fuse_groups([], f32, 1 << 20) == [0]
    assert fuse_groups([256] * 8, f32, 4096) == [0, 4, 8]           # 1 KiB each, 4 KiB groups
    assert fuse_groups([256, 10000, 256], f32, 4096) == [0, 1, 2, 3]  # an oversized buffer is alone
    assert fuse_groups([(1 << 20) // 4] * 1024, f32, 0) == list(range(0, 1025, 256))  # cfg5: 4 x 256 MiB


def test_mixed_plan_is_deterministic():
    """The randomized GPU chain (tests/test_gpu_mixed.py) is the same on every
    rank and in the parent: seeded plan, oracle expectation of the right size."""
    from tests.mixed_plan import expected, make_plan, output_bytes
    a, b = make_plan(11, 40, 3), make_plan(11, 40, 3)
    assert a == b and len(a) == 40
    assert {op["kind"] for op in a} >= {"allreduce", "bcast", "allgather", "coalesced"}
    small = make_plan(5, 6, 2)
    assert expected(small, 2).size == output_bytes(small)


@pytest.mark.parametrize("want,per_cu,cus,share,expect", [
    (512, 4, 256, 1, 512),        # one rank per GPU: the mesh's 2 blocks per CU fit
    (768, 4, 256, 1, 768),        # bench tuning sweep, 3 per CU: still resident
    (4096, 4, 256, 1, 1024),      # RDC_NBLOCKS far above what one GPU holds
    (768, 4, 256, 4, 256),        # round 1's timeout: 4 ranks on one GPU, 768 ring blocks each
    (512, 4, 256, 8, 128),        # 8 ranks on one GPU (the rehearsals)
    (256, 8, 256, 12, 170),       # 12 ranks: floor(8 * 256 / 12)
    (4096, 1, 1, 16, 1),          # never below one block
    (0, 4, 256, 1, 1),
])
def test_resident_grid_clamp(want, per_cu, cus, share, expect):
    """Grids of waiting kernels are clamped so every rank's blocks are
    resident at once (rdc_plan.cpp ResidentGrid): RDC_NBLOCKS / RdcCommTune
    input included."""
    from rdc_amd._lib import _LIB
    got = _LIB.RdcPlanResidentGrid(want, per_cu, cus, share)
    assert got == expect
    assert got * share <= max(per_cu * cus, share)  # all ranks' grids fit together


def test_resident_grid_never_oversubscribes():
    from rdc_amd._lib import _LIB
    rng = np.random.default_rng(3)
    for _ in range(2000):
        want, per_cu, cus, share = (int(rng.integers(1, 8192)), int(rng.integers(1, 9)), int(rng.integers(1, 305)),
                                    int(rng.integers(1, 17)))
        g = _LIB.RdcPlanResidentGrid(want, per_cu, cus, share)
        assert 1 <= g <= want
        assert g == want or g * share <= per_cu * cus or g == 1


def test_auto_schedule_oneshot_vs_mesh():
    """rdc_plan.h OneshotAuto: one-shot while bytes <= 8 MiB and its extra
    egress over the mesh, (n-1)(n-2)/n x bytes, is <= 4 MiB; with
    RDC_ONESHOT_BYTES given, while (n-1) x bytes <= it."""
    from rdc_amd._lib import _LIB
    ONESHOT, MESH, RING = 3, 2, 1
    M = 1 << 20
    scratch = 4080 * M

    def pick(n, b, ob=0):
        return _LIB.RdcPlanAutoAlgo(n, b, scratch, ob)
    # n = 2: the one-shot moves no more bytes than the mesh -> up to 8 MiB
    assert pick(2, 4) == ONESHOT and pick(2, 8 * M) == ONESHOT and pick(2, 8 * M + 4) == RING
    # n = 3: extra = S * 2/3 <= 4 MiB -> S <= 6 MiB
    assert pick(3, 6 * M) == ONESHOT and pick(3, 6 * M + 3 * 4096) == MESH
    # n = 8: extra = S * 42/8 <= 4 MiB -> S <= 798,915 bytes
    assert pick(8, 798912) == ONESHOT and pick(8, 800 * 1024) == MESH
    # explicit RDC_ONESHOT_BYTES keeps the push-budget rule
    assert pick(8, 149792, M) == ONESHOT and pick(8, 150000, M) == MESH
    assert pick(2, 2 * M, M) == RING
    # never beyond half a slot, never for one rank; n = 2 beyond it: the ring
    assert pick(2, 1 << 40) == RING and pick(4, 1 << 40) == MESH and pick(1, 4096) == MESH


def test_direct_default_rule():
    """rdc_plan.h DirectAuto (round 6): an untuned automatic allreduce on a
    multi-process channel takes the direct schedule where the automatic rule
    would pick a two-hand-off schedule (ring at n = 2, mesh from n = 3: above
    the one-shot sizes) and from 16 MiB (32 MiB at n = 2); RDC_DIRECT_BYTES = 0 turns it off, a
    number sets the threshold.  This is the rule the drop-in rdc::Allreduce /
    rdc.allreduce calls get without RdcCommAutotune."""
    from rdc_amd._lib import _LIB
    M = 1 << 20
    scratch = 4080 * M
    AUTO = (1 << 64) - 1

    def direct(n, b, dmin=AUTO, ob=0):
        return _LIB.RdcPlanDirectAuto(n, b, scratch, ob, dmin)
    # n = 2: the ring from 8 MiB, the direct schedule from 32 MiB (profiles/r06/direct_default/)
    assert direct(2, 8 * M + 4) == 0 and direct(2, 32 * M - 4) == 0 and direct(2, 32 * M) == 1
    assert direct(2, 1 << 30) == 1
    # n = 8: the one-shot up to 798,912 bytes, the mesh, then the direct schedule from 16 MiB
    assert direct(8, 798912) == 0 and direct(8, M) == 0 and direct(8, 16 * M - 4) == 0 and direct(8, 16 * M) == 1
    assert direct(8, 256 * M) == 1 and direct(8, 1 << 30) == 1
    # every size where the rule picks ring / mesh and >= the threshold, and nowhere else
    for n in (2, 3, 4, 5, 8, 16):
        for b in (4, 4096, M - 4, M, 3 * M, 6 * M, 8 * M, 9 * M, 16 * M, 20 * M, 32 * M, 64 * M, 1 << 30):
            a = _LIB.RdcPlanAutoAlgo(n, b, scratch, 0)
            assert direct(n, b) == (1 if a in (1, 2) and b >= (32 * M if n == 2 else 16 * M) else 0), (n, b, a)
    # RDC_DIRECT_BYTES=0: never (only algo 6 / RDC_ALGO=direct / an autotuned entry); N: from N bytes
    assert direct(8, 1 << 30, 0) == 0 and direct(2, 1 << 30, 0) == 0
    assert direct(2, 4096, 4096) == 1 and direct(2, 4095, 4096) == 0
    # one rank: never
    assert direct(1, 1 << 30) == 0


PIECES = r'''
import ctypes, json, sys
sys.path.insert(0, sys.argv[1])
from rdc_amd._lib import _LIB
out = {}
for S in [int(x) for x in sys.argv[2:]]:
    b = (ctypes.c_uint64 * 4096)()
    n = ctypes.c_int()
    assert _LIB.RdcPlanHostPieces(S, b, 4096, ctypes.byref(n)) == 0
    out[S] = list(b[:n.value])
print(json.dumps(out))
'''


def host_pieces(sizes, env):
    import json
    import subprocess
    import sys
    e = dict(os.environ, **env)
    p = subprocess.run([sys.executable, "-c", PIECES, ROOT] + [str(s) for s in sizes], env=e, capture_output=True,
                       text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    return {int(k): v for k, v in json.loads(p.stdout).items()}


@pytest.mark.parametrize("piece,ramp", [("16M", "1"), ("8M", "1"), ("8M", "0"), ("4M", "1"), ("1M", "1")])
def test_host_pipeline_pieces(piece, ramp):
    """The host pipeline's contiguous pieces (rdc_host.cpp HostPieceBounds):
    they tile [0, S) in order, interior bounds on 4 KiB (hence element)
    boundaries, one piece up to 16 MiB, pieces of about RDC_HOST_PIECE_BYTES
    P, and with the ramp the first and last three P/8, P/4, P/2 (mirrored)
    for buffers of at least 8 P."""
    P = {"16M": 16 << 20, "8M": 8 << 20, "4M": 4 << 20, "1M": 1 << 20}[piece]
    sizes = [16 << 20, (16 << 20) + 4, 64 << 20, (64 << 20) + 12, 100000012, 256 << 20, 3 * P + 4096 * 7 + 8]
    got = host_pieces(sizes, {"RDC_HOST_PIECE_BYTES": str(P), "RDC_HOST_PIECE_RAMP": ramp})
    for S in sizes:
        b = got[S]
        assert b[0] == 0 and b[-1] == S, (S, b[:4], b[-4:])
        lens = [y - x for x, y in zip(b, b[1:])]
        assert all(l > 0 for l in lens), (S, lens)
        assert all(x % 4096 == 0 for x in b[1:-1]), S
        if S <= 16 << 20:
            assert lens == [S]
            continue
        ramped = ramp == "1" and S >= 8 * P
        if ramped:
            assert lens[:3] == [P // 8, P // 4, P // 2] and lens[-3:-1] == [P // 2, P // 4], (S, lens)
            assert P // 8 <= lens[-1] < P // 8 + 4096, (S, lens)
            mid = lens[3:-3]
        else:
            mid = lens
        assert max(mid) <= P + 4096 and len(mid) == -(-(S - (sum(lens) - sum(mid))) // P), (S, P, mid)


def test_host_pipeline_knobs_parse_units():
    """RDC_HOST_PIECE_BYTES takes the reference's size units (ParseUnit,
    communicator_manager.cc:14-42: 4M == 4194304), and RDC_HOST_INLINE_BYTES
    moves the one-piece threshold (0: every buffer above one piece is
    pipelined)."""
    sizes = [4 << 20, 16 << 20, (16 << 20) + 4096]
    a = host_pieces(sizes, {"RDC_HOST_PIECE_BYTES": "2M"})
    b = host_pieces(sizes, {"RDC_HOST_PIECE_BYTES": str(2 << 20)})
    assert a == b
    assert a[16 << 20] == [0, 16 << 20]                      # inline up to 16 MiB by default
    assert len(a[(16 << 20) + 4096]) - 1 == 3 + 7 + 3         # ramps + pieces of <= 2 MiB above
    c = host_pieces(sizes, {"RDC_HOST_PIECE_BYTES": "2M", "RDC_HOST_INLINE_BYTES": "1M"})
    lens = [y - x for x, y in zip(c[16 << 20], c[16 << 20][1:])]
    assert lens[:3] == [256 << 10, 512 << 10, 1 << 20] and max(lens) <= 2 << 20 and sum(lens) == 16 << 20
    assert [y - x for x, y in zip(c[4 << 20], c[4 << 20][1:])] == [2 << 20, 2 << 20]
    # an explicit 0 pipelines everything above one piece; a malformed value
    # keeps the 16 MiB default (it used to act as 0)
    z = host_pieces(sizes, {"RDC_HOST_PIECE_BYTES": "2M", "RDC_HOST_INLINE_BYTES": "0"})
    assert len(z[4 << 20]) - 1 == 2 and len(z[16 << 20]) - 1 > 1
    for bad in ("abc", "16 M", "4Q", "12MB"):
        m = host_pieces(sizes, {"RDC_HOST_PIECE_BYTES": "2M", "RDC_HOST_INLINE_BYTES": bad})
        assert m == a, bad


def hbm(n, count, dtype, algo):
    from rdc_amd._lib import _LIB
    out = (ctypes.c_uint64 * 5)()
    assert _LIB.RdcPlanHbmBytes(n, count, dtype, algo, out) == 0
    return dict(read=out[0], write=out[1], read_sum=out[2], write_sum=out[3], egress=out[4])


@pytest.mark.parametrize("n", [2, 3, 4, 5, 8, 16])
def test_hbm_byte_model_closed_forms(n):
    """The committed per-schedule HBM byte model (RdcPlanHbmBytes, rdc_plan.cpp
    ModelHbmBytes) bench.py's N > 1 roofline uses.  Closed forms, S = buffer
    bytes: ring 5(n-1)/n S loaded + 4(n-1)/n S stored per rank; mesh
    (3n-2)/n S each way; one-shot (2n-1) S loaded + n S stored; egress
    2(n-1)/n S for ring and mesh (what the link roofline counts) and (n-1) S
    for the one-shot; the pull-mode mesh loads what the mesh loads and
    stores 2n S over the ranks; the direct schedule loads and stores S per
    rank with the mesh's egress.  Ragged Split chunks: the rank sums keep the
    closed forms exactly."""
    for count in (n * 4096, n * 4096 + n - 1, 1001):
        S = 4 * count
        ring, mesh, one = hbm(n, count, 6, 1), hbm(n, count, 6, 2), hbm(n, count, 6, 3)
        assert ring["read_sum"] == 5 * (n - 1) * S and ring["write_sum"] == 4 * (n - 1) * S
        assert mesh["read_sum"] == mesh["write_sum"] == (3 * n - 2) * S
        assert one["read_sum"] == n * (2 * n - 1) * S and one["write_sum"] == n * n * S
        assert hbm(n, count, 6, 4) == one
        pull = hbm(n, count, 6, 5)   # pull-mode mesh: same loads, one local result copy instead of n-1 remote
        assert pull["read_sum"] == mesh["read_sum"] and pull["write_sum"] == 2 * n * S
        assert pull["egress"] == mesh["egress"]
        direct = hbm(n, count, 6, 6)  # registered buffers: each buffer read once and written once
        assert direct["read_sum"] == direct["write_sum"] == n * S
        if count % n == 0:
            assert direct["read"] == direct["write"] == S and direct["egress"] == mesh["egress"]
        if count % n == 0:
            assert ring["read"] * n == 5 * (n - 1) * S and ring["write"] * n == 4 * (n - 1) * S
            assert mesh["read"] * n == (3 * n - 2) * S
            assert ring["egress"] * n == mesh["egress"] * n == 2 * (n - 1) * S
        assert one["egress"] == (n - 1) * S
    # n = 2, 1 GiB: the ring loads 2.5 S and stores 2 S per rank (4.5 S)
    r2 = hbm(2, 1 << 28, 6, 1)
    assert r2["read"] + r2["write"] == 9 * (1 << 30) // 2
    assert hbm(8, 1 << 28, 6, 2)["read"] * 8 == 22 * (1 << 30)   # mesh 5.5 S per rank at n = 8, both ways
    from rdc_amd._lib import _LIB
    assert _LIB.RdcPlanHbmBytes(2, 10, 6, 0, (ctypes.c_uint64 * 5)()) != 0   # auto is not a schedule


def piece_ranges(n, count, dtype, lo, hi, balanced):
    from rdc_amd._lib import _LIB
    off, ln, fold = (ctypes.c_uint64 * 16)(), (ctypes.c_uint64 * 16)(), (ctypes.c_int * 16)()
    assert _LIB.RdcPlanHostPieceRanges(n, count, dtype, lo, hi, balanced, off, ln, fold) == 0
    return [(off[q], ln[q], fold[q]) for q in range(n)]


@pytest.mark.parametrize("n", [2, 3, 5, 8, 16])
def test_host_piece_ranges_keep_every_element_in_its_chunk_order(n):
    """A host-path piece's ranges (rdc_plan.cpp HostPieceRanges): every byte of
    the piece lies in exactly one range, and that range folds in the ring
    order of the element's own Split chunk — chunk-owned (range q = the
    piece's bytes of chunk q) or balanced (each chunk's bytes cut over the
    ranks, at least one rank per chunk, parts within a chunk differing by at
    most one element), which is what keeps the balanced layout bit-exact."""
    rng = np.random.default_rng(n)
    for _ in range(60):
        esz = int(rng.choice([1, 4, 8]))
        dtype = {1: 1, 4: 6, 8: 7}[esz]
        count = int(rng.integers(n, 1 << 22))
        a, b = sorted(int(x) for x in rng.integers(0, count + 1, 2))
        lo, hi = a * esz, b * esz
        split = O.split(count, n)
        for balanced in (0, 1):
            rs = piece_ranges(n, count, dtype, lo, hi, balanced)
            covered = sorted((o, l, f) for o, l, f in rs if l)
            at = 0
            for o, l, f in covered:
                assert o == at, (n, count, lo, hi, balanced, rs)
                e0, e1 = (lo + o) // esz, (lo + o + l) // esz  # global elements of this range
                cb, ce = split[f]
                assert cb <= e0 and e1 <= ce, (n, count, lo, hi, balanced, rs)
                at += l
            assert at == hi - lo
            if not balanced:
                assert [f for _, _, f in rs] == list(range(n))
            else:
                chunks = [q for q in range(n) if max(lo, split[q][0] * esz) < min(hi, split[q][1] * esz)]
                if chunks:
                    assert {f for _, l, f in rs if l} == set(chunks)
                    for q in chunks:
                        parts = [l // esz for _, l, f in rs if f == q]
                        assert len(parts) >= 1 and max(parts) - min(parts) <= 1, (q, parts)
                    assert len([1 for _, l, _ in rs if l]) == min(n, (hi - lo) // esz) or len(chunks) > 1
    # chunk 3 of an 8-rank buffer of 8 Mi fp32 (4 MiB) as one piece: 8 equal parts in its order
    rs = piece_ranges(8, 8 << 20, 6, 4 * (3 << 20), 4 * (4 << 20), 1)
    assert [l for _, l, _ in rs] == [512 << 10] * 8 and {f for _, _, f in rs} == {3}


def test_host_pipeline_default_piece_is_16MiB(monkeypatch):
    """With RDC_HOST_PIECE_BYTES unset, pieces are 16 MiB (round 4's measured
    default, rdc_host.cpp HostPieceBytes): 256 MiB = the ramp (2, 4, 8 MiB),
    pieces of about 16 MiB, the mirrored ramp."""
    monkeypatch.delenv("RDC_HOST_PIECE_BYTES", raising=False)
    monkeypatch.delenv("RDC_HOST_PIECE_RAMP", raising=False)
    b = host_pieces([256 << 20], {})[256 << 20]
    lens = [y - x for x, y in zip(b, b[1:])]
    P = 16 << 20
    assert lens[:3] == [P // 8, P // 4, P // 2] and max(lens) <= P + 4096, lens
    assert sum(lens) == 256 << 20


def _xcd_loads(grid, xcds):
    """Workgroups per XCD of one dispatch (workgroup i -> XCD i % xcds)."""
    return [len(range(x, grid, xcds)) for x in range(xcds)]


@pytest.mark.parametrize("per_cu,ranks,reserve,expect", [
    (2, 1, 1, 496),   # one rank per GPU, its service block's CU kept: 8 x (64 - 2)
    (2, 4, 4, 112),   # 4 ranks on one GPU with services: 8 x floor((64 - 8) / 4)
    (2, 5, 5, 80),    # 5 ranks: the old clamp gave 100, i.e. 13 per XCD x 5 = 65 > 64 on XCDs 0-3
    (2, 8, 8, 48),
    (1, 3, 0, 80),    # one block per CU, 3 ranks sharing the GPU: 8 x floor(32 / 3), full XCDs
    (1, 6, 0, 24),    # 6 ranks: 5/8 of every XCD (20 of 32 CUs) / 6 -> 3 per XCD
    (1, 5, 0, 32),    # the 5 x 3-queue starvation config: 4 per XCD per rank
    (1, 1, 1, 248),   # one rank per GPU: no slack taken
])
def test_resident_grid_per_xcd(per_cu, ranks, reserve, expect):
    """rdc_plan.cpp ResidentGrid with XCDs (RdcPlanResidentGridXcd): on 256 CUs
    in 8 XCDs every XCD holds every rank's workgroups of one dispatch, even
    with every reserved CU on that XCD.  The old whole-GPU clamp let 5 ranks'
    mesh grids of 100 put 65 workgroups on XCD 0's 64 slots, and a spinning
    collective whose workgroup never starts waits out RDC_TIMEOUT (the 5-rank
    host sweep on one GPU)."""
    from rdc_amd._lib import _LIB
    g = _LIB.RdcPlanResidentGridXcd(4096, per_cu, 256, ranks, 8, reserve)
    assert g == expect
    assert max(_xcd_loads(g, 8)) * ranks <= per_cu * 32 - per_cu * reserve
    if per_cu == 1 and ranks >= 5:
        assert max(_xcd_loads(g, 8)) * ranks <= (32 - reserve) * 5 // 8
    assert _LIB.RdcPlanResidentGridXcd(4096, per_cu, 256, ranks, 1, 0) == _LIB.RdcPlanResidentGrid(4096, per_cu, 256,
                                                                                                     ranks)


def test_resident_grid_per_xcd_never_oversubscribes_an_xcd():
    from rdc_amd._lib import _LIB
    rng = np.random.default_rng(5)
    for _ in range(3000):
        xcds = int(rng.choice([1, 2, 4, 8]))
        cus = xcds * int(rng.integers(1, 40))
        want, per_cu, ranks = int(rng.integers(1, 8192)), int(rng.integers(1, 9)), int(rng.integers(1, 17))
        reserve = int(rng.integers(0, 3)) * ranks // 2
        g = _LIB.RdcPlanResidentGridXcd(want, per_cu, cus, ranks, xcds, reserve)
        assert 1 <= g <= max(1, want)
        room = per_cu * (cus // xcds) - per_cu * reserve
        assert g == 1 or max(_xcd_loads(g, xcds)) * ranks <= room, (want, per_cu, cus, ranks, xcds, reserve, g)


@pytest.mark.parametrize("n", [2, 3, 5, 8])
def test_plan_direct_items_cover_each_owner_chunk(n):
    """The coalesced direct launch's owner items (RdcPlanDirectItems, the
    table k_direct walks): for every owner r, the items are exactly Split
    chunk r of every buffer (oracle split), in order, cut into pieces of at
    most `tile` bytes; every element of every buffer belongs to exactly one
    owner's items."""
    from rdc_amd._lib import _LIB
    counts = [1024, 7, 0, 100003, 1, 65536, 3, (1 << 18) + 3]
    for dt, esz in ((6, 4), (10, 2), (0, 1)):
        for tile in (256, 64 << 10):
            covered = [np.zeros(c, dtype=np.int32) for c in counts]
            for r in range(n):
                arr = (ctypes.c_size_t * len(counts))(*counts)
                cap = 1 << 14
                out = (ctypes.c_uint64 * (3 * cap))()
                k = ctypes.c_int()
                assert _LIB.RdcPlanDirectItems(n, r, arr, len(counts), dt, tile, out, cap, ctypes.byref(k)) == 0
                items = [tuple(out[3 * i: 3 * i + 3]) for i in range(k.value)]
                want = []
                for b, c in enumerate(counts):
                    lo, hi = O.split(c, n)[r]
                    so, sl = lo * esz, (hi - lo) * esz
                    want += [(b, so + x, min(tile, sl - x)) for x in range(0, sl, tile)]
                assert items == want, (n, r, dt, tile)
                for b, so, ln in items:
                    covered[b][so // esz: (so + ln) // esz] += 1
            assert all((cv == 1).all() for cv in covered), (n, dt, tile)
    assert _LIB.RdcPlanDirectItems(n, n, (ctypes.c_size_t * 1)(4), 1, 6, 256, None, 0, ctypes.byref(ctypes.c_int())) != 0
