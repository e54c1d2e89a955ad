"""GPU parity: RdcReduce (op::Reducer<OP,DType> on gfx950) vs the CPU oracle,
bit-exact, for every (dtype, op) the reference supports, aligned and
misaligned buffers, sizes around the 16-B vector boundaries."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.gpu_util import VALID, from_dev, ptr, rand_input, same_bits, to_dev

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rdc_amd._lib import _LIB
    return _LIB


@pytest.mark.parametrize("dtype,op", VALID)
def test_reduce_all_types(lib, dtype, op):
    rng = np.random.default_rng(1000 + 16 * dtype + op)
    for count in (1, 7, 33, 1000, 4099):
        for pd, ps in ((0, 0), (4, 4), (2, 6)):
            esz = np.dtype(O.NP_DTYPE[dtype]).itemsize
            pd_b, ps_b = pd * esz, ps * esz
            d = rand_input(rng, count, dtype)
            s = rand_input(rng, count, dtype)
            td, ts = to_dev(d, pd_b), to_dev(s, ps_b)
            assert lib.RdcReduce(ptr(td, pd_b), ptr(ts, ps_b), count, dtype, op, None) == 0, \
                lib.RdcGetLastError()
            torch.cuda.synchronize()
            got = from_dev(td, pd_b, count, dtype)
            want = O.reducer(s.copy(), d.copy(), dtype, op)
            assert same_bits(got, want, dtype), (dtype, op, count, pd, ps)


@pytest.mark.parametrize("dtype,op", [(O.DT_FLOAT32, O.OP_SUM), (O.DT_FLOAT16, O.OP_SUM),
                                      (O.DT_INT8, O.OP_MAX), (O.DT_FLOAT64, O.OP_MIN)])
def test_reduce_large(lib, dtype, op):
    rng = np.random.default_rng(7)
    count = (1 << 22) + 5
    d = rand_input(rng, count, dtype)
    s = rand_input(rng, count, dtype)
    td, ts = to_dev(d, 16), to_dev(s, 16)
    assert lib.RdcReduce(ptr(td, 16), ptr(ts, 16), count, dtype, op, None) == 0
    torch.cuda.synchronize()
    assert same_bits(from_dev(td, 16, count, dtype), O.reducer(s, d.copy(), dtype, op), dtype)


def test_reduce_rejects_bitor_on_float(lib):
    t = torch.zeros(16, dtype=torch.float32, device="cuda")
    assert lib.RdcReduce(ptr(t), ptr(t), 16, O.DT_FLOAT32, O.OP_BITOR, None) != 0
    assert b"unsupported" in lib.RdcGetLastError()


def test_fill_matches_oracle(lib):
    for dtype in range(12):
        count = 10007
        npd = O.NP_DTYPE[dtype]
        t = torch.zeros(count * np.dtype(npd).itemsize + 64, dtype=torch.uint8, device="cuda")
        assert lib.RdcFill(ptr(t), count, dtype, 0x5EED0000, 3, None) == 0
        torch.cuda.synchronize()
        got = from_dev(t, 0, count, dtype)
        want = O.fill(count, dtype, 0x5EED0000, 3)
        assert got.tobytes() == want.tobytes(), dtype


@pytest.mark.parametrize("op", [O.OP_SUM, O.OP_MAX, O.OP_MIN])
def test_reduce_bf16_every_bit_pattern(lib, op):
    """bf16 (hardware v_cvt_pk_bf16_f32 on the Sum path): every one of the
    65536 bit patterns as dst against random patterns (NaNs, infs, denormals
    included), 16-B body and element-wise head/tail, vs the oracle."""
    rng = np.random.default_rng(99 + op)
    d = np.tile(np.arange(65536, dtype=np.uint16), 8)
    s = rng.integers(0, 65536, d.size, dtype=np.uint16)
    for pad in (0, 6):
        td, ts = to_dev(d, pad), to_dev(s, pad)
        assert lib.RdcReduce(ptr(td, pad), ptr(ts, pad), d.size, O.DT_BFLOAT16, op, None) == 0
        torch.cuda.synchronize()
        got = from_dev(td, pad, d.size, O.DT_BFLOAT16)
        want = O.reducer(s.copy(), d.copy(), O.DT_BFLOAT16, op)
        assert same_bits(got, want, O.DT_BFLOAT16), (op, pad)
