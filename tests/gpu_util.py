"""Shared helpers of the GPU parity tests (byte-level device buffers)."""
import ctypes

import numpy as np

from oracle import oracle as O

VALID = [(dt, op) for dt in range(12) for op in range(4) if not (op == 3 and dt in O.FLOAT_DTYPES)]


def to_dev(a, pad=0):
    """numpy array -> uint8 ROCm tensor holding its bytes (+ pad bytes in front)."""
    import torch
    raw = np.frombuffer(np.ascontiguousarray(a).tobytes(), dtype=np.uint8)
    t = torch.zeros(raw.size + pad + 64, dtype=torch.uint8, device="cuda")
    t[pad: pad + raw.size] = torch.from_numpy(raw.copy()).cuda()
    return t


def from_dev(t, pad, count, dtype):
    npd = O.NP_DTYPE[dtype]
    nbytes = count * np.dtype(npd).itemsize
    return np.frombuffer(t[pad: pad + nbytes].cpu().numpy().tobytes(), dtype=npd).copy()


def ptr(t, pad=0):
    return ctypes.c_void_p(t.data_ptr() + pad)


def rand_input(rng, count, dtype, special=True):
    """Full-range integers; floats with full mantissas plus +-0, +-inf, denormals."""
    npd = O.NP_DTYPE[dtype]
    if dtype in (O.DT_FLOAT32, O.DT_FLOAT64, O.DT_FLOAT16):
        x = (rng.standard_normal(count) * rng.choice([1e-3, 1.0, 1e3], count)).astype(npd)
        if special and count >= 8:
            fi = np.finfo(npd)
            idx = rng.choice(count, min(count, 8), replace=False)
            vals = np.array([0.0, -0.0, np.inf, -np.inf, fi.tiny / 4, -fi.tiny / 8, fi.max, -fi.max], dtype=npd)
            x[idx] = vals[: idx.size]
        return x
    if dtype == O.DT_BFLOAT16:
        f = (rng.standard_normal(count) * 3).astype(np.float32)
        x = np.array([O.lib().rdc_oracle_f32_to_bf16(float(v)) for v in f], dtype=np.uint16)
        if special and count >= 8:
            # +-0, +-inf, a denormal, the largest finite (sums overflow to inf), a quiet NaN, -denormal
            vals = np.array([0x0000, 0x8000, 0x7F80, 0xFF80, 0x0001, 0x7F7F, 0x7FC1, 0x8003], dtype=np.uint16)
            idx = rng.choice(count, 8, replace=False)
            x[idx] = vals
        return x
    info = np.iinfo(npd)
    return rng.integers(info.min, info.max, count, dtype=npd, endpoint=True)


def same_bits(a, b, dtype):
    """Bit-exact equality, treating any two NaNs as equal (NaN payloads are not pinned)."""
    if dtype == O.DT_BFLOAT16:
        an, bn = (a & 0x7FFF) > 0x7F80, (b & 0x7FFF) > 0x7F80
        if not np.array_equal(an, bn):
            return False
        return a[~an].tobytes() == b[~bn].tobytes()
    if dtype in (O.DT_FLOAT32, O.DT_FLOAT64, O.DT_FLOAT16):
        an, bn = np.isnan(a), np.isnan(b)
        if not np.array_equal(an, bn):
            return False
        return a[~an].tobytes() == b[~bn].tobytes()
    return a.tobytes() == b.tobytes()
