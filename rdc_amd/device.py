"""Device-memory helpers: torch dtype mapping, op::Reducer on the GPU, and
the synthetic input generator (bit-identical to the CPU oracle's)."""
import ctypes

from ._lib import _LIB, check_call

_TORCH_ENUM = None


def dtype_enum(torch_dtype):
    global _TORCH_ENUM
    if _TORCH_ENUM is None:
        import torch
        m = {
            torch.int8: 0, torch.uint8: 1, torch.int32: 2, torch.int64: 4,
            torch.float32: 6, torch.float64: 7, torch.float16: 10, torch.bfloat16: 11,
        }
        for name, v in (("uint32", 3), ("uint64", 5)):
            if hasattr(torch, name):
                m[getattr(torch, name)] = v
        _TORCH_ENUM = m
    try:
        return _TORCH_ENUM[torch_dtype]
    except KeyError:
        raise TypeError("rdc_amd: dtype %s not supported" % torch_dtype)


def current_stream_ptr(device=None):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _check_tensor(t):
    if not t.is_cuda:
        raise ValueError("rdc_amd: expected a tensor on a ROCm device")
    if not t.is_contiguous():
        raise ValueError("rdc_amd: tensor must be contiguous")


def reduce_(dst, src, op, stream=None):
    """dst = OP(dst, src) element-wise on the GPU (op::Reducer, include/core/mpi.h:113-120)."""
    _check_tensor(dst)
    _check_tensor(src)
    if dst.dtype != src.dtype or dst.numel() != src.numel():
        raise ValueError("rdc_amd: dst/src dtype or size mismatch")
    s = stream if stream is not None else current_stream_ptr(dst.device)
    check_call(_LIB.RdcReduce(ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(src.data_ptr()), dst.numel(),
                              dtype_enum(dst.dtype), int(op), s))
    return dst


def fill_(t, seed, rank, stream=None):
    """Synthetic input u = splitmix64(seed ^ rank<<40 ^ i) mapped per dtype."""
    _check_tensor(t)
    s = stream if stream is not None else current_stream_ptr(t.device)
    check_call(_LIB.RdcFill(ctypes.c_void_p(t.data_ptr()), t.numel(), dtype_enum(t.dtype), seed, rank, s))
    return t
