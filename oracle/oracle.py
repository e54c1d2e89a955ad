"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes/numpy front end over oracle/liboracle.so (the plain-C restatement of
rdc's ring allreduce, oracle/rdc_oracle.c) and, where built, oracle/_ref/
libref_ring.so (the reference's own op::Reducer + utils::Split compiled from
/root/reference/include, oracle/ref_ring.cc).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker.  The product (rdc_amd) never does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(HERE, "liboracle.so")
_REF_PATH = os.path.join(HERE, "_ref", "libref_ring.so")

# mpi::DataType (include/core/mpi.h:19-30) + float16=10, bfloat16=11
DT_INT8, DT_UINT8, DT_INT32, DT_UINT32, DT_INT64, DT_UINT64 = 0, 1, 2, 3, 4, 5
DT_FLOAT32, DT_FLOAT64, DT_LONGLONG, DT_ULONGLONG = 6, 7, 8, 9
DT_FLOAT16, DT_BFLOAT16 = 10, 11
# mpi::OpType (include/core/mpi.h:12-17)
OP_MAX, OP_MIN, OP_SUM, OP_BITOR = 0, 1, 2, 3

# numpy storage dtype per enum (bfloat16 stored as uint16 bits)
NP_DTYPE = {
    DT_INT8: np.int8, DT_UINT8: np.uint8, DT_INT32: np.int32, DT_UINT32: np.uint32,
    DT_INT64: np.int64, DT_UINT64: np.uint64, DT_FLOAT32: np.float32,
    DT_FLOAT64: np.float64, DT_LONGLONG: np.int64, DT_ULONGLONG: np.uint64,
    DT_FLOAT16: np.float16, DT_BFLOAT16: np.uint16,
}
FLOAT_DTYPES = (DT_FLOAT32, DT_FLOAT64, DT_FLOAT16, DT_BFLOAT16)

_lib = None
_ref = None


def build():
    """Compile oracle/ (and oracle/_ref when /root/reference is present)."""
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, u64, i64 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64
        L.rdc_oracle_dtype_size.restype = ctypes.c_size_t
        L.rdc_oracle_split.argtypes = [i64, i64, ctypes.c_int, ctypes.POINTER(i64), ctypes.POINTER(i64)]
        L.rdc_oracle_reducer.argtypes = [vp, vp, u64, ctypes.c_int, ctypes.c_int]
        L.rdc_oracle_ring_schedule.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.POINTER(ctypes.c_int)] * 4
        L.rdc_oracle_allreduce_ring.argtypes = [ctypes.POINTER(vp), ctypes.c_int, u64, ctypes.c_int, ctypes.c_int]
        L.rdc_oracle_allreduce_closed_form.argtypes = [ctypes.POINTER(vp), ctypes.c_int, u64, ctypes.c_int, ctypes.c_int, vp]
        L.rdc_oracle_fill.argtypes = [vp, u64, ctypes.c_int, u64, ctypes.c_int]
        L.rdc_oracle_allreduce_tree.argtypes = [ctypes.POINTER(vp), ctypes.c_int, u64, ctypes.c_int, ctypes.c_int]
        L.rdc_oracle_tree_program.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.rdc_oracle_tree.argtypes = [ctypes.c_int] + [ctypes.POINTER(ctypes.c_int)] * 4
        L.rdc_oracle_fill_at.argtypes = [vp, u64, u64, ctypes.c_int, u64, ctypes.c_int]
        L.rdc_oracle_allreduce_window.argtypes = [ctypes.POINTER(vp), ctypes.c_int, u64, u64, u64, ctypes.c_int,
                                                  ctypes.c_int, vp]
        L.rdc_oracle_splitmix64.restype = u64
        L.rdc_oracle_splitmix64.argtypes = [u64]
        L.rdc_oracle_f32_to_f16.restype = ctypes.c_uint16
        L.rdc_oracle_f32_to_f16.argtypes = [ctypes.c_float]
        L.rdc_oracle_f16_to_f32.restype = ctypes.c_float
        L.rdc_oracle_f16_to_f32.argtypes = [ctypes.c_uint16]
        L.rdc_oracle_f32_to_bf16.restype = ctypes.c_uint16
        L.rdc_oracle_f32_to_bf16.argtypes = [ctypes.c_float]
        _lib = L
    return _lib


def ref_available():
    return os.path.exists(_REF_PATH)


def ref():
    """The reference's own Reducer/Split (oracle/_ref). None if not built."""
    global _ref
    if _ref is None and ref_available():
        R = ctypes.CDLL(_REF_PATH)
        vp = ctypes.c_void_p
        R.ref_reducer.argtypes = [vp, vp, ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
        R.ref_split.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        R.ref_allreduce_ring.argtypes = [ctypes.POINTER(vp), ctypes.c_int, ctypes.c_uint64,
                                         ctypes.c_int, ctypes.c_int]
        _ref = R
    return _ref


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def split(count, n):
    """utils::Split(0, count, n) -> list of (begin, end)."""
    b = (ctypes.c_int64 * n)()
    e = (ctypes.c_int64 * n)()
    lib().rdc_oracle_split(0, count, n, b, e)
    return [(b[i], e[i]) for i in range(n)]


def ring_schedule(n, rank):
    arrs = [(ctypes.c_int * 16)() for _ in range(4)]
    rc = lib().rdc_oracle_ring_schedule(n, rank, *arrs)
    if rc:
        raise RuntimeError("ring_schedule rc=%d" % rc)
    return [list(a[: n - 1]) for a in arrs]


def reducer(src, dst, dtype, op):
    """op::Reducer<OP,DType>(src, dst, len) in place on dst (numpy arrays)."""
    assert src.size == dst.size and dst.flags.c_contiguous and src.flags.c_contiguous
    rc = lib().rdc_oracle_reducer(_ptr(src), _ptr(dst), dst.size, dtype, op)
    if rc:
        raise ValueError("oracle reducer rejects dtype=%d op=%d" % (dtype, op))
    return dst


def allreduce_ring(bufs, dtype, op):
    """Lock-step ring allreduce over per-rank numpy buffers (in place). Returns bufs."""
    n = len(bufs)
    arr = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])
    rc = lib().rdc_oracle_allreduce_ring(arr, n, bufs[0].size, dtype, op)
    if rc:
        raise ValueError("oracle allreduce rc=%d" % rc)
    return bufs


def allreduce_closed_form(bufs, dtype, op):
    n = len(bufs)
    out = np.empty_like(bufs[0])
    arr = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])
    rc = lib().rdc_oracle_allreduce_closed_form(arr, n, bufs[0].size, dtype, op, _ptr(out))
    if rc:
        raise ValueError("oracle closed form rc=%d" % rc)
    return out


def ref_allreduce_ring(bufs, dtype, op):
    R = ref()
    n = len(bufs)
    arr = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])
    rc = R.ref_allreduce_ring(arr, n, bufs[0].size, dtype, op)
    if rc:
        raise ValueError("ref allreduce rc=%d" % rc)
    return bufs


def fill(count, dtype, seed, rank):
    """Synthetic per-rank input (SURVEY.md §8d generator), identical to the device fill."""
    a = np.empty(count, dtype=NP_DTYPE[dtype])
    rc = lib().rdc_oracle_fill(_ptr(a), count, dtype, seed, rank)
    if rc:
        raise ValueError("fill rc=%d" % rc)
    return a


def fill_at(first, count, dtype, seed, rank):
    """Elements [first, first+count) of fill()'s stream (position-keyed)."""
    a = np.empty(count, dtype=NP_DTYPE[dtype])
    rc = lib().rdc_oracle_fill_at(_ptr(a), first, count, dtype, seed, rank)
    if rc:
        raise ValueError("fill_at rc=%d" % rc)
    return a


def expected_window(total, first, m, n, dtype, op, seed):
    """Allreduce result at positions [first, first+m) of a `total`-element
    buffer whose rank-r input is fill(total, dtype, seed, r): the ring's
    per-chunk closed form on the window alone (for full-size checks)."""
    wins = [fill_at(first, m, dtype, seed, r) for r in range(n)]
    out = np.empty(m, dtype=NP_DTYPE[dtype])
    arr = (ctypes.c_void_p * n)(*[w.ctypes.data for w in wins])
    rc = lib().rdc_oracle_allreduce_window(arr, n, total, first, m, dtype, op, _ptr(out))
    if rc:
        raise ValueError("allreduce_window rc=%d" % rc)
    return out


def tree_program(n):
    """The small-buffer (rdc_reduce_ring_mincount) path's fold for n ranks:
    [(dst, src), ...] with acc[dst] = OP(acc[dst], acc[src]), result acc[0]
    (oracle/tree_order.cc)."""
    d, s = (ctypes.c_int * 16)(), (ctypes.c_int * 16)()
    k = lib().rdc_oracle_tree_program(n, d, s)
    if k < 0:
        raise ValueError("tree_program n=%d" % n)
    return [(d[i], s[i]) for i in range(k)]


def tree(n):
    """(children-in-fold-order per rank, parent, depth) of the reference's tree."""
    nc, ch, par, dep = (ctypes.c_int * 16)(), (ctypes.c_int * 256)(), (ctypes.c_int * 16)(), (ctypes.c_int * 16)()
    if lib().rdc_oracle_tree(n, nc, ch, par, dep):
        raise ValueError("tree n=%d" % n)
    return [[ch[r * 16 + i] for i in range(nc[r])] for r in range(n)], list(par[:n]), list(dep[:n])


def allreduce_tree(bufs, dtype, op):
    """TryAllreduceTree over per-rank numpy buffers (in place): every buffer
    receives the root's tree reduction.  Returns bufs."""
    n = len(bufs)
    arr = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])
    rc = lib().rdc_oracle_allreduce_tree(arr, n, bufs[0].size, dtype, op)
    if rc:
        raise ValueError("oracle tree allreduce rc=%d" % rc)
    return bufs


def expected_tree(inputs, dtype, op):
    bufs = [np.ascontiguousarray(x).copy() for x in inputs]
    allreduce_tree(bufs, dtype, op)
    return bufs[0]


def expected_allreduce(inputs, dtype, op):
    """Reference result for per-rank inputs (copies; inputs untouched)."""
    bufs = [np.ascontiguousarray(x).copy() for x in inputs]
    allreduce_ring(bufs, dtype, op)
    return bufs[0]
