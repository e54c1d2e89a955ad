"""rdc's Python surface (rdc/core.py) over the MI355X device path.

Same names, argument meaning and results as the reference module:
``init``, ``finalize``, ``get_rank``, ``get_world_size``, ``tracker_print``,
``get_processor_name``, ``broadcast`` (pickled objects), ``allreduce``
(ndarray copy semantics) and the ``Op`` enum (rdc/core.py:16-27).  The
reference binds ``_LIB.Rdc*`` symbols that were never implemented
(SURVEY.md §0 finding 3); here they are the C ABI of librdc_amd.so.

Device extension: ``allreduce`` also takes a ROCm ``torch.Tensor`` and then
reduces it in place on the GPU, stream-ordered on torch's current stream.
"""
import ctypes
import pickle
import sys
from enum import Enum

import numpy as np

from ._lib import _LIB, check_call


class Op(Enum):
    """Reduction operators = mpi::OpType (include/core/mpi.h:12-17)."""
    MAX = 0
    MIN = 1
    SUM = 2
    BITOR = 3

    def __int__(self):
        return self.value


# numpy dtype -> mpi::DataType (rdc/core.py:160-169 = include/core/mpi.h:19-30),
# plus the MI355X additions float16 = 10 (bfloat16 = 11 via torch only)
DTYPE_ENUM__ = {
    np.dtype("int8"): 0,
    np.dtype("uint8"): 1,
    np.dtype("int32"): 2,
    np.dtype("uint32"): 3,
    np.dtype("int64"): 4,
    np.dtype("uint64"): 5,
    np.dtype("float32"): 6,
    np.dtype("float64"): 7,
    np.dtype("float16"): 10,
}


def init(args=None, lib="standard", lib_dll=None):
    """Initialise rdc (RdcInit); ``args`` defaults to sys.argv (key=val pairs are parameters)."""
    del lib, lib_dll  # one backend: the MI355X device path
    if args is None:
        args = sys.argv
    enc = [a.encode() if isinstance(a, str) else bytes(a) for a in args]
    arr = (ctypes.c_char_p * max(1, len(enc)))()
    arr[: len(enc)] = enc
    check_call(_LIB.RdcInit(len(enc), arr))


def finalize():
    check_call(_LIB.RdcFinalize())


def get_rank():
    return _LIB.RdcGetRank()


def get_world_size():
    return _LIB.RdcGetWorldSize()


def is_distributed():
    return bool(_LIB.RdcIsDistributed())


def tracker_print(msg):
    if not isinstance(msg, str):
        msg = str(msg)
    check_call(_LIB.RdcTrackerPrint(msg.encode("utf-8")))


def get_processor_name():
    mxlen = 256
    length = ctypes.c_ulong()
    buf = ctypes.create_string_buffer(mxlen)
    check_call(_LIB.RdcGetProcessorName(buf, ctypes.byref(length), mxlen))
    return buf.value


def barrier():
    check_call(_LIB.RdcBarrier())


def broadcast(data, root):
    """Broadcast a picklable object from ``root`` (two RdcBroadcast calls:
    length, then payload — rdc/core.py:121-156)."""
    rank = get_rank()
    length = ctypes.c_ulong()
    payload = None
    if root == rank:
        if data is None:
            raise ValueError("need to pass in data when broadcasting")
        payload = pickle.dumps(data, protocol=pickle.HIGHEST_PROTOCOL)
        length.value = len(payload)
    check_call(_LIB.RdcBroadcast(ctypes.byref(length), ctypes.sizeof(ctypes.c_ulong), root))
    if root != rank:
        dptr = (ctypes.c_char * length.value)()
        check_call(_LIB.RdcBroadcast(ctypes.cast(dptr, ctypes.c_void_p), length.value, root))
        return pickle.loads(dptr.raw)
    src = ctypes.create_string_buffer(payload, len(payload))
    check_call(_LIB.RdcBroadcast(ctypes.cast(src, ctypes.c_void_p), length.value, root))
    return data


_PREPARE_T = ctypes.CFUNCTYPE(None, ctypes.c_void_p)


def _torch_dtype_enum(t):
    from . import device
    return device.dtype_enum(t.dtype)


def allreduce(data, op, prepare_fun=None):
    """Allreduce across ranks.

    numpy.ndarray: returns the reduced, flattened array (a copy unless ravel
    gave a view of ``data`` — the reference's rule, rdc/core.py:196-217).
    torch.Tensor on a ROCm device: reduced in place on the GPU and returned.
    ``prepare_fun(data)``, if given, runs before the reduction.
    """
    op = int(Op(op) if not isinstance(op, Op) else op)
    if type(data).__module__.startswith("torch"):
        from . import comm as _comm
        if prepare_fun is not None:
            prepare_fun(data)
        return _comm.get_comm("main").allreduce(data, op)
    return host_allreduce(data, op, prepare_fun)


def host_allreduce(data, op, prepare_fun=None, comm=None):
    """rdc/core.py:172-217 on a host ndarray: RdcAllreduce on "main", or
    RdcAllreduceOn on the communicator handle ``comm``."""
    op = int(Op(op) if not isinstance(op, Op) else op)
    if not isinstance(data, np.ndarray):
        raise TypeError("allreduce only takes in numpy.ndarray or torch.Tensor")
    buf = data.ravel()
    if buf.base is data.base:
        buf = buf.copy()
    if buf.dtype not in DTYPE_ENUM__:
        raise TypeError("data type %s not supported" % str(buf.dtype))
    if not buf.flags.c_contiguous:
        buf = np.ascontiguousarray(buf)
    if comm is not None:
        if prepare_fun is not None:
            prepare_fun(data)
        check_call(_LIB.RdcAllreduceOn(comm, buf.ctypes.data_as(ctypes.c_void_p), buf.size,
                                       DTYPE_ENUM__[buf.dtype], op))
        return buf
    cb = None
    if prepare_fun is not None:
        cb = _PREPARE_T(lambda _arg: prepare_fun(data))
    check_call(_LIB.RdcAllreduce(buf.ctypes.data_as(ctypes.c_void_p), buf.size, DTYPE_ENUM__[buf.dtype], op,
                                 ctypes.cast(cb, ctypes.c_void_p) if cb is not None else None, None))
    return buf


def allreduce_coalesced(arrays, op):
    """Bucketed allreduce of a list of arrays of one dtype, in place: the
    result of ``allreduce`` on each one (bit-identical), moved in fused device
    launches (RdcAllreduceCoalesced).  numpy arrays (contiguous) or ROCm
    tensors (stream-ordered on torch's current stream).  Returns the list."""
    op = int(Op(op) if not isinstance(op, Op) else op)
    if not arrays:
        return arrays
    if type(arrays[0]).__module__.startswith("torch"):
        from . import comm as _comm
        return _comm.get_comm("main").allreduce_coalesced(arrays, op)
    for a in arrays:
        if not isinstance(a, np.ndarray) or not a.flags.c_contiguous:
            raise TypeError("allreduce_coalesced takes contiguous numpy arrays")
        if a.dtype != arrays[0].dtype:
            raise TypeError("allreduce_coalesced needs one dtype")
    if arrays[0].dtype not in DTYPE_ENUM__:
        raise TypeError("data type %s not supported" % str(arrays[0].dtype))
    nb = len(arrays)
    ptrs = (ctypes.c_void_p * nb)(*[a.ctypes.data for a in arrays])
    counts = (ctypes.c_size_t * nb)(*[a.size for a in arrays])
    check_call(_LIB.RdcAllreduceCoalesced(ptrs, counts, nb, DTYPE_ENUM__[arrays[0].dtype], op))
    return arrays


def allgather(arrays):
    """Allgather of host arrays (rdc::Allgather, include/api.h:47-52): arrays[c]
    is pre-sized on every rank and arrays[get_rank()] holds this rank's data;
    on return every arrays[c] holds rank c's data.  In place; returns arrays."""
    n = get_world_size()
    if len(arrays) != n:
        raise ValueError("allgather needs one array per rank")
    for a in arrays:
        if not isinstance(a, np.ndarray) or not a.flags.c_contiguous:
            raise TypeError("allgather takes contiguous numpy arrays")
    ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrays])
    sizes = (ctypes.c_size_t * n)(*[a.nbytes for a in arrays])
    check_call(_LIB.RdcAllgather(ptrs, sizes))
    return arrays


def send(buf, dest):
    """rdc::Send on the main communicator (include/api.h:10, rdc-inl.h:53-62):
    blocking send of a Buffer / ndarray / bytes / ROCm tensor to rank ``dest``."""
    from .comm import get_comm
    get_comm("main").send(buf, dest)


def recv(buf, src):
    """rdc::Recv on the main communicator (include/api.h:11): blocking receive
    into ``buf`` from rank ``src``; returns ``buf``."""
    from .comm import get_comm
    return get_comm("main").recv(buf, src)
