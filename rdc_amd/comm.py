"""Communicator handles — rdc/comm.py's ``new_comm`` / ``get_comm`` / ``Comm``
(rdc/comm.py:36-112) over the MI355X device path, plus single-process
multi-rank groups (``init_group``) for driving several GPUs from one process.
"""
import ctypes

from ._lib import _LIB, RdcError, check_call
from . import device as _dev
from .buffer import Buffer

# WorkStatus (include/core/work_request.h:23-30)
WS_PENDING, WS_RUNNING, WS_FINISHED, WS_ERROR = 1 << 1, 1 << 2, 1 << 3, 1 << 6


class TuneCand(ctypes.Structure):
    """RdcTuneCand (include/rdc_amd.h): one launch shape timed by RdcCommAutotune."""
    _fields_ = [("algo", ctypes.c_int), ("mesh_s16", ctypes.c_int), ("mesh_r16", ctypes.c_int),
                ("max_blocks", ctypes.c_int),
                ("tiles_per_block", ctypes.c_int), ("ms", ctypes.c_double), ("ms_min", ctypes.c_double),
                ("ms_max", ctypes.c_double)]


class WorkComp(object):
    """Completion of an isend / irecv (rdc/comm.py:11-33).  Holds the buffer
    alive until the handle is dropped."""
    __slots__ = ("handle", "own_handle", "_buf")

    def __init__(self, handle=None, own_handle=True, buf=None):
        self.handle = handle if handle is not None else ctypes.c_void_p()
        self.own_handle = own_handle
        self._buf = buf

    def __del__(self):
        h = getattr(self, "handle", None)
        if getattr(self, "own_handle", False) and h:
            _LIB.RdcDelWorkCompletion(h)
            self.handle = ctypes.c_void_p()

    def wait(self):
        """Block until the transfer finished; 0 on success (raises on error)."""
        rc = _LIB.RdcWorkCompletionWait(self.handle)
        if rc != 0:
            raise RdcError(_LIB.RdcWorkCompletionError(self.handle).decode("utf-8", "replace"))
        return rc

    def status(self):
        """WorkStatus bits: WS_PENDING, WS_FINISHED or WS_ERROR."""
        return _LIB.RdcWorkCompletionStatus(self.handle)


def _is_tensor(x):
    return hasattr(x, "data_ptr") and hasattr(x, "is_cuda")

ALGO_AUTO, ALGO_RING, ALGO_MESH, ALGO_ONESHOT, ALGO_TREE, ALGO_MESH_PULL, ALGO_DIRECT = 0, 1, 2, 3, 4, 5, 6
_ALGOS = {"auto": ALGO_AUTO, "ring": ALGO_RING, "mesh": ALGO_MESH, "oneshot": ALGO_ONESHOT, "tree": ALGO_TREE,
          "mesh_pull": ALGO_MESH_PULL, "direct": ALGO_DIRECT}


class Comm(object):
    """A communicator handle.  Collectives are in place on device memory and
    stream-ordered (torch's current stream unless ``stream`` is given)."""
    __slots__ = ("handle", "own_handle")

    def __init__(self, handle=None, own_handle=False):
        self.handle = ctypes.c_void_p(handle) if isinstance(handle, int) else (handle or ctypes.c_void_p())
        self.own_handle = own_handle

    @property
    def rank(self):
        return _LIB.RdcCommRank(self.handle)

    @property
    def world_size(self):
        return _LIB.RdcCommSize(self.handle)

    @property
    def device(self):
        return _LIB.RdcCommDevice(self.handle)

    @property
    def alloc_kind(self):
        return _LIB.RdcCommAllocKind(self.handle)

    def allreduce(self, tensor, op, algo="auto", stream=None):
        """In-place allreduce of a contiguous ROCm tensor on this
        communicator; returns it.  A numpy array takes rdc.allreduce's host
        path and copy rule (rdc/core.py:196-217) on this communicator
        (rdc::Allreduce<OP>(buf, count, comm_name), include/api.h:62-64) and
        returns the reduced flat array."""
        if not _is_tensor(tensor):
            from .core import host_allreduce
            return host_allreduce(tensor, op, comm=self.handle)
        _dev._check_tensor(tensor)
        s = stream if stream is not None else _dev.current_stream_ptr(tensor.device)
        check_call(_LIB.RdcCommAllreduceEx(self.handle, ctypes.c_void_p(tensor.data_ptr()), tensor.numel(),
                                           _dev.dtype_enum(tensor.dtype), int(op), _ALGOS[algo], s))
        return tensor

    def allreduce_coalesced(self, tensors, op, algo="auto", stream=None):
        """Bucketed allreduce of a list of contiguous ROCm tensors of one dtype,
        in place: the result of ``allreduce`` on each tensor in order
        (bit-identical), moved in fused launches.  Returns the list."""
        if not tensors:
            return tensors
        for t in tensors:
            _dev._check_tensor(t)
            if t.dtype != tensors[0].dtype:
                raise ValueError("rdc_amd: allreduce_coalesced needs one dtype")
        nb = len(tensors)
        ptrs = (ctypes.c_void_p * nb)(*[t.data_ptr() for t in tensors])
        counts = (ctypes.c_size_t * nb)(*[t.numel() for t in tensors])
        s = stream if stream is not None else _dev.current_stream_ptr(tensors[0].device)
        check_call(_LIB.RdcCommAllreduceCoalesced(self.handle, ptrs, counts, nb, _dev.dtype_enum(tensors[0].dtype),
                                                  int(op), _ALGOS[algo], s))
        return tensors

    def allreduce_ptr(self, ptr, count, dtype, op, algo=ALGO_AUTO, stream=None):
        check_call(_LIB.RdcCommAllreduceEx(self.handle, ctypes.c_void_p(ptr), count, dtype, int(op), algo,
                                           stream))

    def broadcast(self, tensor, root, stream=None):
        _dev._check_tensor(tensor)
        s = stream if stream is not None else _dev.current_stream_ptr(tensor.device)
        check_call(_LIB.RdcCommBroadcast(self.handle, ctypes.c_void_p(tensor.data_ptr()),
                                         tensor.numel() * tensor.element_size(), root, s))
        return tensor

    def allgather(self, tensors, stream=None):
        """tensors[c] (contiguous, ROCm) receives rank c's data; tensors[rank] is
        this rank's input.  Sizes may differ per rank.  In place; returns the list."""
        n = self.world_size
        if len(tensors) != n:
            raise ValueError("rdc_amd: allgather needs one tensor per rank")
        for t in tensors:
            _dev._check_tensor(t)
        ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in tensors])
        sizes = (ctypes.c_size_t * n)(*[t.numel() * t.element_size() for t in tensors])
        s = stream if stream is not None else _dev.current_stream_ptr(tensors[0].device)
        check_call(_LIB.RdcCommAllgather(self.handle, ptrs, sizes, s))
        return tensors

    # ----------------------------------------------------- point-to-point --
    def isend(self, buf, dest_rank):
        """Non-blocking send of a Buffer, ndarray, bytes/bytearray or ROCm
        tensor to ``dest_rank`` (rdc/comm.py:46-63).  A device tensor is sent
        after the work already queued on torch's current stream."""
        if _is_tensor(buf) and buf.is_cuda:
            _dev._check_tensor(buf)
            wc = WorkComp(buf=buf)
            check_call(_LIB.RdcCommISend(ctypes.byref(wc.handle), self.handle, ctypes.c_void_p(buf.data_ptr()),
                                         buf.numel() * buf.element_size(), int(dest_rank),
                                         _dev.current_stream_ptr(buf.device)))
            return wc
        b = buf if isinstance(buf, Buffer) else Buffer(buf)
        wc = WorkComp(buf=b)
        check_call(_LIB.RdcISend(ctypes.byref(wc.handle), self.handle, b.handle, int(dest_rank)))
        return wc

    def irecv(self, buf, src_rank):
        """Non-blocking receive into a Buffer, ndarray, bytearray or ROCm tensor
        from ``src_rank`` (rdc/comm.py:65-80)."""
        if _is_tensor(buf) and buf.is_cuda:
            _dev._check_tensor(buf)
            wc = WorkComp(buf=buf)
            check_call(_LIB.RdcCommIRecv(ctypes.byref(wc.handle), self.handle, ctypes.c_void_p(buf.data_ptr()),
                                         buf.numel() * buf.element_size(), int(src_rank),
                                         _dev.current_stream_ptr(buf.device)))
            return wc
        b = buf if isinstance(buf, Buffer) else Buffer(buf)
        h = _LIB.RdcIRecv(self.handle, b.handle, int(src_rank))
        if not h:
            raise RdcError(_LIB.RdcGetLastError().decode("utf-8", "replace"))
        return WorkComp(ctypes.c_void_p(h), buf=b)

    def send(self, buf, dest_rank):
        """Blocking send (ICommunicator::Send, include/comm/communicator.h:56-62)."""
        self.isend(buf, dest_rank).wait()

    def recv(self, buf, src_rank):
        """Blocking receive (ICommunicator::Recv); returns ``buf``."""
        self.irecv(buf, src_rank).wait()
        return buf

    def get_param(self, key):
        """A communicator parameter (RdcCommGetParam): "rdc_reduce_ring_mincount",
        "RDC_SCRATCH_BYTES", "RDC_TILE_BYTES", "RDC_NBLOCKS", "slot_bytes", "ranks_per_gpu"."""
        v = ctypes.c_uint64()
        check_call(_LIB.RdcCommGetParam(self.handle, key.encode("utf-8"), ctypes.byref(v)))
        return v.value

    def tune(self, mesh_s16=4, mesh_r16=8, max_blocks=0, tile_bytes=0):
        """Mesh role split (sixteenths of the grid), grid (0 = auto) and tile
        bytes (0 = auto) for the following collectives (RdcCommTune); every
        rank must pass the same values.  Results stay bit-identical."""
        check_call(_LIB.RdcCommTune(self.handle, int(mesh_s16), int(mesh_r16), int(max_blocks), int(tile_bytes)))

    def set_poison(self, on=True):
        """Debug mode (RdcCommSetPoison, RDC_POISON_SCRATCH): consumers overwrite
        every scratch range they finished reading with 0xFF bytes, so a read
        before the producer's next publish lands NaN / all-ones words."""
        check_call(_LIB.RdcCommSetPoison(self.handle, 1 if on else 0))

    def direct_release(self):
        """Close this rank's mappings of peer buffers of the direct schedule
        and turn the schedule off for this communicator (RdcCommDirectRelease):
        call on every rank to release peers' freed allocations that the
        mappings keep alive."""
        check_call(_LIB.RdcCommDirectRelease(self.handle))

    def autotune(self, nbytes, dtype=None, reps=3, stream=None):
        """Collective (every rank, same arguments): time the ring, the mesh and
        (where it fits) the one-shot, then the launch shapes of the fastest for allreduces of `nbytes`
        (mesh role split, grid, tiles per block), agree on the slowest rank's times and keep the
        fastest (RdcCommAutotune).  Returns {"chosen": {...} or None,
        "candidates": [{...,"ms"}]}; None chosen = the size takes the tree
        order and nothing changed.  Results stay bit-identical."""
        if dtype is None:
            dtype = 6  # mpi::kFloat32
        elif not isinstance(dtype, int):
            dtype = _dev.dtype_enum(dtype)
        if stream is None:
            import torch
            stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        room = 32
        cand = (TuneCand * room)()
        nc, best = ctypes.c_int(0), ctypes.c_int(-1)
        check_call(_LIB.RdcCommAutotune(self.handle, int(nbytes), int(dtype), int(reps), stream,
                                        ctypes.cast(cand, ctypes.c_void_p), room, ctypes.byref(nc),
                                        ctypes.byref(best)))

        def row(c):
            return {"schedule": {1: "ring", 2: "mesh", 3: "oneshot", 5: "mesh_pull", 6: "direct"}.get(c.algo, c.algo),
                    "split": [c.mesh_s16, c.mesh_r16], "grid": c.max_blocks or "auto",
                    "tiles_per_block": c.tiles_per_block or "auto", "ms": round(c.ms, 4),
                    "spread_ms": [round(c.ms_min, 4), round(c.ms_max, 4)]}
        rows = [row(cand[k]) for k in range(nc.value)]
        return {"chosen": rows[best.value] if best.value >= 0 else None, "candidates": rows}

    def check(self, stream=None):
        """Synchronise the stream and raise if a device-side wait failed."""
        if stream is None:
            import torch
            stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        check_call(_LIB.RdcCommCheck(self.handle, stream))

    def destroy(self):
        if self.handle:
            check_call(_LIB.RdcCommDestroy(self.handle))
            self.handle = ctypes.c_void_p()


def new_comm(name):
    """Create (collectively) the communicator ``name``."""
    comm = Comm()
    if isinstance(name, str):
        name = name.encode("utf-8")
    elif not isinstance(name, bytes):
        raise TypeError("name must be a string or bytearray")
    check_call(_LIB.RdcNewCommunicator(ctypes.byref(comm.handle), name))
    return comm


def get_comm(name="main"):
    """Existing communicator ``name`` ("main" is created on first use)."""
    comm = Comm()
    if isinstance(name, str):
        name = name.encode("utf-8")
    elif not isinstance(name, bytes):
        raise TypeError("name must be a string or bytearray")
    check_call(_LIB.RdcGetCommunicator(ctypes.byref(comm.handle), name))
    return comm


def create_group(ranks, name="", parent=None):
    """Sub-communicator over ``ranks`` (ranks of ``parent``, default "main";
    group rank i = ranks[i]), rdc::CreateGroup (include/api.h:124-125).
    Collective over every rank of the parent; returns None on non-members."""
    comm = Comm(own_handle=True)
    arr = (ctypes.c_int * len(ranks))(*[int(r) for r in ranks])
    check_call(_LIB.RdcCreateGroup(ctypes.byref(comm.handle), parent.handle if parent is not None else None, arr,
                                   len(ranks), name.encode("utf-8") if isinstance(name, str) else name))
    return comm if comm.handle else None


def init_group(devices, scratch_bytes=0):
    """Single-process group: one communicator per entry of ``devices``
    (device ids may repeat).  Returns the list of Comm, rank i = devices[i]."""
    n = len(devices)
    handles = (ctypes.c_void_p * n)()
    devs = (ctypes.c_int * n)(*devices)
    check_call(_LIB.RdcCommInitAll(handles, n, devs, scratch_bytes))
    return [Comm(ctypes.c_void_p(handles[i]), own_handle=True) for i in range(n)]
