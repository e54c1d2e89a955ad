"""rdc_amd — MI355X-native allreduce path for akkaze/rdc.

Drop-in for rdc's communicator surface (include/rdc.h, rdc/core.py,
rdc/comm.py): the ring reduce-scatter + allgather of
src/comm/communicator_collective.cc runs as gfx950 HIP kernels moving HBM
tiles between GPUs over xGMI peer-to-peer, bit-identical to the reference's
CPU ring.  Native code: librdc_amd.so (rdc_amd/csrc, C ABI in
include/rdc_amd.h); this package is the Python binding.
"""
from ._lib import LIB_PATH, RdcError, build  # noqa: F401
from .core import (DTYPE_ENUM__, Op, allgather, allreduce, allreduce_coalesced, barrier, broadcast, finalize, get_processor_name,  # noqa: F401
                   get_rank, get_world_size, init, is_distributed, recv, send, tracker_print)
from .comm import (ALGO_AUTO, ALGO_MESH, ALGO_ONESHOT, ALGO_RING, ALGO_TREE, WS_ERROR, WS_FINISHED,  # noqa: F401
                   WS_PENDING, Comm, WorkComp, create_group, get_comm, init_group, new_comm)
from .buffer import Buffer, PinnedArray, pinned_empty  # noqa: F401
from .device import dtype_enum, fill_, reduce_  # noqa: F401

__all__ = [
    "Op", "init", "finalize", "get_rank", "get_world_size", "is_distributed", "tracker_print",
    "get_processor_name", "barrier", "broadcast", "allreduce", "allreduce_coalesced", "allgather", "Comm", "new_comm", "get_comm",
    "Buffer", "PinnedArray", "pinned_empty", "WorkComp", "send", "recv",
    "init_group", "create_group", "reduce_", "fill_", "dtype_enum", "RdcError",
]
