"""rdc Buffer — rdc/buffer.py (and the pybind ``rdc.Buffer`` of
src/frontend/rdc.cc:17-78) over librdc_amd.so's ``RdcNewBuffer``.

A Buffer is a view (address, size) of memory the caller owns: a numpy array,
a ``bytes`` / ``bytearray`` (pytest/comm.py, pytest/buffer.py), a contiguous
ROCm tensor, or a raw ``addr=``/``size=`` pair.  ``bytes`` are immutable in
Python, so a Buffer made from them holds a private writable copy (what a
receive lands in; read it back with ``.bytes()``).
"""
import ctypes

import numpy as np

from ._lib import _LIB, check_call


class Buffer(object):
    __slots__ = ("handle", "pinned", "addr", "size", "dtype", "_keep", "_np")

    def __init__(self, buf=None, addr=None, size=None, pinned=False):
        self.handle = ctypes.c_void_p()
        self.pinned = bool(pinned)
        self.dtype = np.dtype(np.uint8)
        self._keep = None
        self._np = None
        if buf is not None:
            if isinstance(buf, np.ndarray):
                if not buf.flags["C_CONTIGUOUS"]:
                    raise ValueError("rdc_amd: Buffer needs a C-contiguous array")
                self._keep = buf
                self._np = buf
                self.addr = buf.ctypes.data
                self.size = buf.size * buf.itemsize
                self.dtype = buf.dtype
            elif isinstance(buf, (bytes, bytearray)):
                if isinstance(buf, bytes):
                    buf = bytearray(buf)  # writable private copy
                self._keep = buf
                self._np = np.frombuffer(buf, dtype=np.uint8) if len(buf) else np.zeros(0, np.uint8)
                self.addr = self._np.ctypes.data if len(buf) else 0
                self.size = len(buf)
            elif hasattr(buf, "data_ptr") and hasattr(buf, "is_contiguous"):  # torch tensor
                if not buf.is_contiguous():
                    raise ValueError("rdc_amd: Buffer needs a contiguous tensor")
                self._keep = buf
                self.addr = buf.data_ptr()
                self.size = buf.numel() * buf.element_size()
            else:
                raise TypeError("unsupport type for buffer")
        elif addr is not None:
            if size is None:
                raise ValueError("size must accompany with addr")
            self.addr = int(addr.value if isinstance(addr, ctypes.c_void_p) else addr)
            self.size = int(size)
        else:
            raise TypeError("Buffer needs buf= or addr=/size=")
        check_call(_LIB.RdcNewBuffer(ctypes.byref(self.handle), ctypes.c_void_p(self.addr), self.size,
                                     1 if self.pinned else 0))

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            _LIB.RdcDelBuffer(h)
            self.handle = ctypes.c_void_p()

    def __len__(self):
        return self.size

    def to_numpy(self):
        """The host array the buffer views (a copy for device memory)."""
        if self._np is not None:
            return self._np
        if self._keep is not None and hasattr(self._keep, "cpu"):
            return self._keep.cpu().numpy()
        return np.ctypeslib.as_array((ctypes.c_uint8 * self.size).from_address(self.addr)).copy()

    def __array__(self, dtype=None, copy=None):
        a = self.to_numpy()
        return a.astype(dtype) if dtype is not None else a

    def bytes(self):
        return self.to_numpy().tobytes()


class PinnedArray(np.ndarray):
    """An ndarray over page-aligned host memory registered with the HIP
    runtime for as long as the array or any view of it lives (see
    ``pinned_empty``)."""

    def __array_finalize__(self, obj):
        self._rdc_buf = getattr(obj, "_rdc_buf", None)


def pinned_empty(shape, dtype=np.float32):
    """A host array whose memory is an anonymous mmap registered through
    ``RdcNewBuffer(..., pinned=1)`` (the reference's pinned Buffer,
    include/transport/buffer.h:61,91).  ``allreduce`` reduces such an array in
    place (``ravel`` gives a view of its memory, rdc/core.py:196-199), and the
    library DMAs it straight from and into these pages instead of copying it
    through pinned staging memory.  The registration ends with the last
    reference to the array or its views."""
    import mmap
    dtype = np.dtype(dtype)
    count = int(np.prod(shape, dtype=np.int64)) if np.ndim(shape) else int(shape)
    nbytes = count * dtype.itemsize
    span = max(1, (nbytes + mmap.PAGESIZE - 1) // mmap.PAGESIZE) * mmap.PAGESIZE
    mem = np.frombuffer(mmap.mmap(-1, span), dtype=np.uint8)
    mem[:] = 0  # fault every page in before it is pinned
    buf = Buffer(mem, pinned=True)
    arr = mem[:nbytes].view(dtype).reshape(shape).view(PinnedArray)
    arr._rdc_buf = buf
    return arr
