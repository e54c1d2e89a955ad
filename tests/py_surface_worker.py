"""Worker for tests/test_gpu_entrypoints.py::test_python_surface_across_ranks.

The reference's Python harness shape (pytest/allreduce.py: float64
a[i] = rank + n + i, MAX then SUM, under `launcher_local -n N`) through
rdc_amd's Python surface, launched by `python -m rdc_amd.launcher -n N`,
plus the rest of rdc/core.py's and rdc/comm.py's contract at world size > 1:

* allreduce's copy rule (rdc/core.py:196-199: ``buf = data.ravel()``, copied
  when ``buf.base is data.base``): an owning 1-D array and an owning 2-D array
  are reduced in place (the result is a flat view of their memory); a 1-D view
  and a non-contiguous array come back as new arrays and stay untouched;
* ``prepare_fun(data)`` runs inside RdcAllreduce before the reduction
  (rdc/core.py:207-216) — it fills ``data``, so it reaches the reduction only
  when the buffer is ``data``'s memory (the reference's rule, kept);
* ``broadcast(obj, root)`` from a non-zero root (two RdcBroadcast calls,
  rdc/core.py:121-156), a dict and a 200 KB object;
* ``new_comm("x")`` / ``get_comm("x")`` (rdc/comm.py:83-112): a host
  allreduce on the handle, an isend/irecv ring of ndarrays (rdc/comm.py:46-80),
  and a device (ROCm tensor) allreduce;
* every dtype of DTYPE_ENUM__ (rdc/core.py:160-169) with SUM and MAX.
Integer results are exact known answers; float64 values of the form
rank + n + i are exact in any order.  Prints "rank R: python surface OK".
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import rdc_amd as rdc  # noqa: E402


def check(cond, what):
    if not cond:
        raise AssertionError("rank %d: %s" % (rdc.get_rank(), what))


def main():
    rdc.init()
    rank, world = rdc.get_rank(), rdc.get_world_size()
    check(world > 1, "world size %d" % world)

    # pytest/allreduce.py: n = 3 by default; also a buffer that is not tiny
    for n in (3, 1000, 300001):
        a = np.zeros(n)
        for i in range(n) if n <= 1000 else ():
            a[i] = rank + n + i
        if n > 1000:
            a[:] = rank + n + np.arange(n)
        idx = np.arange(n, dtype=np.float64)
        a = rdc.allreduce(a, rdc.Op.MAX)
        check(np.array_equal(a, (world - 1) + n + idx), "MAX n=%d" % n)
        a[:] = rank + n + idx
        a = rdc.allreduce(a, rdc.Op.SUM)
        check(np.array_equal(a, world * (n + idx) + world * (world - 1) // 2), "SUM n=%d" % n)

    # the copy rule: owning arrays in place, views / non-contiguous copied
    own = np.full(7, float(rank))
    res = rdc.allreduce(own, rdc.Op.SUM)
    want = float(world * (world - 1) // 2)
    check(np.shares_memory(res, own) and np.all(own == want) and np.all(res == want), "owning 1-D in place")
    two = np.arange(12, dtype=np.float64).reshape(3, 4) + rank
    res = rdc.allreduce(two, rdc.Op.MAX)
    check(res.shape == (12,) and np.shares_memory(res, two), "owning 2-D: flat view of its memory")
    check(np.array_equal(res, np.arange(12) + world - 1) and np.array_equal(two.ravel(), res), "2-D MAX")
    base = np.arange(10, dtype=np.float64) + rank
    view = base[2:]
    res = rdc.allreduce(view, rdc.Op.SUM)
    check(not np.shares_memory(res, base) and np.array_equal(view, np.arange(2, 10) + rank), "1-D view copied")
    check(np.array_equal(res, world * np.arange(2, 10) + world * (world - 1) // 2), "1-D view SUM")
    nc = (np.arange(24, dtype=np.float64).reshape(4, 6) + rank)[:, ::2]
    before = nc.copy()
    res = rdc.allreduce(nc, rdc.Op.MIN)
    check(not np.shares_memory(res, nc) and np.array_equal(nc, before), "non-contiguous copied")
    check(np.array_equal(res, (np.arange(24).reshape(4, 6)[:, ::2]).ravel()), "non-contiguous MIN")

    # prepare_fun fills data inside RdcAllreduce, before the reduction
    calls = []

    def prep(d):
        calls.append(d.shape)
        d[:] = rank + 5 + np.arange(d.size)

    lazy = np.zeros(5)
    res = rdc.allreduce(lazy, rdc.Op.SUM, prepare_fun=prep)
    check(calls == [(5,)], "prepare_fun called once with data: %r" % calls)
    check(np.array_equal(res, world * (5 + np.arange(5)) + world * (world - 1) // 2), "prepare_fun result")
    # on a view the buffer is a copy taken before prepare_fun (reference rule)
    holder = np.zeros(9)
    lazy_view = holder[4:]
    res = rdc.allreduce(lazy_view, rdc.Op.SUM, prepare_fun=prep)
    check(len(calls) == 2 and np.all(res == 0) and np.array_equal(lazy_view, rank + 5 + np.arange(5)),
          "prepare_fun on a view fills data, not the copied buffer")

    # every dtype of the reference's table, SUM and MAX
    for dt in (np.int8, np.uint8, np.int32, np.uint32, np.int64, np.uint64, np.float32, np.float64):
        x = (np.arange(33) % 5 + rank).astype(dt)
        s = rdc.allreduce(x, rdc.Op.SUM)
        check(s.dtype == dt and np.array_equal(s, (world * (np.arange(33) % 5) + world * (world - 1) // 2)
                                               .astype(dt)), "SUM %s" % np.dtype(dt).name)
        x = (np.arange(33) % 5 + rank).astype(dt)
        m = rdc.allreduce(x, rdc.Op.MAX)
        check(np.array_equal(m, (np.arange(33) % 5 + world - 1).astype(dt)), "MAX %s" % np.dtype(dt).name)
    bo = rdc.allreduce(np.array([1 << rank, 0], dtype=np.int32), rdc.Op.BITOR)
    check(bo[0] == (1 << world) - 1, "BITOR")

    # pickled broadcast from a non-zero root (and back from root 0)
    root = 1
    obj = {"from": rank, "payload": list(range(10)), "name": "rdc"} if rank == root else None
    got = rdc.broadcast(obj, root)
    check(got == {"from": root, "payload": list(range(10)), "name": "rdc"}, "broadcast dict from root 1")
    big = (b"x" * 200000 + bytes([rank])) if rank == 0 else None
    got = rdc.broadcast(big, 0)
    check(got == b"x" * 200000 + b"\x00", "broadcast 200 KB from root 0")
    tail = rdc.broadcast(("tail", rank) if rank == world - 1 else None, world - 1)
    check(tail == ("tail", world - 1), "broadcast tuple from the last rank")

    # named communicator handles (rdc/comm.py:83-112)
    cx = rdc.new_comm("x")
    cx2 = rdc.get_comm("x")
    check(cx.handle.value == cx2.handle.value, "get_comm returns new_comm's handle")
    h = np.full(100, float(rank + 1))
    r = cx.allreduce(h, rdc.Op.SUM)
    check(np.all(r == world * (world + 1) / 2), "host allreduce on comm x")
    # isend / irecv ring of ndarrays on x
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    out_msg = np.arange(64, dtype=np.float32) + rank
    in_msg = np.zeros(64, dtype=np.float32)
    ws = cx.isend(out_msg, nxt)
    wr = cx.irecv(in_msg, prv)
    check(ws.wait() == 0 and wr.wait() == 0, "isend/irecv completion")
    check(np.array_equal(in_msg, np.arange(64, dtype=np.float32) + prv), "irecv payload from the previous rank")
    # a device allreduce on x (ROCm tensor, stream-ordered, in place)
    import torch
    t = torch.full((4096,), float(rank), dtype=torch.float32, device="cuda")
    cx.allreduce(t, rdc.Op.SUM)
    cx.check()
    check(bool(torch.all(t == float(world * (world - 1) // 2))), "device allreduce on comm x")
    # and through rdc.allreduce on the main communicator
    t2 = torch.full((1000,), float(rank), dtype=torch.float64, device="cuda")
    rdc.allreduce(t2, rdc.Op.MAX)
    torch.cuda.synchronize()
    check(bool(torch.all(t2 == float(world - 1))), "device allreduce via rdc.allreduce")

    # a registered host array (rdc_amd.pinned_empty): reduced in place, and the
    # library DMAs its pages directly (host_registered_calls counts the calls)
    import ctypes
    from rdc_amd._lib import _LIB, check_call
    hm = rdc.get_comm("main").handle
    reg0, reg1 = ctypes.c_uint64(), ctypes.c_uint64()
    check_call(_LIB.RdcCommGetParam(hm, b"host_registered_calls", ctypes.byref(reg0)))
    for count in (1 << 20, (6 << 20) + 3):  # one 4 MiB piece; a 24 MiB + 12 B pipeline
        pa = rdc.pinned_empty(count, np.float32)
        pa[:] = rank + np.arange(count) % 7
        res = rdc.allreduce(pa, rdc.Op.SUM)
        want = (world * (np.arange(count) % 7) + world * (world - 1) // 2).astype(np.float32)
        check(np.shares_memory(res, pa) and np.array_equal(pa, want), "pinned_empty SUM count=%d" % count)
        del res, pa
    check_call(_LIB.RdcCommGetParam(hm, b"host_registered_calls", ctypes.byref(reg1)))
    check(reg1.value - reg0.value == 2, "registered host calls: %d" % (reg1.value - reg0.value))

    rdc.finalize()
    print("rank %d: python surface OK" % rank, flush=True)


if __name__ == "__main__":
    main()
