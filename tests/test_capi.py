"""CPU: the C-ABI library loads, exports every entry point include/rdc_amd.h
declares, and behaves like the reference's API where no GPU is needed
(world size 1, parameter parsing, error reporting, host planning)."""
import ctypes
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "rdc_amd.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(Rdc\w+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from rdc_amd._lib import LIB_PATH, _LIB
    syms = declared_symbols()
    assert len(syms) >= 25
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB_PATH]).decode()
    exported = set(re.findall(r" T (Rdc\w+)", out))
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    for s in syms:  # and the Python binding knows each signature
        assert getattr(_LIB, s).restype is not None or s in ()


def test_reference_python_callers_are_covered():
    """Every _LIB.Rdc* name the reference's Python package calls for this path
    exists in the C ABI (rdc/core.py, rdc/comm.py)."""
    needed = {"RdcInit", "RdcFinalize", "RdcGetRank", "RdcGetWorldSize", "RdcTrackerPrint",
              "RdcGetProcessorName", "RdcBroadcast", "RdcAllreduce", "RdcNewCommunicator", "RdcGetCommunicator",
              # rdc/comm.py:25-76 (point-to-point) and rdc/buffer.py:34-38
              "RdcISend", "RdcIRecv", "RdcWorkCompletionWait", "RdcWorkCompletionStatus", "RdcDelWorkCompletion",
              "RdcNewBuffer", "RdcDelBuffer"}
    ref = "/root/reference/rdc"
    if os.path.isdir(ref):  # read as text only
        called = set()
        for f in ("core.py", "comm.py", "buffer.py"):
            called |= set(re.findall(r"_LIB\.(Rdc\w+)", open(os.path.join(ref, f)).read()))
        # checkpointing (RdcCheckPoint / RdcLoadCheckPoint / RdcVersionNumber) and
        # RdcEnvGetIntEnv are outside the allreduce path
        out_of_scope = {"RdcCheckPoint", "RdcLoadCheckPoint", "RdcVersionNumber", "RdcEnvGetIntEnv"}
        assert called - out_of_scope <= set(declared_symbols())
    assert needed <= set(declared_symbols())


def test_buffer_and_workcomp_host_side():
    """rdc.Buffer over ndarray / bytes / bytearray / addr+size (rdc/buffer.py,
    pytest/buffer.py, pytest/comm.py) and the WorkComp status constants; no GPU."""
    out = run_py(
        "import numpy as np, ctypes, rdc_amd\n"
        "b = rdc_amd.Buffer(b'hello'); assert b.bytes() == b'hello' and len(b) == 5\n"
        "a = np.random.random_sample(200).astype(np.float32); B = rdc_amd.Buffer(a)\n"
        "assert np.array_equal(np.array(B), a) and B.size == 800\n"
        "ba = bytearray(b'abc'); C = rdc_amd.Buffer(ba); ba[0] = 120; assert C.bytes() == b'xbc'\n"
        "D = rdc_amd.Buffer(addr=a.ctypes.data, size=8); assert np.array_equal(D.to_numpy().view(np.float32), a[:2])\n"
        "E = rdc_amd.Buffer(b'')\n"
        "assert (rdc_amd.WS_PENDING, rdc_amd.WS_FINISHED, rdc_amd.WS_ERROR) == (2, 8, 64)\n"
        "from rdc_amd._lib import _LIB\n"
        "assert _LIB.RdcWorkCompletionStatus(None) == 64\n"
        "assert _LIB.RdcIRecv(None, B.handle, 1) is None and b'null communicator' in _LIB.RdcGetLastError()\n"
        "print('ok')\n")
    assert "ok" in out


def run_py(code, env=None):
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=e, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    return p.stdout


def test_world_size_one_semantics():
    out = run_py(r'''
import numpy as np, rdc_amd as r
r.init(["prog", "rdc_reduce_ring_mincount=4K"])
assert r.get_rank() == 0 and r.get_world_size() == 1 and not r.is_distributed()
a = np.arange(6, dtype=np.float32).reshape(2, 3)
called = []
b = r.allreduce(a, r.Op.SUM, prepare_fun=lambda d: called.append(d.shape))
assert b.shape == (6,) and np.array_equal(b, a.ravel()) and called == [(2, 3)]
assert r.broadcast({"k": [1, 2]}, 0) == {"k": [1, 2]}
r.tracker_print("hello")
assert len(r.get_processor_name()) > 0
r.barrier()
r.finalize()
print("OK")
''')
    assert "OK" in out


def test_errors_are_reported_not_fatal():
    out = run_py(r'''
import ctypes, numpy as np, rdc_amd as r
from rdc_amd._lib import _LIB
assert _LIB.RdcAllreduce(None, 4, 6, 2, None, None) != 0
assert b"RdcInit" in _LIB.RdcGetLastError()
r.init([])
buf = np.zeros(4, dtype=np.float32)
p = buf.ctypes.data_as(ctypes.c_void_p)
assert _LIB.RdcAllreduce(p, 4, 99, 2, None, None) != 0 and b"dtype" in _LIB.RdcGetLastError()
assert _LIB.RdcAllreduce(p, 4, 6, 3, None, None) != 0 and b"BITOR" in _LIB.RdcGetLastError()
assert _LIB.RdcAllreduce(p, 4, 6, 7, None, None) != 0 and b"op" in _LIB.RdcGetLastError()
assert _LIB.RdcSetParam(b"RDC_SCRATCH_BYTES", b"12Q") != 0
assert _LIB.RdcSetParam(b"RDC_SCRATCH_BYTES", b"256M") == 0
assert _LIB.RdcBroadcast(p, 16, 1) != 0 and b"root" in _LIB.RdcGetLastError()
h = ctypes.c_void_p()
assert _LIB.RdcGetCommunicator(ctypes.byref(h), b"nope") != 0 and b"nope" in _LIB.RdcGetLastError()
assert _LIB.RdcCommAllreduce(None, p, 4, 6, 2, None) != 0
print("OK")
''')
    assert "OK" in out


def test_bad_rank_rejected():
    out = run_py(r'''
import rdc_amd as r
from rdc_amd._lib import RdcError
try:
    r.init(["RDC_RANK=3", "RDC_WORLD_SIZE=2"])
except RdcError as e:
    assert "bad rank" in str(e); print("OK")
''')
    assert "OK" in out


def test_reference_enum_values():
    import rdc_amd
    assert [int(o) for o in (rdc_amd.Op.MAX, rdc_amd.Op.MIN, rdc_amd.Op.SUM, rdc_amd.Op.BITOR)] == [0, 1, 2, 3]
    d = rdc_amd.DTYPE_ENUM__
    assert [d[np.dtype(t)] for t in ("int8", "uint8", "int32", "uint32", "int64", "uint64", "float32", "float64")] \
        == list(range(8))


def test_cpp_header_compiles():
    """include/rdc.h (the reference's C++ surface over the C ABI) builds and links."""
    src = os.path.join(ROOT, "tests", "cpp", "known_answer.cc")
    exe = os.path.join("/tmp", "rdc_known_answer_%d" % os.getpid())
    subprocess.check_call(["g++", "-std=c++11", "-O1", "-I", os.path.join(ROOT, "include"), src, "-o", exe,
                           "-L", os.path.join(ROOT, "rdc_amd"), "-lrdc_amd",
                           "-Wl,-rpath," + os.path.join(ROOT, "rdc_amd")])
    # world size 1 runs without a GPU: Allreduce is a no-op, checks hold
    env = dict(os.environ, RDC_WORLD_SIZE="1")
    p = subprocess.run([exe, "5"], env=env, capture_output=True, text=True, timeout=60)
    os.unlink(exe)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "known-answer OK" in p.stdout


def test_header_op_reducer_matches_reference(tmp_path):
    """include/rdc.h's op::Reducer<OP,DType> and op::X::Reduce (mpi.h:84-120)
    fold the same bytes as the reference's own header compiled (oracle/_ref
    ref_reducer) for every (dtype, op) the reference defines, on random
    values plus the edge cases: NaN on either side, signed zeros, +-inf,
    integer overflow (wraps) and extremes."""
    from oracle import oracle as O
    if not O.ref_available():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    so = str(tmp_path / "libop_reducer_shim.so")
    subprocess.check_call(["g++", "-std=c++11", "-O2", "-shared", "-fPIC", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "op_reducer_shim.cc"), "-o", so,
                           "-L", os.path.join(ROOT, "rdc_amd"), "-lrdc_amd", "-Wl,-rpath," + os.path.join(ROOT, "rdc_amd")])
    H = ctypes.CDLL(so)
    vp = ctypes.c_void_p
    H.hdr_reducer.argtypes = [vp, vp, ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
    kt = (ctypes.c_int * 4)()
    H.hdr_op_types(kt)
    assert list(kt) == [O.OP_MAX, O.OP_MIN, O.OP_SUM, O.OP_BITOR]
    R = O.ref()
    rng = np.random.default_rng(41)
    n = 4099
    checked = 0
    for dt in range(10):
        npd = O.NP_DTYPE[dt]
        ops = (O.OP_MAX, O.OP_MIN, O.OP_SUM) + (() if dt in (O.DT_FLOAT32, O.DT_FLOAT64) else (O.OP_BITOR,))
        for op in ops:
            if dt in (O.DT_FLOAT32, O.DT_FLOAT64):
                s = (rng.standard_normal(n) * 1e3).astype(npd)
                d = (rng.standard_normal(n) * 1e3).astype(npd)
                special = np.array([np.nan, 1.0, -0.0, 0.0, np.inf, -np.inf, np.nan, 3.0], dtype=npd)
                s[:8] = special
                d[:8] = special[::-1]
            else:
                info = np.iinfo(npd)
                s = rng.integers(info.min, info.max, n, dtype=npd, endpoint=True)
                d = rng.integers(info.min, info.max, n, dtype=npd, endpoint=True)
                s[:4] = [info.max, info.min, info.max, 0]
                d[:4] = [info.max, info.min, info.min, info.max]
            want, got = d.copy(), d.copy()
            assert R.ref_reducer(s.ctypes.data, want.ctypes.data, n, dt, op) == 0
            assert H.hdr_reducer(s.ctypes.data, got.ctypes.data, n, dt, op) == 0
            assert got.tobytes() == want.tobytes(), (dt, op)
            checked += 1
    assert checked == 38  # 8 integer types x 4 ops + 2 float types x 3 ops


def test_pinned_empty_is_reduced_in_place():
    """rdc_amd.pinned_empty: page-aligned host memory behind a pinned Buffer
    (registration itself needs a GPU); allreduce's copy rule (rdc/core.py:
    196-199) keeps it in place, so the registered pages are what the library
    DMAs; views keep the registration alive."""
    import numpy as np
    import rdc_amd
    a = rdc_amd.pinned_empty((3, 5), np.float64)
    assert isinstance(a, rdc_amd.PinnedArray) and a.shape == (3, 5) and a.dtype == np.float64
    assert a.ctypes.data % 4096 == 0 and np.all(a == 0)
    flat = a.ravel()
    assert flat.base is not a.base and np.shares_memory(flat, a)  # not copied by host_allreduce
    assert flat._rdc_buf is a._rdc_buf is not None and a._rdc_buf.pinned
