"""Loader of the native library librdc_amd.so (built in-tree for gfx950).

There is no CPU fallback: if the library is missing, importing the package
fails loudly.  Build it with ``make -C rdc_amd/csrc`` (or
``__graft_entry__.build()``).
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librdc_amd.so")


def build(jobs=4):
    """Compile librdc_amd.so with hipcc --offload-arch=gfx950."""
    subprocess.check_call(["make", "-s", "-j%d" % jobs, "-C", os.path.join(HERE, "csrc")])


def _load():
    # torch wheels bundle their own libamdhip64 (soname libamdhip64.so.7, but
    # linked by the name libamdhip64.so).  Import torch first so this library
    # binds to the runtime torch already loaded; loading ours first would put
    # two HIP runtimes in one process.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "rdc_amd: native library %s is missing; build it with `make -C rdc_amd/csrc` "
            "(the MI355X path has no CPU fallback)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, i, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
    pvp = ctypes.POINTER(ctypes.c_void_p)
    sig = {
        "RdcInit": (i, [i, ctypes.POINTER(ctypes.c_char_p)]),
        "RdcFinalize": (i, []),
        "RdcGetRank": (i, []),
        "RdcGetWorldSize": (i, []),
        "RdcIsDistributed": (i, []),
        "RdcTrackerPrint": (i, [ctypes.c_char_p]),
        "RdcGetProcessorName": (i, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_ulong), ctypes.c_ulong]),
        "RdcBarrier": (i, []),
        "RdcAllreduce": (i, [vp, sz, i, i, vp, vp]),
        "RdcBroadcast": (i, [vp, ctypes.c_ulong, i]),
        "RdcAllreduceOn": (i, [vp, vp, sz, i, i]),
        "RdcAllgather": (i, [pvp, ctypes.POINTER(ctypes.c_size_t)]),
        "RdcAllgatherOn": (i, [vp, pvp, ctypes.POINTER(ctypes.c_size_t)]),
        "RdcCommAllgather": (i, [vp, pvp, ctypes.POINTER(ctypes.c_size_t), vp]),
        "RdcBroadcastOn": (i, [vp, vp, sz, i]),
        "RdcNewCommunicator": (i, [pvp, ctypes.c_char_p]),
        "RdcGetCommunicator": (i, [pvp, ctypes.c_char_p]),
        "RdcCreateGroup": (i, [pvp, vp, ctypes.POINTER(ctypes.c_int), i, ctypes.c_char_p]),
        "RdcCommGetParam": (i, [vp, ctypes.c_char_p, ctypes.POINTER(u64)]),
        "RdcPlanTree": (i, [i, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
        "RdcPlanResidentGrid": (i, [i, i, i, i]),
        "RdcPlanResidentGridXcd": (i, [i, i, i, i, i, i]),
        "RdcCommAllreduce": (i, [vp, vp, sz, i, i, vp]),
        "RdcCommAllreduceEx": (i, [vp, vp, sz, i, i, i, vp]),
        "RdcCommBroadcast": (i, [vp, vp, sz, i, vp]),
        "RdcCommCheck": (i, [vp, vp]),
        "RdcCommProbe": (i, [vp, i, sz, i, vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(sz)]),
        "RdcCommTraceNext": (i, [vp, vp, sz]),
        "RdcCommTune": (i, [vp, i, i, i, sz]),
        "RdcCommSetPoison": (i, [vp, i]),
        "RdcCommDirectRelease": (i, [vp]),
        "RdcCommAutotune": (i, [vp, sz, i, i, vp, vp, i, ctypes.POINTER(i), ctypes.POINTER(i)]),
        "RdcCommLastLaunch": (i, [vp, ctypes.POINTER(u64)]),
        "RdcCommLaunchCounter": (i, [vp, ctypes.POINTER(u64)]),
        "RdcCommSetLaunchCounter": (i, [vp, u64]),
        "RdcCommRank": (i, [vp]),
        "RdcCommSize": (i, [vp]),
        "RdcCommDevice": (i, [vp]),
        "RdcCommAllocKind": (i, [vp]),
        "RdcCommInitAll": (i, [pvp, i, ctypes.POINTER(ctypes.c_int), sz]),
        "RdcCommDestroy": (i, [vp]),
        "RdcReduce": (i, [vp, vp, sz, i, i, vp]),
        "RdcFill": (i, [vp, sz, i, u64, i, vp]),
        "RdcMemcpy": (i, [vp, vp, sz]),
        "RdcPlanLayout": (i, [i, sz, ctypes.POINTER(u64)]),
        "RdcPlanHbmBytes": (i, [i, sz, i, i, ctypes.POINTER(u64)]),
        "RdcPlanDirectItems": (i, [i, i, ctypes.POINTER(sz), i, i, u64, ctypes.POINTER(u64), i, ctypes.POINTER(i)]),
        "RdcPlanHostPieceRanges": (i, [i, sz, i, u64, u64, i, ctypes.POINTER(u64), ctypes.POINTER(u64),
                                       ctypes.POINTER(ctypes.c_int)]),
        "RdcPlanAutoAlgo": (i, [i, sz, sz, sz]),
        "RdcPlanDirectAuto": (i, [i, sz, sz, sz, u64]),
        "RdcPlanHostPieces": (i, [sz, ctypes.POINTER(ctypes.c_uint64), i, ctypes.POINTER(i)]),
        "RdcPlanAllreduce": (i, [i, sz, i, sz, i, sz, i, ctypes.POINTER(u64), i, ctypes.POINTER(ctypes.c_int)]),
        "RdcAllreduceCoalesced": (i, [pvp, ctypes.POINTER(sz), i, i, i]),
        "RdcAllreduceCoalescedOn": (i, [vp, pvp, ctypes.POINTER(sz), i, i, i]),
        "RdcCommAllreduceCoalesced": (i, [vp, pvp, ctypes.POINTER(sz), i, i, i, i, vp]),
        "RdcPlanCoalesced": (i, [i, ctypes.POINTER(sz), i, i, ctypes.POINTER(u64), ctypes.POINTER(u64), i,
                                 ctypes.POINTER(ctypes.c_int)]),
        "RdcPlanFuseGroups": (i, [ctypes.POINTER(sz), i, i, sz, ctypes.POINTER(ctypes.c_int), i,
                                  ctypes.POINTER(ctypes.c_int)]),
        "RdcNewBuffer": (i, [pvp, vp, sz, i]),
        "RdcDelBuffer": (i, [vp]),
        "RdcISend": (i, [pvp, vp, vp, i]),
        "RdcIRecv": (vp, [vp, vp, i]),
        "RdcWorkCompletionWait": (i, [vp]),
        "RdcWorkCompletionStatus": (i, [vp]),
        "RdcWorkCompletionError": (ctypes.c_char_p, [vp]),
        "RdcDelWorkCompletion": (i, [vp]),
        "RdcSend": (i, [vp, sz, i]),
        "RdcRecv": (i, [vp, sz, i]),
        "RdcCommISend": (i, [pvp, vp, vp, sz, i, vp]),
        "RdcCommIRecv": (i, [pvp, vp, vp, sz, i, vp]),
        "RdcSetParam": (i, [ctypes.c_char_p, ctypes.c_char_p]),
        "RdcGetLastError": (ctypes.c_char_p, []),
        "RdcVersion": (ctypes.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


_LIB = _load()


class RdcError(RuntimeError):
    pass


def check_call(rc):
    """Raise RdcError with the library's message when rc != 0."""
    if rc != 0:
        raise RdcError(_LIB.RdcGetLastError().decode("utf-8", "replace"))
    return rc
