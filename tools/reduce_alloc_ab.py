"""N=1 reduce kernel (RdcReduce, 1 GiB fp32) timed on differently allocated
buffers, alternating, in one process: torch.empty per buffer; halves of one
2 GiB torch.empty; hipMalloc'd through the HIP runtime directly.  Events
over 30 launches after 5 warm-ups, best of 3 rounds each.
    python tools/reduce_alloc_ab.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from rdc_amd._lib import _LIB, check_call
    import rdc_amd
    S = 1 << 30
    n = S // 4
    hip = ctypes.CDLL("libamdhip64.so")
    stream = torch.cuda.current_stream()
    sp = ctypes.c_void_p(stream.cuda_stream)

    def hip_buf():
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(S)) == 0
        return p.value

    t_d, t_s = torch.empty(n, device="cuda"), torch.empty(n, device="cuda")
    big = torch.empty(2 * n, device="cuda")
    h_d, h_s = hip_buf(), hip_buf()
    cases = {"torch_two": (t_d.data_ptr(), t_s.data_ptr()),
             "torch_one_2GiB": (big.data_ptr(), big.data_ptr() + S),
             "hipMalloc_two": (h_d, h_s)}
    for d, s in cases.values():
        check_call(_LIB.RdcFill(ctypes.c_void_p(d), n, 6, 0x5EED0000, 0, sp))
        check_call(_LIB.RdcFill(ctypes.c_void_p(s), n, 6, 0x5EED0000, 1, sp))
    torch.cuda.synchronize()
    res = {k: [] for k in cases}
    for _ in range(3):
        for k, (d, s) in cases.items():
            for _ in range(5):
                check_call(_LIB.RdcReduce(ctypes.c_void_p(d), ctypes.c_void_p(s), n, 6, 2, sp))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(30):
                check_call(_LIB.RdcReduce(ctypes.c_void_p(d), ctypes.c_void_p(s), n, 6, 2, sp))
            e1.record(stream)
            torch.cuda.synchronize()
            res[k].append(round(e0.elapsed_time(e1) / 30, 4))
    out = {k: {"ms": v, "best_TBps": round(3 * S / (min(v) * 1e-3) / 1e12, 3),
               "addr_mod_2MiB": [hex(x % (2 << 20)) for x in cases[k]]} for k, v in res.items()}
    print(json.dumps(out))
    del rdc_amd


if __name__ == "__main__":
    main()
