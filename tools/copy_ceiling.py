#!/usr/bin/env python
"""HBM ceilings of plain streaming kernels on this GPU, for reading the
shared-HBM fractions of the N > 1 rehearsals: torch's device copy (S read +
S written, the direct schedule's 1:1 mix), a 2-read-1-write add (k_reduce's
mix) and a read-only sum.  1 GiB fp32 per operand, HIP events, median of
20 launches.

    python tools/copy_ceiling.py [MiB]
"""
import json
import sys

import torch


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    n = (mib << 20) // 4
    a = torch.rand(n, device="cuda")
    b = torch.rand(n, device="cuda")
    c = torch.empty(n, device="cuda")
    S = n * 4

    def timed(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        return ts[len(ts) // 2]

    out = {}
    for name, fn, moved in (("copy (1 read : 1 write)", lambda: c.copy_(a), 2 * S),
                            ("add (2 reads : 1 write)", lambda: torch.add(a, b, out=c), 3 * S),
                            ("sum (read only)", lambda: a.sum(), S)):
        ms = timed(fn)
        out[name] = {"ms": round(ms, 4), "TBps": round(moved / ms / 1e9, 3), "frac_of_8TBps": round(moved / ms / 8e9, 4)}
    print(json.dumps({"bytes_per_operand": S, "ceilings": out}), flush=True)


if __name__ == "__main__":
    main()
