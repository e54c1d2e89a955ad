"""Per-call timeline of a host allreduce from rocprofv3 CSV traces
(--kernel-trace --memory-copy-trace; tools/host_registered_trace.sh).

    python tools/copy_timeline.py <rocprofv3 output dir of one rank> <pieces per call>

HIP's device-to-host copies run as __amd_rocclr_copyBuffer kernels (no
memory-copy record): they are counted as the D2H direction.
Per call: wall (first H2D start -> last D2H end), the busy time of each copy
direction and of the kernels (union of intervals), and the tail after the
last H2D.
"""
import csv
import glob
import os
import sys


def load(d, pat):
    rows = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    d = sys.argv[1]
    copies = load(d, "*memory_copy_trace.csv")
    kernels = load(d, "*kernel_trace.csv")
    h2d, d2h = [], []
    for r in copies:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        kind = (r.get("Direction") or r.get("Operation") or r.get("Kind") or "")
        if "HOST_TO_DEVICE" in kind:
            h2d.append((s, e))
        elif "DEVICE_TO_HOST" in kind:
            d2h.append((s, e))
    # HIP moves device -> host with a copy kernel (__amd_rocclr_copyBuffer),
    # not an SDMA copy: those kernels are the D2H direction here
    ks = []
    for r in kernels:
        s, e, name = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "")
        if "rocclr_copyBuffer" in name:
            d2h.append((s, e))
        elif "rocclr_fill" not in name:
            ks.append((s, e, name))
    h2d.sort()
    d2h.sort()
    # every call moves the same K pieces each way: the i-th K H2D copies and
    # the i-th K D2H copies belong to call i
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    calls = [[h2d[i][0]] for i in range(0, len(h2d), K)]
    starts = [c[0] for c in calls] + [1 << 62]
    print("calls: %d   H2D copies %d   D2H copies %d   kernels %d" % (len(calls), len(h2d), len(d2h), len(ks)))
    for i in range(len(calls)):
        lo, hi = starts[i], starts[i + 1]
        ch = h2d[i * K:(i + 1) * K]
        cd = d2h[i * K:(i + 1) * K]
        ck = [(s, e) for s, e, _ in ks if lo <= s < hi]
        if not ch or not cd:
            continue
        end = max(e for _, e in cd)
        last_h = max(e for _, e in ch)
        print("call %d: wall %.3f ms | H2D n=%d busy %.3f ms (last ends at %.3f) | D2H n=%d busy %.3f ms "
              "(first starts at %.3f) | kernels n=%d busy %.3f ms | tail after last H2D %.3f ms"
              % (i, (end - lo) / 1e6, len(ch), union(ch) / 1e6, (last_h - lo) / 1e6, len(cd), union(cd) / 1e6,
                 (min(s for s, _ in cd) - lo) / 1e6, len(ck), union(ck) / 1e6, (end - last_h) / 1e6))


if __name__ == "__main__":
    main()
