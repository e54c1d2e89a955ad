"""Cross-rank timeline of the host path at n = 2 (tools/host_registered_trace.sh output; TRB = its directory):
the union of both ranks' H2D / D2H / allreduce intervals per call and the last call's event sequence."""
import sys
sys.path.insert(0, "tools")
import copy_timeline as T
import os
base = os.environ.get("TRB", "gpurun_out/host_registered_trace/")
K = 13
for pin in ("pin1", "pin0"):
    per = []
    for r in (0, 1):
        d = base + "%s_r%d" % (pin, r)
        copies = T.load(d, "*memory_copy_trace.csv"); kernels = T.load(d, "*kernel_trace.csv")
        h2d = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in copies if "HOST_TO_DEVICE" in x["Direction"])
        d2h = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in kernels if "copyBuffer" in x["Kernel_Name"])
        ar = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in kernels if "rdc_amd" in x["Kernel_Name"])
        per.append((h2d, d2h, ar))
    for i in range(1, 7):
        H = per[0][0][i*K:(i+1)*K] + per[1][0][i*K:(i+1)*K]
        D = per[0][1][i*K:(i+1)*K] + per[1][1][i*K:(i+1)*K]
        A = per[0][2][i*K:(i+1)*K] + per[1][2][i*K:(i+1)*K]
        t0 = min(s for s, _ in H); t1 = max(e for _, e in D)
        print("%s call %d: wall %.3f | H2D union %.3f (span %.3f) | D2H union %.3f | AR union %.3f | per-piece H2D ms r0: %s" % (
            pin, i, (t1-t0)/1e6, T.union(H)/1e6, (max(e for _, e in H)-t0)/1e6, T.union(D)/1e6, T.union(A)/1e6,
            " ".join("%.2f" % ((e-s)/1e6) for s, e in per[0][0][i*K:(i+1)*K])))
        if i == 6:
            ev = sorted([(s, "H%d" % r) for r in (0, 1) for s, e in per[r][0][i*K:(i+1)*K]] + [(e, "h%d" % r) for r in (0, 1) for s, e in per[r][0][i*K:(i+1)*K]] +
                        [(s, "A%d" % r) for r in (0, 1) for s, e in per[r][2][i*K:(i+1)*K]] + [(e, "a%d" % r) for r in (0, 1) for s, e in per[r][2][i*K:(i+1)*K]] +
                        [(s, "D%d" % r) for r in (0, 1) for s, e in per[r][1][i*K:(i+1)*K]] + [(e, "d%d" % r) for r in (0, 1) for s, e in per[r][1][i*K:(i+1)*K]])
            print(" ".join("%s@%.2f" % (n, (t - t0)/1e6) for t, n in ev))
