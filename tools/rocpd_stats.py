#!/usr/bin/env python
"""rocprofv3's rocpd database (its default output on ROCm 7.2) -> the
kernel_stats.csv summary `rocprofv3 --stats` writes in csv mode: one row per
kernel name with calls, total / average / min / max duration (ns) and its
share of the total, sorted by total time.

    python tools/rocpd_stats.py RESULTS.db OUT.csv
"""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, n, tot, avg, mn, mx in rows:
            w.writerow([name, n, int(tot), round(avg, 1), round(100.0 * tot / total, 2), int(mn), int(mx)])


if __name__ == "__main__":
    main()
