"""Kernel stats (the columns of rocprofv3's kernel_stats.csv) from a rocprofv3 SQLite output
(run_results.db), for runs made without --output-format csv.
usage: python tools/rocpd_stats.py run_results.db out.csv"""
import csv
import math
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    agg = {}
    for name, d in c.execute("select name, duration from kernels"):
        agg.setdefault(name, []).append(float(d))
    tot = sum(sum(v) for v in agg.values())
    rows = []
    for name, v in agg.items():
        n, s = len(v), sum(v)
        mean = s / n
        sd = math.sqrt(sum((x - mean) ** 2 for x in v) / n)
        rows.append([name, n, int(s), mean, 100.0 * s / tot, int(min(v)), int(max(v)), sd])
    rows.sort(key=lambda r: -r[2])
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        w.writerows(rows)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
