#!/usr/bin/env python
"""Per-kernel statistics from a rocprofv3 rocpd database (ROCm 7 writes `<name>_results.db` by
default), in the column layout of rocprofv3's `--stats` kernel_stats.csv.

    python tools/rocpd_stats.py gpurun_out/prof12/run_results.db > profiles/r01_c_kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main(path, out=sys.stdout):
    con = sqlite3.connect(path)
    rows = con.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
        "avg(duration*duration) from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(out, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for name, n, tot, avg, mn, mx, sq in rows:
        std = max(sq - avg * avg, 0.0) ** 0.5
        w.writerow([name, n, int(tot), round(avg, 3), round(100.0 * tot / total, 2), int(mn), int(mx), round(std, 3)])


if __name__ == "__main__":
    main(sys.argv[1])
