#!/usr/bin/env python
"""Per-(kernel, grid) statistics from a rocprofv3 rocpd database: the same kernel launched at several shapes
(e.g. tools/mattn_bench.py's three key lengths) split by its grid.

    python tools/rocpd_grid.py gpurun_out/kt_g/kt_results.db [substring ...]
"""
import re
import sqlite3
import sys


def short(name):
    name = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", name)
    return name[:60]


def main(path, subs):
    con = sqlite3.connect(path)
    rows = con.execute("select name, grid_x, grid_y, workgroup_x, lds_size, count(*), avg(duration), min(duration) "
                       "from kernels group by name, grid_x, grid_y order by name, grid_x, grid_y").fetchall()
    print(f"{'kernel':60s} {'grid':>14s} {'wg':>5s} {'lds':>7s} {'calls':>5s} {'avg_us':>9s} {'min_us':>9s}")
    for name, gx, gy, wx, lds, n, avg, mn in rows:
        if subs and not any(s in name for s in subs):
            continue
        print(f"{short(name):60s} {gx // max(wx, 1):>7d}x{gy:<6d} {wx:>5d} {lds:>7d} {n:>5d} {avg / 1e3:9.2f} {mn / 1e3:9.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
