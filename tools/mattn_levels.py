#!/usr/bin/env python
"""Per-level masked-attention kernel times from a rocprofv3 kernel trace of tools/mattn_bench.py.

The bench runs, for each of its six (config, Lk) cases in order, 23 forward calls and then 23 forward + backward
calls, so the i-th case owns forward-kernel launches 46 i .. 46 i + 45 and every other masked-attention kernel
launched between them.  Prints the median duration (us) of each kernel family per case.

    python tools/mattn_levels.py gpurun_out/r5p_prof_xcd1/mattn_results.db [more.db ...]
"""
import sqlite3
import statistics
import sys

CASES = [("config 2", 1024), ("config 2", 4096), ("config 2", 16384),
         ("config 4", 1024), ("config 4", 4096), ("config 4", 16384)]
FAMILIES = (("fwd", "mattn_fwd_kernel"), ("combine", "mattn_combine"), ("bwd", "mattn_bwd"),
            ("dq_reduce", "mattn_dq_reduce_kernel"))


def family(name):
    for fam, key in FAMILIES:
        if key in name:
            return fam
    return None


def levels(path):
    con = sqlite3.connect(path)
    rows = con.execute("select name, duration from kernels order by start").fetchall()
    per = {}
    nfwd = 0
    for name, dur in rows:
        fam = family(name)
        if fam is None:
            continue
        # every other kernel follows the forward launch it belongs to
        case = min((nfwd if fam == "fwd" else max(nfwd - 1, 0)) // 46, len(CASES) - 1)
        if fam == "fwd":
            nfwd += 1
        per.setdefault((case, fam), []).append(dur / 1e3)
    return per


def main(paths):
    for path in paths:
        per = levels(path)
        print(f"== {path}")
        for i, (cfg, lk) in enumerate(CASES):
            parts = {fam: statistics.median(per[(i, fam)]) for fam, _ in FAMILIES if (i, fam) in per}
            fwd = parts.get("fwd", 0.0) + parts.get("combine", 0.0)
            bwd = parts.get("bwd", 0.0) + parts.get("dq_reduce", 0.0)
            print(f"  {cfg} Lk={lk:5d}: fwd {parts.get('fwd', 0):6.1f} + combine {parts.get('combine', 0):4.1f} = "
                  f"{fwd:6.1f}   bwd {parts.get('bwd', 0):6.1f} + dq_reduce {parts.get('dq_reduce', 0):4.1f} = {bwd:6.1f}")


if __name__ == "__main__":
    main(sys.argv[1:])
