#!/usr/bin/env python
"""Per-kernel summary of rocprofv3 --pmc CSVs (one or more passes over the same command).

    python tools/pmc_summary.py gpurun_out/r2a_sq/sq_counter_collection.csv [more.csv ...] [--top 25] [--json out]

Counters are summed per dispatch (rocprofv3 writes one row per dispatch and counter) and averaged over a
kernel's dispatches.  Derived columns, with the gfx950 units of /opt/skills/guides/MI355X_MICROARCH.md:
  clk_GHz      the clock the chip held during the kernel's dispatches.  GRBM_GUI_ACTIVE / 8 (summed over the 8
               XCDs) / dispatch duration for dispatches of 0.3 ms or more; below that the GRBM quotient reads high
               (MI355X_MICROARCH.md 'DVFS give-back': 2.5-6.7 GHz were reported for the masked-attention and reduce
               kernels), so short dispatches use SQ_BUSY_CYCLES / k / duration, k = the SQ_BUSY_CYCLES : GRBM/8 ratio
               of this input's >= 1 ms dispatches (about 31: one SQ per shader engine, 32 on the chip, busy ~97 % of
               a long kernel), or 32 when the input has none.  Capped at 2.4 GHz (the chip's top clock); clk_src says
               which ("grbm", "sq_busy", "cap").
  mfma_busy    SQ_VALU_MFMA_BUSY_CYCLES / (clk * duration * 1024 SIMDs)
  mfma_peak_frac  the MFMA work the kernel issued (SQ_INSTS_VALU_MFMA_MOPS_* x 512 FLOP) / duration / the dense peak
               of its dtype: utilisation against the chip's peak, independent of any clock estimate
  mfma_TF      (SQ_INSTS_VALU_MFMA_MOPS_{BF16,F16,F32} * 512) / duration, and its fraction of the dense peak
               of that dtype (bf16/f16 2500 TF, f32 157.3 TF)
  hbm_GBs      (2 * FETCH_SIZE + WRITE_SIZE) KB / duration (FETCH_SIZE doubled: gfx950 tallies 128-B reads at 64 B)
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import re

PEAK_TF = {"BF16": 2500.0, "F16": 2500.0, "F32": 157.3}


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\(.*", "", name)  # drop the argument list
    return name[:110]


def load(paths):
    # (kernel, dispatch) -> counters; durations per dispatch
    disp = collections.defaultdict(dict)
    dur = {}
    for path in paths:
        with open(path) as f:
            for r in csv.DictReader(f):
                key = (path, r["Dispatch_Id"])
                k = short(r["Kernel_Name"])
                disp[(k, key)][r["Counter_Name"]] = disp[(k, key)].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                dur[(k, key)] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, key), ctrs in disp.items():
        for c, v in ctrs.items():
            per[k][c].append(v)
        per[k]["_dur"].append(dur[(k, key)])
    return per


MAX_CLK_GHZ = 2.4
SHORT_S = 0.3e-3


def sq_busy_ratio(per):
    """SQ_BUSY_CYCLES per GRBM_GUI_ACTIVE / 8 cycle on this input's dispatches of 1 ms or more (median)."""
    rs = []
    for cols in per.values():
        for d, sq, g in zip(cols["_dur"], cols.get("SQ_BUSY_CYCLES", []), cols.get("GRBM_GUI_ACTIVE", [])):
            if d >= 1e-3 and g > 0:
                rs.append(sq / (g / 8))
    rs.sort()
    return rs[len(rs) // 2] if rs else 32.0


def kernel_clock(d, grbm, sq_busy, k_sq):
    """(GHz, source) for a mean dispatch of d seconds (see the module docstring)."""
    if grbm and d >= SHORT_S:
        clk, src = grbm / 8 / d / 1e9, "grbm"
    elif sq_busy:
        clk, src = sq_busy / k_sq / d / 1e9, "sq_busy"
    elif grbm:
        clk, src = grbm / 8 / d / 1e9, "grbm"
    else:
        return None, None
    return (MAX_CLK_GHZ, "cap") if clk > MAX_CLK_GHZ else (clk, src)


def summarize(per):
    rows = []
    k_sq = sq_busy_ratio(per)
    for k, cols in per.items():
        mean = {c: sum(v) / len(v) for c, v in cols.items()}
        n = len(cols["_dur"])
        d = mean["_dur"]
        row = {"kernel": k, "dispatches": n, "mean_ms": d * 1e3, "total_ms": sum(cols["_dur"]) * 1e3}
        clk, src = kernel_clock(d, mean.get("GRBM_GUI_ACTIVE"), mean.get("SQ_BUSY_CYCLES"), k_sq) if d > 0 else (None, None)
        if clk:
            row["clk_GHz"], row["clk_src"] = clk, src
        if "SQ_VALU_MFMA_BUSY_CYCLES" in mean and clk:
            row["mfma_busy"] = mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (clk * 1e9 * d * 1024)
        peak = []
        for dt in ("BF16", "F16", "F32"):
            c = f"SQ_INSTS_VALU_MFMA_MOPS_{dt}"
            if mean.get(c):
                tf = mean[c] * 512 / d / 1e12
                row[f"mfma_{dt}_TF"] = tf
                row[f"mfma_{dt}_frac"] = tf / PEAK_TF[dt]
                peak.append(tf / PEAK_TF[dt])
        if peak:
            row["mfma_peak_frac"] = sum(peak)
        if "FETCH_SIZE" in mean:
            row["fetch_B"] = 2 * mean["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in mean:
            row["write_B"] = mean["WRITE_SIZE"] * 1024
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
                  "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"):
            if c in mean:
                row[c] = mean[c]
        row["counters"] = {c: v for c, v in mean.items() if c != "_dur"}
        rows.append(row)
    rows.sort(key=lambda r: -r["total_ms"])
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--json", default=None)
    ap.add_argument("--all", action="store_true", help="every counter's per-dispatch mean, per kernel")
    a = ap.parse_args()
    rows = summarize(load(a.csv))
    cols = ["dispatches", "mean_ms", "total_ms", "clk_GHz", "clk_src", "mfma_busy", "mfma_peak_frac", "mfma_BF16_TF",
            "mfma_F16_TF", "mfma_F32_TF", "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS"]
    print("kernel".ljust(70) + "".join(c[:12].rjust(13) for c in cols))
    for r in rows[: a.top]:
        print(r["kernel"][:69].ljust(70) + "".join(
            (f"{r[c]:13.4g}" if isinstance(r.get(c), float) else str(r.get(c, "")).rjust(13)) for c in cols))
    if a.all:
        for r in rows[: a.top]:
            print(f"\n{r['kernel']}  ({r['dispatches']} dispatches, {r['mean_ms']:.4f} ms)")
            for c, v in sorted(r["counters"].items()):
                print(f"  {c:32s} {v:16.6g}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
