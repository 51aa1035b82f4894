#!/usr/bin/env python
"""Per-kernel roofline table of one bench step: the top kernels by time, each with its
algorithmic roofline fraction (bench.py's roofline_all, for the hand-written families) and counter evidence
(rocprofv3 PMC: MFMA busy, clock, HBM bytes -> achieved HBM GB/s and traffic / algorithmic bytes).

    python tools/roofline_table.py --stats profiles/r02_x_kernel_stats.csv --pmc profiles/r02_x_pmc_summary.json \\
        --bench profiles/r02_x_bench.json --steps 4 --out profiles/r02_x_roofline.md

--steps: bench steps the kernel-stats trace covers (warm-up included) to express totals per step.
"""
from __future__ import annotations

import argparse
import csv
import json
import re

FAMILY = [  # kernel-name pattern -> bench.py roofline family
    (r"^x3_nt_kernel", "x3_gemm_nt"), (r"^x3_tn_kernel", "x3_gemm_tn"), (r"^x3_conv_kernel", "x3_conv"),
    (r"^x3_conv_wgrad_kernel", "x3_conv_wgrad"), (r"^msda_bwd", "msda_bwd"), (r"^msda_fused_fwd|^msda_fwd", "msda_fwd"),
    (r"mattn_bwd_kernel", "masked_attn_bwd"), (r"mattn_fwd_kernel", "masked_attn_fwd"),
    (r"mask_heads_kernel", "mask_heads_fwd"), (r"mask_de_kernel", "mask_heads_bwd_embed"),
    (r"mask_df_kernel", "mask_heads_bwd_feats"), (r"attn_mask_bits_kernel", "attn_mask_bits"),
]
HBM_PEAK = 8000.0


def short(name: str) -> str:
    name = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "")
    m = re.match(r"_ZN12_GLOBAL__N_1\d+(\w+?)I", name)
    if m:
        name = m.group(1)
    return re.sub(r"\(.*", "", name)[:70]


def family(name: str):
    for pat, fam in FAMILY:
        if re.search(pat, name):
            return fam
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats", required=True)
    ap.add_argument("--pmc", required=True)
    ap.add_argument("--bench", required=True)
    ap.add_argument("--steps", type=float, default=4.0)
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    stats = {}
    for r in csv.DictReader(open(a.stats)):
        k = short(r["Name"])
        t = stats.setdefault(k, [0.0, 0])
        t[0] += float(r["TotalDurationNs"]) / 1e6 / a.steps
        t[1] += int(r["Calls"])
    pmc = {}
    for r in json.load(open(a.pmc)):
        k = short(r["kernel"])
        pmc.setdefault(k, r)
    bench = json.loads(open(a.bench).read().splitlines()[0])
    fams = {r["kernel"]: r for r in bench.get("roofline_all") or []}
    total = sum(v[0] for v in stats.values())
    rows = []
    for k, (ms, calls) in sorted(stats.items(), key=lambda kv: -kv[1][0])[:a.top]:
        p = pmc.get(k, {})
        fam = family(k)
        fr = fams.get(fam) if fam else None
        dur = p.get("mean_ms")
        hbm = None
        if dur and (p.get("fetch_B") or p.get("write_B")):
            hbm = (p.get("fetch_B", 0) + p.get("write_B", 0)) / (dur * 1e-3) / 1e9
        rows.append({
            "kernel": k, "ms_per_step": round(ms, 3), "share": round(ms / total, 4),
            "family": fam, "bound": fr.get("bound") if fr else None,
            "roofline_frac": fr.get("frac") if fr else None,
            "mfma_busy": round(p["mfma_busy"], 3) if p.get("mfma_busy") else None,
            "clk_GHz": round(p["clk_GHz"], 2) if p.get("clk_GHz") else None,
            "pmc_hbm_GBs": round(hbm, 1) if hbm else None,
            "pmc_hbm_frac": round(hbm / HBM_PEAK, 4) if hbm else None,
        })
    with open(a.out, "w") as f:
        f.write(f"# Top {a.top} kernels of one bench step ({total:.1f} ms of kernel time per step)\n\n")
        f.write("roofline_frac: algorithmic work / mean launch / peak (bench.py roofline_all; MFMA families price "
                "6 bf16 products per fp32 x3 product against 2.5 PF). mfma_busy: SQ_VALU_MFMA_BUSY_CYCLES / "
                "(GRBM_GUI_ACTIVE/8 x 1024 SIMDs). pmc_hbm: (2 x FETCH_SIZE + WRITE_SIZE) / mean duration.\n\n")
        f.write("| kernel | ms/step | share | family | bound | roofline frac | MFMA busy | clk GHz | PMC HBM GB/s | PMC HBM frac |\n")
        f.write("|---|---|---|---|---|---|---|---|---|---|\n")
        for r in rows:
            f.write("| " + " | ".join("" if r[c] is None else str(r[c]) for c in
                                     ("kernel", "ms_per_step", "share", "family", "bound", "roofline_frac", "mfma_busy",
                                      "clk_GHz", "pmc_hbm_GBs", "pmc_hbm_frac")) + " |\n")
    with open(a.out.replace(".md", ".json"), "w") as f:
        json.dump(rows, f, indent=1)
    print(open(a.out).read())


if __name__ == "__main__":
    main()
