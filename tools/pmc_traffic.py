"""Turn a FETCH_SIZE pass and a WRITE_SIZE pass (rocprofv3 --pmc, separate runs) over the MSDA backward
into profiles/msda_bwd_traffic.json, the HBM-traffic figure bench.py reports as roofline.traffic.

Units and gfx950 corrections follow /opt/skills/guides/MI355X_MICROARCH.md: both counters are KB;
FETCH_SIZE is doubled (gfx950 tallies 128-B read requests at 64 B), WRITE_SIZE is taken as reported.

usage: python tools/pmc_traffic.py FETCH.csv WRITE.csv [--copy-as r01_l]
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import shutil
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# 115.60 MB per 1024² image per launch (fp32), 16 images per launch at config 2.
ALGO_BYTES = 1849688064


def _mean(path: str, counter: str):
    vals, name = [], None
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter and "msda_bwd" in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
                name = r["Kernel_Name"]
    if not vals:
        raise SystemExit(f"no {counter} rows for msda_bwd in {path}")
    return statistics.fmean(vals), len(vals), name


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--copy-as", default=None, help="also copy the CSVs to profiles/<tag>_pmc_{fetch,write}.csv")
    a = ap.parse_args()
    fkb, nf, name = _mean(a.fetch, "FETCH_SIZE")
    wkb, nw, _ = _mean(a.write, "WRITE_SIZE")
    srcs = [a.fetch, a.write]
    if a.copy_as:
        srcs = [f"profiles/{a.copy_as}_pmc_fetch.csv", f"profiles/{a.copy_as}_pmc_write.csv"]
        shutil.copy(a.fetch, os.path.join(ROOT, srcs[0]))
        shutil.copy(a.write, os.path.join(ROOT, srcs[1]))
    fetch_b = int(round(fkb * 1024 * 2))
    write_b = int(round(wkb * 1024))
    out = {
        "kernel": name[:120] + "... (m2f_msda_fused_bwd_f32), config 2 shapes, 16 images",
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over one bench step "
                  "(tools/gpu/pmc.sh), the MSDA-backward dispatches of each pass averaged; FETCH_SIZE/WRITE_SIZE "
                  "are KB; FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B read requests at "
                  "64 B), WRITE_SIZE as reported",
        "dispatches": [nf, nw],
        "fetch_size_kb_raw": round(fkb, 1),
        "write_size_kb_raw": round(wkb, 1),
        "fetch_bytes_per_launch": fetch_b,
        "write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": fetch_b + write_b,
        "algorithmic_bytes_per_launch": ALGO_BYTES,
        "traffic_over_algorithmic": round((fetch_b + write_b) / ALGO_BYTES, 3),
        "source_files": srcs,
    }
    with open(os.path.join(ROOT, "profiles", "msda_bwd_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
