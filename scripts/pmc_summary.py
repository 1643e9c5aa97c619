"""Summarise the fused-pass PMC runs (scripts/pmc_pass.sh): per counter, the
mean per dispatch of k_rsvd_pass* (first dispatch dropped: cold caches), for
the inter (final 0) and last-pass (final 1) forms; markdown table on stdout,
the raw counter CSVs copied to the given directory.  HBM bytes are
FETCH_SIZE x 1024 divided by the MEASURED streaming ratio of the LDS-DMA
workload in the calibration file (scripts/pmc_calibrate.sh ->
profiles/r5/pmc_cal/calibration.json), not an assumed factor.

usage: python scripts/pmc_summary.py gpurun_out/pmc5 profiles/r5/pmc5 profiles/r5/pmc_cal/calibration.json"""
from __future__ import annotations

import json

import csv
import glob
import os
import shutil
import sys
from collections import defaultdict


def collect(root, final):
    vals = defaultdict(list)
    ticks = []
    for path in sorted(glob.glob(os.path.join(root, f"f{final}_g*", "**", "*counter_collection.csv"), recursive=True)):
        per = defaultdict(dict)
        with open(path) as f:
            for row in csv.DictReader(f):
                if "k_rsvd_pass" not in row["Kernel_Name"]:
                    continue
                d = int(row["Dispatch_Id"])
                per[d][row["Counter_Name"]] = per[d].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
                per[d]["_t"] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3
        ds = sorted(per)[1:]
        for d in ds:
            for c, v in per[d].items():
                if c == "_t":
                    ticks.append(v)
                else:
                    vals[c].append(v)
    return {c: sum(v) / len(v) for c, v in vals.items() if v}, (sum(ticks) / len(ticks) if ticks else None)


def main():
    root, dest, calp = sys.argv[1], sys.argv[2], sys.argv[3]
    cal = json.load(open(calp))
    ratio = cal["ldsdma"]   # FETCH_SIZE x 1024 / true bytes of a known LDS-DMA stream
    os.makedirs(dest, exist_ok=True)
    for path in glob.glob(os.path.join(root, "f*_g*", "**", "*counter_collection.csv"), recursive=True):
        tag = os.path.relpath(path, root).split(os.sep)[0]
        shutil.copy(path, os.path.join(dest, f"{tag}.csv"))
    inter, ti = collect(root, 0)
    fin, tf = collect(root, 1)
    names = sorted(set(inter) | set(fin))
    print("| counter | inter pass (final 0) | last pass (final 1) |")
    print("|---|---:|---:|")
    for c in names:
        print(f"| {c} | {inter.get(c, float('nan')):.4g} | {fin.get(c, float('nan')):.4g} |")
    print(f"| dispatch time under counters (us) | {ti or float('nan'):.1f} | {tf or float('nan'):.1f} |")
    for tag, d, t in (("inter", inter, ti), ("last", fin, tf)):
        if not d:
            continue
        wc = d.get("SQ_WAVE_CYCLES")
        out = []
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in d:
                    out.append(f"{c} {100 * d[c] / wc:.0f}% of wave cycles")
        if "GRBM_GUI_ACTIVE" in d and "SQ_VALU_MFMA_BUSY_CYCLES" in d:
            cyc = d["GRBM_GUI_ACTIVE"] / 8
            out.append(f"MFMA busy {100 * d['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / cyc:.0f}% (per SIMD over GRBM_GUI_ACTIVE/8)")
        if "FETCH_SIZE" in d and t:
            by = d["FETCH_SIZE"] * 1024 / ratio
            out.append(f"HBM read {by / 1e9:.2f} GB (FETCH_SIZE x 1024 / {ratio:.3f} calibrated) = "
                       f"{by / (t * 1e-6) / 1e12:.2f} TB/s under counters")
        if "SQ_LDS_BANK_CONFLICT" in d and "SQ_LDS_IDX_ACTIVE" in d:
            out.append(f"LDS bank conflicts {100 * d['SQ_LDS_BANK_CONFLICT'] / d['SQ_LDS_IDX_ACTIVE']:.0f}% of LDS cycles")
        print(f"\n{tag}: " + "; ".join(out))


if __name__ == "__main__":
    main()
