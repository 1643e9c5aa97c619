"""FETCH_SIZE calibration table from scripts/pmc_calibrate.sh output: per
workload, the dispatches whose name matches the workload's hint (first one
dropped: warm-up), mean FETCH_SIZE (KB units x 1024) against the bytes a
perfect kernel reads.  The streaming ratio is the factor to apply to
FETCH_SIZE of wide coalesced reads (LDS-DMA or 16-B loads); the gather
ratios bound what a random-row kernel can do.

usage: python scripts/pmc_calib_summary.py gpurun_out/pmc_cal profiles/r5/pmc_cal > profiles/r5/pmc_calibration.md"""
from __future__ import annotations

import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict


def load(root, op):
    meta = None
    with open(os.path.join(root, f"{op}.log")) as f:
        for line in f:
            if line.startswith("{"):
                meta = json.loads(line)
    paths = glob.glob(os.path.join(root, op, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(lambda: [0.0, None, ""])
    for p in paths:
        with open(p) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] != "FETCH_SIZE":
                    continue
                d = int(row["Dispatch_Id"])
                per[d][0] += float(row["Counter_Value"])
                per[d][1] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3
                per[d][2] = row["Kernel_Name"]
    return meta, per, paths


def main():
    root, dest = sys.argv[1], sys.argv[2]
    os.makedirs(dest, exist_ok=True)
    rows = []
    for op in ("stream", "ldsdma", "gather128", "gather64", "cwt"):
        if not os.path.exists(os.path.join(root, f"{op}.log")):
            continue
        meta, per, paths = load(root, op)
        for p in paths:
            shutil.copy(p, os.path.join(dest, f"{op}.csv"))
        if meta is None:
            continue
        hits = [(d, v) for d, v in sorted(per.items()) if meta["kernel_hint"] in v[2]]
        if len(hits) > 1:
            hits = hits[1:]
        if not hits:
            continue
        fetch = sum(v[0] for _, v in hits) / len(hits) * 1024.0
        t = sum(v[1] for _, v in hits) / len(hits)
        rows.append((op, meta["expected_read_bytes"], fetch, t, hits[0][1][2][:60], len(hits)))
    print("# FETCH_SIZE calibration (gfx950, rocprofv3 --pmc FETCH_SIZE)\n")
    print("| workload | kernel | bytes a perfect kernel reads | FETCH_SIZE x 1024 per dispatch | ratio FETCH / true | us under counters |")
    print("|---|---|---:|---:|---:|---:|")
    for op, exp, fetch, t, name, nd in rows:
        print(f"| {op} | `{name}` ({nd} dispatches) | {exp / 1e9:.3f} GB | {fetch / 1e9:.3f} GB | {fetch / exp:.3f} | {t:.1f} |")
    cal = {op: fetch / exp for op, exp, fetch, *_ in rows}
    if "stream" in cal or "ldsdma" in cal:
        s = cal.get("ldsdma", cal.get("stream"))
        print(f"\nStreaming factor: true bytes = FETCH_SIZE x 1024 / {s:.3f} (wide coalesced reads).")
    for op in ("gather128", "gather64"):
        if op in cal:
            print(f"{op}: a random-row gather shows {cal[op]:.2f} x its useful bytes in FETCH_SIZE.")
    if "cwt" in cal and "gather128" in cal:
        print(f"cwt: {cal['cwt']:.2f} x its CSR bytes in FETCH_SIZE.")
    json.dump(cal, open(os.path.join(dest, "calibration.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
