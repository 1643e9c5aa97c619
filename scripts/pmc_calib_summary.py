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
    for op in ("stream", "ldsdma", "gather128", "gather64", "rgather128", "rgather64", "cwt"):
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
    for op in ("gather128", "gather64", "rgather128", "rgather64"):
        if op in cal:
            print(f"{op}: a random-row gather shows {cal[op]:.2f} x its useful bytes in FETCH_SIZE.")
    if "cwt" in cal and "gather128" in cal:
        print(f"cwt: {cal['cwt']:.2f} x its CSR bytes in FETCH_SIZE.")
    # useful-byte throughput: the random-row gathers bound what the CWT (rows
    # of 10 nnz = 80 B of column + value, visited in random bucket order) can do
    bw = {op: exp / (t * 1e-6) / 1e9 for op, exp, fetch, t, *_ in rows}
    print("\n| workload | useful GB/s under counters |")
    print("|---|---:|")
    for op, v in bw.items():
        print(f"| {op} | {v:.0f} |")
    # line-request rate (FETCH_SIZE x 1024 / 64 B per second): what a random
    # access kernel is bounded by, whatever its useful bytes per line
    rate = {op: fetch / 64 / (t * 1e-6) / 1e9 for op, exp, fetch, t, *_ in rows}
    print("\n| workload | 64-B fetch requests per ns (FETCH_SIZE x 1024 / 64 / time) |")
    print("|---|---:|")
    for op, v in rate.items():
        print(f"| {op} | {v:.1f} |")
    best = max((rate[o] for o in ("rgather128", "rgather64", "gather128", "gather64") if o in rate), default=None)
    if "cwt" in rate and best:
        print(f"\ncwt issues {rate['cwt']:.1f} fetch requests per ns: {100 * rate['cwt'] / best:.0f}% of the best "
              f"random-gather rate measured here ({best:.1f}).")
    if "cwt" in bw and "gather64" in bw and "gather128" in bw:
        print(f"\ncwt moves its CSR at {bw['cwt']:.0f} GB/s: {100 * bw['cwt'] / bw['gather64']:.0f}% of the 64-B "
              f"random-row gather ({bw['gather64']:.0f} GB/s) and {100 * bw['cwt'] / bw['gather128']:.0f}% of the "
              f"128-B one ({bw['gather128']:.0f} GB/s); its 80-B rows sit between the two.")
    json.dump(cal, open(os.path.join(dest, "calibration.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
