"""Median per-position kernel durations of the engine's randSVD calls in a
rocprofv3 kernel trace (calls delimited by the FJLT-operator launch; the
first `skip` calls dropped).  usage: call_positions.py <kernel_trace.csv> [skip]"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_fjlt_zt" in r["Kernel_Name"]]
calls = [rows[a:b] for a, b in zip(starts, starts[1:])][skip:]
n = min(len(c) for c in calls)
spans = [(int(c[n - 1]["End_Timestamp"]) - int(c[0]["Start_Timestamp"])) / 1e3 for c in calls]
print(f"calls {len(calls)}  kernels/call {n}  span median {statistics.median(spans):.1f} us")
tail = 0.0
for p in range(n):
    d = [(int(c[p]["End_Timestamp"]) - int(c[p]["Start_Timestamp"])) / 1e3 for c in calls]
    name = calls[0][p]["Kernel_Name"]
    short = name.split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")[:60]
    med = statistics.median(d)
    if "pass5" not in name:
        tail += med
    print(f"{p:3d} {med:8.1f} {min(d):8.1f}  {short}")
print(f"non-pass kernels (median sum) {tail:.1f} us")
