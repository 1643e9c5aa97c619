"""One randSVD call (engine path) from a rocprofv3 kernel trace: the last
complete call between two FJLT-operator launches; span, busy, gaps, kernels.
usage: trace_engine.py <kernel_trace.csv>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_fjlt_zt" in r["Kernel_Name"]]
a, b = starts[-2], starts[-1]
seg = rows[a:b]
t0 = int(seg[0]["Start_Timestamp"])
busy, prev, gaps = 0, None, []
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    if prev is not None:
        gaps.append((s - prev, r["Kernel_Name"][:60]))
    prev = e
span = int(seg[-1]["End_Timestamp"]) - t0
print(f"call span {span / 1e3:.1f} us busy {busy / 1e3:.1f} us kernels {len(seg)}")
for g, n in sorted(gaps, reverse=True)[:6]:
    print(f"  gap {g / 1e3:8.1f} us before {n}")
for r in seg:
    print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:8.1f}  {r['Kernel_Name'][:80]}")
