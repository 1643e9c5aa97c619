"""Summarise one bench step from a rocprofv3 kernel trace: span, busy time,
largest idle gaps, kernel list.  usage: trace_step.py <kernel_trace.csv>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
FINAL = ("k_tsk_pass<128, 3, true, true, true", "k_tsk_pass<128, 3, true, false, true")
idx = [i for i, r in enumerate(rows) if any(p in r["Kernel_Name"] for p in FINAL)]
a, b = idx[-2], idx[-1]
# step = from the first pass of step i to the first pass of step i+1
starts = [i for i, r in enumerate(rows) if i < b and any(
    p in r["Kernel_Name"] for p in ("k_tsk_pass<128, 3, true, true, false", "k_tsk_pass<128, 3, true, false, false"))]
first = [i for i in starts if i < a]
a0 = first[-2] if len(first) >= 2 else first[-1]
b0 = [i for i in starts if i > a][0] if any(i > a for i in starts) else b
seg = rows[a0:b0]
t0 = int(seg[0]["Start_Timestamp"])
busy, prev, gaps = 0, None, []
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    if prev is not None:
        gaps.append((s - prev, r["Kernel_Name"][:60]))
    prev = e
span = int(seg[-1]["End_Timestamp"]) - t0
print(f"step span {span / 1e3:.1f} us busy {busy / 1e3:.1f} us kernels {len(seg)}")
for g, n in sorted(gaps, reverse=True)[:8]:
    print(f"  gap {g / 1e3:8.1f} us before {n}")
if "-v" in sys.argv:
    for r in seg:
        print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:8.1f}  {r['Kernel_Name'][:70]}")
