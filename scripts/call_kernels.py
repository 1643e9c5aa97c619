"""Per-call kernel table of a rocprofv3 kernel trace: the calls are the
windows between consecutive launches of a marker kernel (e.g. k_fjlt_z, the
first kernel of a general-engine call); prints total us and count per kernel
name for call number CALL.  usage: call_kernels.py trace.csv MARKER CALL [N]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
mark, call = sys.argv[2], int(sys.argv[3])
top = int(sys.argv[4]) if len(sys.argv) > 4 else 14
st = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
a, b = st[call], (st[call + 1] if call + 1 < len(st) else len(rows))
agg = collections.OrderedDict()
for r in rows[a:b]:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    key = n[:40] if n.startswith("Cijk") else n.split("(")[0][:80]
    agg.setdefault(key, [0, 0])
    agg[key][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg[key][1] += 1
span = (int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
print(f"call {call} of {len(st)}: span {span:.1f} us, busy {sum(v[0] for v in agg.values()) / 1e3:.1f} us")
for k, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:top]:
    print(f"{t / 1e3:10.1f} {c:4d} {k}")
