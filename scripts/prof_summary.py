#!/usr/bin/env python
"""Summarise a rocprofv3 ``*_kernel_stats.csv`` into a markdown table.

usage: python scripts/prof_summary.py gpurun_out/prof/run_kernel_stats.csv [title] [top]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else path
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    rows = list(csv.DictReader(open(path)))
    print(f"# {title}\n")
    print("| kernel | calls | total us | avg us | % |")
    print("|---|---:|---:|---:|---:|")
    for r in rows[:top]:
        name = r["Name"].replace("|", "/")
        if len(name) > 110:
            name = name[:107] + "..."
        print(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e3:.1f} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")


if __name__ == "__main__":
    main()
