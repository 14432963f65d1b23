#!/usr/bin/env python3
"""Summarise a rocprofv3 *_kernel_stats.csv (top kernels by total time)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 14
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("| kernel | calls | total ms | avg us | % |\n|---|---|---|---|---|")
for r in rows[:n]:
    print(f"| {r['Name'][:90]} | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.2f} | "
          f"{float(r['AverageNs'])/1e3:.1f} | {100*float(r['TotalDurationNs'])/tot:.1f} |")
print(f"\ntotal kernel time: {tot/1e6:.2f} ms")
