#!/usr/bin/env python3
"""Per-kernel average of rocprofv3 --pmc counter CSVs (one or more passes):
tools/pmc_summary.py dir1/p_counter_collection.csv [dir2/...] [--match substr,...]"""
import collections
import csv
import sys

args = sys.argv[1:]
match = None
if "--match" in args:
    i = args.index("--match")
    match = args[i + 1].split(",")
    del args[i:i + 2]
files = args
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(collections.Counter)
for f in files:
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if match:
            hit = [m for m in match if m in name]
            if not hit:
                continue
            k = hit[0]
        else:
            k = name[:80]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k][r["Counter_Name"]] += 1
for k, d in agg.items():
    print(k)
    for c in sorted(d):
        print(f"    {c:24s} {d[c] / n[k][c]:16.4g}")
