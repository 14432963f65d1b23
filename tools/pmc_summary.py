#!/usr/bin/env python3
"""Per-kernel average of rocprofv3 --pmc counter CSVs (one or more passes):
tools/pmc_summary.py dir1/p_counter_collection.csv [dir2/...] [--match substr,...] [--per N]
--per N: sums over every dispatch divided by N (e.g. the trials of the run)
instead of per-dispatch averages, plus memory-side MB per N (TCC_EA0 read
requests x 128 B, 64-byte write requests x 64 B, the other writes x 32 B)."""
import collections
import csv
import sys

args = sys.argv[1:]
match = None
per = None
if "--per" in args:
    i = args.index("--per")
    per = float(args[i + 1])
    del args[i:i + 2]
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
tot_mb = 0.0
for k, d in agg.items():
    print(k)
    for c in sorted(d):
        print(f"    {c:24s} {(d[c] / per if per else d[c] / n[k][c]):16.4g}")
    if per and "TCC_EA0_RDREQ_sum" in d and "TCC_EA0_WRREQ_sum" in d and "TCC_EA0_WRREQ_64B_sum" in d:
        rd = d["TCC_EA0_RDREQ_sum"] * 128 / per / 1e6
        w64 = d["TCC_EA0_WRREQ_64B_sum"]
        wr = (w64 * 64 + (d["TCC_EA0_WRREQ_sum"] - w64) * 32) / per / 1e6
        tot_mb += rd + wr
        print(f"    memory-side MB per unit: read {rd:.2f} write {wr:.2f}")
        if "TCC_EA0_RDREQ_DRAM_sum" in d:
            print(f"    of the reads from DRAM: {d['TCC_EA0_RDREQ_DRAM_sum'] * 128 / per / 1e6:.2f} MB")
if per:
    print(f"total memory-side MB per unit (matched kernels): {tot_mb:.2f}")
