#!/usr/bin/env python3
"""Median host time per HIP API call (hipLaunchKernel by kernel) after the
first T ms of a rocprofv3 --hip-trace run: where launches are slow.
tools/expt/launch_stats.py <hip_api_trace.csv[.gz]> <kernel_trace.csv[.gz]> [--after-ms T]"""
import csv
import gzip
import statistics
import sys
from collections import defaultdict


def rd(p):
    return csv.DictReader(gzip.open(p, "rt") if p.endswith(".gz") else open(p))


def main():
    api = list(rd(sys.argv[1]))
    ker = {r["Correlation_Id"]: r["Kernel_Name"] for r in rd(sys.argv[2])}
    after = float(sys.argv[sys.argv.index("--after-ms") + 1]) if "--after-ms" in sys.argv else 200.0
    t0 = min(int(a["Start_Timestamp"]) for a in api)
    by = defaultdict(list)
    for a in api:
        if (int(a["Start_Timestamp"]) - t0) / 1e6 < after:
            continue
        d = (int(a["End_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3
        by[a["Function"]].append(d)
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:12]:
        print(f"{k:28s} n={len(v):5d} sum={sum(v) / 1e3:8.2f} ms median={statistics.median(v):7.1f} us")


if __name__ == "__main__":
    main()
