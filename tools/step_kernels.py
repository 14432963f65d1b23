#!/usr/bin/env python3
"""Per-step kernel time of a bench kernel trace (rocprofv3 kernel_trace.csv):
the timed window starts at the dedispersion launch of step --skip (warmup
steps excluded), kernels grouped by name, GPU busy fraction of the window.
    tools/step_kernels.py kernel_trace.csv --skip 2 --steps 4"""
import argparse
import csv
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=2)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--top", type=int, default=24)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    torch_end = max((e for s, e, n in iv if "at::native" in n), default=0)
    iv = [x for x in iv if x[0] > torch_end]
    starts = [s for s, e, n in iv if "dedisperse" in n]
    w0 = starts[a.skip]
    win = [x for x in iv if x[0] >= w0]
    span = win[-1][1] - w0
    busy, cs, ce = 0, win[0][0], win[0][1]
    fam, cnt = defaultdict(float), defaultdict(int)
    for s, e, n in win:
        k = n.replace("(anonymous namespace)::", "").replace("psoup::kern::", "").replace("void ", "")
        k = re.sub(r"\(.*", "", k)[:70]
        fam[k] += (e - s) / 1e6
        cnt[k] += 1
        if s > ce:
            busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print(f"window {span / 1e6:.1f} ms = {span / 1e6 / a.steps:.1f} ms/step; GPU busy {100 * busy / span:.1f}%")
    print("| kernel | ms/step | calls/step |\n|---|---|---|")
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"| {k} | {v / a.steps:.2f} | {cnt[k] / a.steps:.1f} |")
    print(f"| (all kernels) | {sum(fam.values()) / a.steps:.2f} | |")


if __name__ == "__main__":
    main()
