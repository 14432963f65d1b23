#!/usr/bin/env python3
"""GPU busy/idle timeline of a rocprofv3 kernel trace: union of kernel
intervals, idle gaps (histogram), and busy time by kernel family over a
window.  tools/trace_gaps.py kernel_trace.csv [--after-ms T]"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    after = float(sys.argv[sys.argv.index("--after-ms") + 1]) if "--after-ms" in sys.argv else 0.0
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    t0 = iv[0][0]
    iv = [x for x in iv if (x[0] - t0) * 1e-6 >= after]
    t0 = iv[0][0]
    busy, cur_s, cur_e, gaps = 0, iv[0][0], iv[0][1], []
    fam = defaultdict(float)
    for s, e, name in iv:
        key = name.split("(")[0].split("::")[-1][:40]
        fam[key] += (e - s) * 1e-6
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = iv[-1][1] - t0
    print(f"window {span * 1e-6:.2f} ms, GPU busy {busy * 1e-6:.2f} ms ({100 * busy / span:.1f}%), "
          f"{len(gaps)} idle gaps totalling {sum(gaps) * 1e-6:.2f} ms")
    for lo, hi in ((0, 5e3), (5e3, 2e4), (2e4, 1e5), (1e5, 1e6), (1e6, 1e12)):
        g = [x for x in gaps if lo <= x < hi]
        print(f"  gaps {lo / 1e3:6.0f}-{hi / 1e3:<8.0f} us: {len(g):5d}  total {sum(g) * 1e-6:8.2f} ms")
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1])[:8]:
        print(f"  {k:42s} {v:9.2f} ms (summed durations)")


if __name__ == "__main__":
    main()
