#!/usr/bin/env python3
"""Idle gaps of a rocprofv3 kernel trace (the last 40% of the timeline): busy
fraction, idle time by the kernels around each gap, the largest gaps."""
import csv, sys, re
rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), re.sub(r"^void |psoup::kern::|\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0][:50], r["Queue_Id"]) for r in rows)
# last 3 steps: take the final 40% of the timeline
t0 = ev[int(len(ev)*0.6)][0]; ev = [e for e in ev if e[0] >= t0]
end = ev[0][0]; gaps = []
busy = 0
prev = None
for s, e, n, q in ev:
    if s > end:
        gaps.append((s - end, prev, n))
    if e > end:
        busy += e - max(s, end); end = e
    prev = n
span = ev[-1][1] - ev[0][0]
print(f"span {span/1e6:.2f} ms busy {busy/span:.1%} kernels {len(ev)}")
gaps.sort(reverse=True)
tot = sum(g for g, _, _ in gaps)
print(f"idle {tot/1e6:.2f} ms in {len(gaps)} gaps")
from collections import Counter
c = Counter()
for g, a, b in gaps:
    c[(a, b)] += g
for (a, b), g in c.most_common(12):
    print(f"{g/1e6:7.3f} ms  after {a}  before {b}")
print("--- largest gaps")
ev2 = ev
end = ev2[0][0]; prevn = None
lst = []
for i, (s, e, n, q) in enumerate(ev2):
    if s > end + 20000:
        lst.append((s - end, i))
    end = max(end, e)
for g, i in sorted(lst, reverse=True)[:8]:
    ctx = ev2[max(0, i-3):i+2]
    print(f"gap {g/1e3:.0f} us at +{(ev2[i][0]-ev2[0][0])/1e3:.0f} us:", " | ".join(f"{x[2][:40]}(q{x[3]},{(x[1]-x[0])/1e3:.0f}us)" for x in ctx))
