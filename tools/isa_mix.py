#!/usr/bin/env python3
"""Instruction mix of kernels in a hipcc -S listing: tools/isa_mix.py file.s substr [substr...]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read().split("\n")
for key in sys.argv[2:]:
    start = next(i for i, l in enumerate(s) if re.match(r"^_Z\S*" + re.escape(key) + r"\S*:", l))
    c = Counter()
    for l in s[start + 1:]:
        t = l.strip()
        if t.startswith("s_endpgm"):
            break
        if not t or t.startswith((".", ";", "/")) or t.endswith(":"):
            continue
        c[t.split()[0]] += 1
    meta = [l for l in s[start:] if re.match(r"\s*; (NumVgprs|Occupancy|NumAgprs|LDSByteSize):", l)][:4]
    tot = sum(c.values())
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    print(f"{key}: {tot} instrs, {valu} VALU; " + " ".join(m.strip() for m in meta))
    print("  " + ", ".join(f"{k} {v}" for k, v in c.most_common(24)))
