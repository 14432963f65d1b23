#!/usr/bin/env python3
"""Print selected fields (dotted paths into nested dicts) of each JSON line:
    summarize_jsonl.py FILE field [field.sub ...]"""
import json
import sys


def get(d, path):
    for k in path.split("."):
        if isinstance(d, list) and k.isdigit() and int(k) < len(d):
            d = d[int(k)]
        elif isinstance(d, dict):
            d = d.get(k)
        else:
            return None
    return d


for line in open(sys.argv[1]):
    line = line.strip()
    if line.startswith("{"):
        d = json.loads(line)
        print("  ".join(f"{f}={get(d, f)}" for f in sys.argv[2:]))
