#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 SQLite output (``*_results.db``):
the same table ``rocprofv3 --stats`` prints, for runs that only wrote the
database.  Kernel names are shortened to the function name plus template
arguments.

    python tools/rocpd_stats.py gpurun_out/r3/prof_forcepg/forcepg_results.db [--top 30] [--grep nccl]
"""
import argparse
import re
import sqlite3


def short(name: str) -> str:
    if name.endswith(")"):  # drop the parameter list (matching parenthesis from the end)
        depth = 0
        for i in range(len(name) - 1, -1, -1):
            depth += {")": 1, "(": -1}.get(name[i], 0)
            if depth == 0:
                name = name[:i]
                break
    name = name.replace("psoup::kern::(anonymous namespace)::", "")
    return name.replace("void ", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--grep", default=None, help="only kernels whose name matches (regex, case-insensitive)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels "
                     "order by total_duration desc").fetchall()
    if a.grep:
        rows = [r for r in rows if re.search(a.grep, r[0], re.I)]
    total = sum(r[2] for r in rows)
    # top_kernels reports durations in microseconds
    print(f"{'kernel':70s} {'calls':>7s} {'total ms':>10s} {'avg us':>9s} {'%':>6s}")
    for name, calls, tot, avg, pct in rows[:a.top]:
        print(f"{short(name)[:70]:70s} {calls:7d} {tot / 1e3:10.3f} {avg:9.2f} {pct:6.2f}")
    print(f"{'(listed total)':70s} {sum(r[1] for r in rows):7d} {total / 1e3:10.3f}")


if __name__ == "__main__":
    main()
