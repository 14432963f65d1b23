#!/usr/bin/env python3
"""Stage times of repeated runs of the golden command next to the reference's.

    python tools/golden_times.py gpurun_out/r4async/golden_native_* -- gpurun_out/r4async/golden_py_*

Each argument is an output directory of
`peasoup -i tests/data/tutorial.fil --dm_end 250 --acc_start -5 --acc_end 5 -n 4 --npdmp 10`
(native bin/peasoup before `--`, the Python driver after it).  Prints a
markdown table: per stage the median (min-max) over the runs and the ratio of
the reference's time (tests/data/golden_overview.xml:295-301, two Tesla C2070)
to the median.  The first run of a process pays the code-object load, so it is
shown separately as `first`."""
import statistics
import sys
import xml.etree.ElementTree as ET
from pathlib import Path

STAGES = ("reading", "dedispersion", "searching", "folding", "total")
REPO = Path(__file__).resolve().parents[1]


def times(d):
    root = ET.parse(Path(d) / "overview.xml").getroot()
    et = root.find("execution_times")
    return {s: float(et.find(s).text) for s in STAGES}


def main(argv):
    root = ET.parse(REPO / "tests" / "data" / "golden_overview.xml").getroot()
    et = root.find("execution_times")
    ref = {s: float(et.find(s).text) for s in STAGES}
    groups, cur = [[]], 0
    for a in argv:
        if a == "--":
            groups.append([])
            cur += 1
        else:
            groups[cur].append(a)
    names = ["native bin/peasoup", "Python driver (1 rank)"]
    for name, dirs in zip(names, groups):
        if not dirs:
            continue
        runs = [times(d) for d in sorted(dirs) if Path(d).is_dir()]
        print(f"\n### {name}: {len(runs)} runs\n")
        print("| stage | C2070 (s) | MI355X median (s) | min - max | first run | C2070 / MI355X |")
        print("|---|---|---|---|---|---|")
        for s in STAGES:
            v = [r[s] for r in runs]
            rest = v[1:] if len(v) > 1 else v
            med = statistics.median(rest)
            ratio = ref[s] / med if med > 0 else float("inf")
            print(f"| {s} | {ref[s]:.4f} | {med:.4f} | {min(rest):.4f} - {max(rest):.4f} | {v[0]:.4f} | {ratio:.1f}x |")


if __name__ == "__main__":
    main(sys.argv[1:])
