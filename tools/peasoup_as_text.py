#!/usr/bin/env python3
"""Print a peasoup output directory as a text table (tools/peasoup_as_text.py
of the reference, Python 3)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from peasoup_amd.utils.outputs import PeasoupOutput  # noqa: E402


def main() -> int:
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("outdir", help="directory holding overview.xml and candidates.peasoup")
    p.add_argument("--hits", action="store_true", help="also list every associated detection")
    a = p.parse_args()
    out = PeasoupOutput(os.path.join(a.outdir, "overview.xml"), os.path.join(a.outdir, "candidates.peasoup"))
    print(out.as_text())
    if a.hits:
        for i in range(len(out)):
            c = out.get_candidate(i)
            print(f"# candidate {i}: {len(c.hits)} detections")
            for h in c.hits:
                print(f"   dm={h['dm']:.3f} dm_idx={h['dm_idx']} acc={h['acc']:.3f} nh={h['nh']} "
                      f"snr={h['snr']:.2f} freq={h['freq']:.9f}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
