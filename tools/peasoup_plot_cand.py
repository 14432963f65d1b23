#!/usr/bin/env python3
"""Candidate diagnostic plots of a peasoup output directory (the reference's
CandidatePlotter, tools/peasoup_tools.py:167-412): profile, sub-integrations,
sub-integration statistics, info table, DM / acceleration / S/N scatters of
the associated hits, DM-acceleration map, every candidate in period-DM space.

    peasoup_plot_cand.py OUTDIR [INDEX ...] [-o FILE] [--all N] [--predictor]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from peasoup_amd.utils.plotting import CandidatePlotter, plot_all  # noqa: E402


def main() -> int:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("outdir")
    p.add_argument("index", type=int, nargs="*")
    p.add_argument("-o", "--output", default=None, help="file name (one index only)")
    p.add_argument("--all", type=int, default=0, help="plot the first N candidates as Cand%%04d.png")
    p.add_argument("--predictor", action="store_true", help="print each candidate's predictor instead")
    a = p.parse_args()
    if a.all:
        for f in plot_all(a.outdir, a.all):
            print(f)
        return 0
    pl = CandidatePlotter(a.outdir)
    for i in a.index or [0]:
        if a.predictor:
            print(pl.overview.make_predictor(i))
            continue
        out = a.output if (a.output and len(a.index) <= 1) else os.path.join(a.outdir, "Cand%04d.png" % i)
        print(pl.plot_cand(i, out))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
