#!/usr/bin/env python3
"""Plot one candidate (fold sub-integrations, profile, DM/acc hits) -- the
reference's CandidatePlotter (tools/peasoup_tools.py) in Python 3.  Needs
matplotlib; without it the panels are written as .npy arrays instead."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from peasoup_amd.utils.outputs import PeasoupOutput  # noqa: E402


def main() -> int:
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument("outdir")
    p.add_argument("index", type=int)
    p.add_argument("-o", "--output", default=None)
    a = p.parse_args()
    out = PeasoupOutput(os.path.join(a.outdir, "overview.xml"), os.path.join(a.outdir, "candidates.peasoup"))
    c = out.get_candidate(a.index)
    base = a.output or os.path.join(a.outdir, f"cand_{a.index:04d}")
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        if c.fold is not None:
            np.save(base + "_fold.npy", c.fold)
        np.save(base + "_hits.npy", c.hits)
        print(f"matplotlib not available; wrote {base}_fold.npy / _hits.npy")
        return 0
    fig, ax = plt.subplots(2, 2, figsize=(10, 8))
    if c.fold is not None:
        ax[0, 0].imshow(c.fold, aspect="auto", origin="lower")
        ax[0, 0].set_title("sub-integrations")
        ax[1, 0].plot(np.concatenate([c.fold.sum(0)] * 2))
        ax[1, 0].set_title("profile")
    ax[0, 1].scatter(c.hits["dm"], c.hits["snr"], s=6)
    ax[0, 1].set_xlabel("DM")
    ax[1, 1].scatter(c.hits["acc"], c.hits["snr"], s=6)
    ax[1, 1].set_xlabel("acc (m/s^2)")
    fig.suptitle(f"P={c.info['period']:.9f}s DM={c.info['dm']:.2f} S/N={c.info['snr']:.1f} fold S/N={c.info['folded_snr']:.1f}")
    fig.savefig(base + ".png")
    print(base + ".png")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
