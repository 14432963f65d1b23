#!/usr/bin/env python3
"""CPU microbenchmark of the per-trial harmonic distiller (the engine's
settings: tol 1e-4, 16 harmonics, fractional, no kept relations) on
synthetic trials: harmonics of a few bright fundamentals at every sum level
plus unrelated crossings.  Checks the indexed path against the O(n^2) scan."""
import sys
import os
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from peasoup_amd import _C  # noqa: E402


def trial(rng, n, nfund=3):
    c = []
    f0s = rng.uniform(0.5, 300.0, nfund)
    for i in range(n):
        nh = int(rng.integers(0, 4))
        if rng.random() < 0.7:
            f = f0s[i % nfund] * int(rng.integers(1, 40)) / (1 << int(rng.integers(0, nh + 1))) * (1 + 2e-5 * rng.standard_normal())
        else:
            f = rng.uniform(0.1, 1100.0)
        c.append(_C.Candidate(10.0, 3, 0.0, nh, float(9 + 200 * rng.random()), float(f)))
    return c


def main():
    rng = np.random.default_rng(1)
    hd = _C.HarmonicDistiller(1e-4, 16.0, False, True)
    for n in (16, 64, 200, 1000, 5000):
        trials = [trial(rng, n) for _ in range(max(3, 20000 // n))]
        t0 = time.perf_counter()
        outs = [hd.distill(t) for t in trials]
        dt = (time.perf_counter() - t0) / len(trials)
        ok = all([(x.freq, x.snr) for x in a] == [(x.freq, x.snr) for x in hd.distill_reference(t)]
                 for a, t in zip(outs[:3], trials[:3]))
        print(f"n={n:5d}  {dt * 1e6:9.1f} us/trial  {dt * 1e9 / n:8.1f} ns/cand  kept {np.mean([len(o) for o in outs]):7.1f}"
              f"  equal_to_scan={ok}", flush=True)


if __name__ == "__main__":
    main()
