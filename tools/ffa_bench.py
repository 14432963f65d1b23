#!/usr/bin/env python3
"""FFA search throughput on one GPU: DM trials/s for a synthetic dedispersed
series (u8 noise + a long-period pulse train) of 2^log2n samples.

    python tools/ffa_bench.py [--log2n 23] [--tsamp 64e-6] [--p_start 0.8] [--p_end 20] [--min_dc 0.001] [--dms 4]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from peasoup_amd import _C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=23)
    ap.add_argument("--tsamp", type=float, default=64e-6)
    ap.add_argument("--p_start", type=float, default=0.8)
    ap.add_argument("--p_end", type=float, default=20.0)
    ap.add_argument("--min_dc", type=float, default=0.001)
    ap.add_argument("--dms", type=int, default=4)
    a = ap.parse_args()
    n = 1 << a.log2n
    p = _C.FfaParams()
    p.tsamp, p.p_start, p.p_end, p.min_dc = a.tsamp, a.p_start, a.p_end, a.min_dc
    s = torch.cuda.current_stream().cuda_stream
    eng = _C.FfaEngine(p, n, s)
    rng = np.random.default_rng(0)
    t = np.arange(n) * a.tsamp
    ph = (t / 3.3) % 1.0
    x = rng.normal(128, 8, n) + 6.0 * (np.minimum(ph, 1 - ph) < 0.005)
    trial = torch.from_numpy(np.clip(np.rint(x), 0, 255).astype(np.uint8)).cuda()
    eng.search(trial.data_ptr(), 10.0, 0)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for d in range(a.dms):
        c = eng.search(trial.data_ptr(), 10.0, d)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.dms
    best = c[0] if c else None
    print(json.dumps({"metric": "FFA DM trials/s", "value": round(1.0 / dt, 3), "ms_per_dm": round(1e3 * dt, 3),
                      "log2n": a.log2n, "profiles_per_dm": eng.profiles // (a.dms + 1), "base_bins": _C.ffa_base_bins(p),
                      "best_period": best.period if best else None, "best_snr": best.snr if best else None}))


if __name__ == "__main__":
    main()
