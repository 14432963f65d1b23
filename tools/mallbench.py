#!/usr/bin/env python3
"""Per-kernel time of the fused-FFT search chain (colpass -> rowpass -> r2c ->
harmonic) as a function of the trial batch K, with HIP events between the
kernels: does re-reading an intermediate right after it was written (small K,
Infinity-Cache resident) beat streaming it through HBM (large K)?

    python tools/mallbench.py [--log2n 23] [--Ks 1,2,4,8,16,32,64] [--reps 6]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from peasoup_amd import _C  # noqa: E402

K_ = _C.kernels


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=23)
    ap.add_argument("--Ks", default="1,2,4,8,16,32,64")
    ap.add_argument("--reps", type=int, default=6)
    a = ap.parse_args()
    dev = torch.device("cuda")
    n = 1 << a.log2n
    M = n // 2
    s = torch.cuda.current_stream().cuda_stream
    g = K_.fft4_geometry(M)
    x = torch.randn(n, device=dev)
    tab = torch.from_numpy(K_.fft4_tables(g)).to(dev)
    xp = torch.empty(g.insize, device=dev)
    K_.fft4_pad_input(x.data_ptr(), n, xp.data_ptr(), g, s)
    st = torch.tensor([1.0, 2.0, 0.5, 0.0], device=dev)
    nb = M + 1
    cap = 1 << 20
    out = torch.empty(cap * 3, dtype=torch.int32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    for K in [int(v) for v in a.Ks.split(",")]:
        accs = 200.0 + 1.464 * np.arange(K)  # consecutive legacy-plan steps at 2^23 x 64 us (as in a real batch)
        af = torch.tensor([v * 64e-6 / (2 * 299792458.0) for v in accs], dtype=torch.float64, device=dev)
        Y = torch.empty(K * g.ystride * 2, device=dev)
        X = torch.empty(K * g.xstride * 2, device=dev)
        P = torch.empty(K * nb, device=dev)
        steps = [
            ("colpass", lambda: K_.fft4_resample_colpass(x.data_ptr(), xp.data_ptr(), n, af.data_ptr(), K,
                                                         Y.data_ptr(), g, tab.data_ptr(), s)),
            ("rowpass", lambda: K_.fft4_rowpass(Y.data_ptr(), X.data_ptr(), K, g, tab.data_ptr(), s)),
            ("r2c", lambda: K_.r2c_interbin_normalise_tiled(X.data_ptr(), g.n1, g.n2, g.xstride, P.data_ptr(), nb,
                                                            K, nb, st.data_ptr(), float(n), s)),
            ("harm", lambda: K_.harmonic_peaks_batch(P.data_ptr(), nb, nb, K, 3, [1, 2, 4, 8, 16], [nb] * 5, 9.0,
                                                     cap, out.data_ptr(), cnt.data_ptr(), s)),
        ]
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(steps) + 1)]
        tot = np.zeros(len(steps))
        reps = max(2, a.reps * 32 // (K * 4)) if K < 32 else a.reps
        for r in range(reps + 1):
            ev[0].record()
            for i, (_, fn) in enumerate(steps):
                fn()
                ev[i + 1].record()
            torch.cuda.synchronize()
            if r:
                tot += [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(len(steps))]
        per = tot / reps / K
        print(f"K={K:3d} " + " ".join(f"{nm}={v:6.2f}" for (nm, _), v in zip(steps, per)) +
              f"  sum={per.sum():6.2f} us/trial", flush=True)
        del Y, X, P


if __name__ == "__main__":
    main()
