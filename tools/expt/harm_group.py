#!/usr/bin/env python3
"""Experiment: r2c+interbin and harmonic-sum kernels run over a 32-trial batch
either as two whole-batch launches or interleaved in groups of G trials
(r2c(G) -> harm(G) -> next group), so each group's P (G x 16.7 MB at 2^23)
is re-read while it is still in the 256 MB Infinity Cache.  Also the harmonic
kernel alone on P sets of K trials, re-run back to back (P resident in MALL
when K x 16.7 MB << 256 MB)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from peasoup_amd import _C  # noqa: E402

K_ = _C.kernels


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    dev = torch.device("cuda")
    n = 1 << 23
    M = n // 2
    K = 32
    s = torch.cuda.current_stream().cuda_stream
    g = K_.fft4_geometry(M)
    X = torch.randn(K * g.xstride * 2, device=dev)
    nb = M + 1
    P = torch.empty(K * nb, device=dev)
    st = torch.tensor([0.0, 1.0, 1000.0, 0.0], device=dev)
    cap = 1 << 20
    out = torch.empty(cap * 3, dtype=torch.int32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    starts = [1, 2, 4, 8, 16]
    ends = [nb] * 5

    def r2c(k0, k):
        K_.r2c_interbin_normalise_tiled(X.data_ptr() + 8 * k0 * g.xstride, g.n1, g.n2, g.xstride,
                                        P.data_ptr() + 4 * k0 * nb, nb, k, nb, st.data_ptr(), float(n), s)

    def harm(k0, k):
        K_.harmonic_peaks_batch(P.data_ptr() + 4 * k0 * nb, nb, nb, k, 3, starts, ends, 9.0, cap, out.data_ptr(),
                                cnt.data_ptr(), s)

    r2c(0, K)
    torch.cuda.synchronize()
    print(f"P stats: mean {P.mean().item():.3f} std {P.std().item():.3f}", flush=True)
    t_r = timeit(lambda: r2c(0, K))
    t_h = timeit(lambda: harm(0, K))
    print(f"whole batch: r2c {t_r / K:.2f} us/trial  harm {t_h / K:.2f} us/trial  sum {(t_r + t_h) / K:.2f}", flush=True)
    for G in (1, 2, 4, 8, 16):
        def grouped():
            for k0 in range(0, K, G):
                r2c(k0, G)
                harm(k0, G)
        t = timeit(grouped)
        print(f"groups of {G:2d}: r2c+harm {t / K:.2f} us/trial", flush=True)
    for Kh in (1, 2, 4, 8, 16, 32):
        t = timeit(lambda: harm(0, Kh), reps=20)
        print(f"harm alone K={Kh:2d} (P {Kh * nb * 4 / 2**20:.0f} MiB, re-run): {t / Kh:.2f} us/trial", flush=True)
    for Kr in (1, 2, 4, 8, 16, 32):
        t = timeit(lambda: r2c(0, Kr), reps=20)
        print(f"r2c alone K={Kr:2d}: {t / Kr:.2f} us/trial", flush=True)


if __name__ == "__main__":
    main()
