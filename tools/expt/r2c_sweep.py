#!/usr/bin/env python3
"""Tiled r2c + interbin + normalise kernel at the headline size (K trials of
M = 2^22 complex): LDS-plane vs cross-lane-shuffle neighbour exchange and an
occupancy cap (harmonic_set_flags bits 16-23); outputs checked bit-identical.  One stream.

    python tools/expt/r2c_sweep.py [--K 32] [--reps 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from peasoup_amd import _C  # noqa: E402

K_ = _C.kernels


def timeit(fn, reps):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=23)
    ap.add_argument("--K", type=int, default=32)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda")
    M = 1 << (a.log2n - 1)
    K = a.K
    s = torch.cuda.current_stream().cuda_stream
    g = K_.fft4_geometry(M)
    X = torch.randn(K * g.xstride * 2, device=dev)
    pstride = (M + 1 + 63) // 64 * 64
    P = torch.empty(K * pstride, device=dev)
    st = torch.tensor([1.0, 2.0, 0.5, 0.0], device=dev)

    def r2c():
        K_.r2c_interbin_normalise_tiled(X.data_ptr(), g.n1, g.n2, g.xstride, P.data_ptr(), pstride, K, M + 1,
                                        st.data_ptr(), float(1 << a.log2n), s)

    K_.harmonic_set_flags(1 | 16)  # LDS-plane kernel: the reference output
    P.zero_()
    r2c()
    torch.cuda.synchronize()
    ref = P.clone()
    # LDS-plane kernel: static LDS ~33 KiB = 4 workgroups/CU (+20 KiB -> 3);
    # shuffle kernel: register-bound occupancy
    for name, fl in [("lds planes (4 WG/CU)", 1 | 16), ("lds planes 3 WG/CU", 1 | 16 | (20 << 16)),
                     ("shuffles", 1), ("lds planes (4 WG/CU)", 1 | 16), ("shuffles", 1)]:
        K_.harmonic_set_flags(fl)
        P.zero_()
        us = timeit(r2c, a.reps)
        torch.cuda.synchronize()
        same = torch.equal(P, ref)
        if not same:
            d = (P != ref).nonzero().flatten()
            kk, bins = d // pstride, d % pstride
            col, row = bins % g.n2, bins // g.n2
            print(f"  {d.numel()} differ; max |diff| {float((P - ref).abs().max()):.3g}; "
                  f"trials {kk.unique()[:5].tolist()}; first bins {bins[:8].tolist()}; "
                  f"columns mod 256 {torch.bincount(col % 256, minlength=256).nonzero().flatten()[:16].tolist()}; "
                  f"rows {row[:8].tolist()}", flush=True)
        print(f"r2c tiled {name:22s} {us:9.1f} us/launch {us / K:7.2f} us/trial "
              f"{K * 12 * M / us / 1e3:7.0f} GB/s  {'identical' if same else 'DIFFERS'}", flush=True)
    K_.harmonic_set_flags(1)


if __name__ == "__main__":
    main()
