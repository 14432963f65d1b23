#!/usr/bin/env python3
"""Microbenchmark of the fused pass B (fft4_rowpass_r2c, kFft4FusedR2c)
against the unfused pass B + tiled r2c, and of the harmonic sum on the
natural vs the fused pass's blocked spectrum layout, at the headline size.

    python tools/kbench_fused.py [--log2n 23] [--K 32] [--reps 10]

One line per kernel: time per launch, per trial, effective bandwidth of the
bytes the kernel must move (HIP-event timing, one stream).
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from peasoup_amd import _C  # noqa: E402

K_ = _C.kernels
FUSED = 2097152


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=23)
    ap.add_argument("--K", type=int, default=32)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda")
    n = 1 << a.log2n
    M = n // 2
    K = a.K
    s = torch.cuda.current_stream().cuda_stream
    base_flags = K_.fft4_flags()
    K_.fft4_set_flags(base_flags | FUSED)
    g = K_.fft4_geometry(M)
    assert g.ok and K_.fft4_fused_r2c_ok(g)
    x = torch.randn(n, device=dev)
    tab = torch.from_numpy(K_.fft4_tables(g)).to(dev)
    tsamp = 64e-6
    accs = 200.0 + 1.464 * np.arange(K)
    af = torch.tensor([a_ * tsamp / (2 * 299792458.0) for a_ in accs], dtype=torch.float64, device=dev)
    xp = torch.empty(g.insize, device=dev)
    Y = torch.empty(K * g.ystride * 2, device=dev)
    X = torch.empty(K * g.xstride * 2, device=dev)
    pst = (M + 4 + 7) // 8 * 8
    P = torch.empty(K * pst, device=dev)
    Pb = torch.empty(K * pst, device=dev)
    st = torch.tensor([0.0, 1.0, float(np.sqrt(M)) / n, 0.0], device=dev)
    GB = 1e9

    def report(name, us, nbytes):
        print(f"{name:44s} {us:9.1f} us/launch {us / K:8.2f} us/trial {nbytes / (us * 1e-6) / GB:8.0f} GB/s",
              flush=True)

    K_.fft4_pad_input(x.data_ptr(), n, xp.data_ptr(), g, s)
    tc = timeit(lambda: K_.fft4_resample_colpass(x.data_ptr(), xp.data_ptr(), n, af.data_ptr(), K, Y.data_ptr(), g,
                                                 tab.data_ptr(), s), a.reps)
    report("colpass", tc, K * 8 * M)
    tr = timeit(lambda: K_.fft4_rowpass(Y.data_ptr(), X.data_ptr(), K, g, tab.data_ptr(), s, M + 1), a.reps)
    report("rowpass (unfused)", tr, K * 16 * M)
    tz = timeit(lambda: K_.r2c_interbin_normalise_tiled(X.data_ptr(), g.n1, g.n2, g.xstride, P.data_ptr(), pst, K,
                                                        M + 1, st.data_ptr(), float(n), s), a.reps)
    report("r2c tiled (unfused)", tz, K * 12 * M)
    report("  rowpass + r2c", tr + tz, K * 28 * M)
    tf = timeit(lambda: K_.fft4_rowpass_r2c(Y.data_ptr(), Pb.data_ptr(), pst, K, g, tab.data_ptr(), st.data_ptr(),
                                            float(n), M + 1, s), a.reps)
    report("rowpass_r2c (fused)", tf, K * (8 * M * 9 // 8 + 4 * M))
    lay = K_.fft4_p_layout(g)
    tu = timeit(lambda: K_.p_unblock(Pb.data_ptr(), P.data_ptr(), pst, K, lay, M + 1, s), a.reps)
    report("p_unblock (blocked -> natural)", tu, K * 8 * M)
    report("  fused + unblock", tf + tu, K * (8 * M * 9 // 8 + 12 * M))
    # harmonic sum on both layouts (the same spectra)
    K_.p_relayout(Pb.data_ptr(), P.data_ptr(), pst, K, lay, 1, s)
    nat = _C.kernels.PLayout()
    cap = 1 << 22
    out = torch.empty(cap * 3, dtype=torch.int32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    nb = M + 1
    df = 1.0 / (n * tsamp)
    starts = [int(0.1 / df * (1 << h)) for h in range(6)]
    ends = [min(nb, int(1100.0 / df * (1 << h))) for h in range(6)]
    for name, buf, layout in (("natural", P, nat), ("blocked", Pb, lay)):
        def harm():
            cnt.zero_()
            K_.harmonic_peaks_batch(buf.data_ptr(), nb, pst, K, 3, starts, ends, 9.0, cap, out.data_ptr(),
                                    cnt.data_ptr(), s, layout)
        th = timeit(harm, a.reps)
        report(f"harmonic_peaks n=3 {name} (peaks {int(cnt.item())})", th, K * 4 * M)
    K_.fft4_set_flags(base_flags)


if __name__ == "__main__":
    main()
