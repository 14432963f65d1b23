#!/usr/bin/env python3
"""Per-kernel microbenchmark of the acceleration-search hot path at the
headline size (2^23-point series, K trials per batch), with HIP-event timing.

    python tools/kbench.py [--log2n 23] [--K 32] [--reps 10] [--flags 0,1,259,3331]

Prints one line per (kernel, variant): time per launch, per trial, and the
effective HBM bandwidth of the bytes the kernel must move.
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
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
    return e0.elapsed_time(e1) * 1e3 / reps  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=23)
    ap.add_argument("--K", type=int, default=32)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--flags", default="")
    a = ap.parse_args()
    dev = torch.device("cuda")
    n = 1 << a.log2n
    M = n // 2
    K = a.K
    s = torch.cuda.current_stream().cuda_stream
    g = K_.fft4_geometry(M)
    assert g.ok
    x = torch.randn(n, device=dev)
    tab = torch.from_numpy(K_.fft4_tables(g)).to(dev)
    tsamp = 64e-6
    accs = 200.0 + 1.464 * np.arange(K)  # consecutive legacy-plan steps at 2^23 x 64 us (as in a real batch)
    af = torch.tensor([a_ * tsamp / (2 * 299792458.0) for a_ in accs], dtype=torch.float64, device=dev)
    xp = torch.empty(g.insize, device=dev)
    Y = torch.empty(K * g.ystride * 2, device=dev)
    X = torch.empty(K * g.xstride * 2, device=dev)
    P = torch.empty(K * (M + 1), device=dev)
    st = torch.tensor([1.0, 2.0, 0.5, 0.0], device=dev)
    GB = 1e9
    rows = []

    def report(name, us, nbytes):
        rows.append((name, us))
        print(f"{name:44s} {us:9.1f} us/launch {us / K:8.2f} us/trial {nbytes / (us * 1e-6) / GB:8.0f} GB/s",
              flush=True)

    big = torch.empty(K * M * 2, device=dev)
    big2 = torch.empty_like(big)
    report("torch copy (K*M complex)", timeit(lambda: big2.copy_(big), a.reps), 2 * big.numel() * 4)
    del big, big2
    K_.fft4_pad_input(x.data_ptr(), n, xp.data_ptr(), g, s)
    report("pad_input", timeit(lambda: K_.fft4_pad_input(x.data_ptr(), n, xp.data_ptr(), g, s), a.reps) * K,
           2 * 4 * n)
    f_default = K_.fft4_flags()
    for f in [int(v) for v in a.flags.split(",") if v] or [f_default]:
        K_.fft4_set_flags(f)
        tc = timeit(lambda: K_.fft4_resample_colpass(x.data_ptr(), xp.data_ptr(), n, af.data_ptr(), K, Y.data_ptr(), g,
                                                     tab.data_ptr(), s), a.reps)
        report(f"colpass flags={f}", tc, K * 8 * M)
        tr = timeit(lambda: K_.fft4_rowpass(Y.data_ptr(), X.data_ptr(), K, g, tab.data_ptr(), s), a.reps)
        report(f"rowpass flags={f}", tr, K * 16 * M)
    for blk_w in (0, 4, 8):
        row, blk, lw = (g.xpitch, 8, 3) if blk_w == 0 else (blk_w, blk_w * g.n1, blk_w.bit_length() - 1)
        tz = timeit(lambda: K_.r2c_interbin_normalise_batch(X.data_ptr(), M, g.xstride, g.log2_xrow, row, blk, lw,
                                                            P.data_ptr(), M + 1, K, M + 1, st.data_ptr(), float(n), s),
                    a.reps)
        report(f"r2c_interbin_normalise block={blk_w}", tz, K * (8 * M + 4 * M))
    tz = timeit(lambda: K_.r2c_interbin_normalise_tiled(X.data_ptr(), g.n1, g.n2, g.xstride, P.data_ptr(), M + 1, K,
                                                        M + 1, st.data_ptr(), float(n), s), a.reps)
    report("r2c_interbin_normalise tiled", tz, K * (8 * M + 4 * M))
    qs = (M + 1 + 63) // 64 * 64
    Qr = torch.empty(K * qs, dtype=torch.uint8, device=dev)
    tz = timeit(lambda: K_.r2c_interbin_normalise_tiled(X.data_ptr(), g.n1, g.n2, g.xstride, P.data_ptr(), M + 1, K,
                                                        M + 1, st.data_ptr(), float(n), s, Qr.data_ptr(), qs), a.reps)
    report("r2c_interbin_normalise tiled + screening bytes", tz, K * (8 * M + 5 * M))
    del Qr
    K_.fft4_set_flags(f_default)
    # fused spectrum pass (the default search path): Y -> blocked P + Q
    pst = (M + 1 + 63) // 64 * 64
    qst2 = (M + 1 + K_.spec_q_shift + 63) // 64 * 64
    Pb = torch.empty(K * pst, device=dev)
    Qb = torch.empty(K * qst2, dtype=torch.uint8, device=dev)
    tz = timeit(lambda: K_.fft4_rowpass_spectrum(Y.data_ptr(), K, g, tab.data_ptr(), Pb.data_ptr(), pst, Qb.data_ptr(),
                                                 qst2, st.data_ptr(), float(n), s), a.reps)
    for pair in (False, True) if K_.fft4_pair_y(g) else (False,):
        g.ypair = pair
        K_.fft4_resample_colpass(x.data_ptr(), xp.data_ptr(), n, af.data_ptr(), K, Y.data_ptr(), g, tab.data_ptr(), s)
        tz = timeit(lambda: K_.fft4_rowpass_spectrum(Y.data_ptr(), K, g, tab.data_ptr(), Pb.data_ptr(), pst,
                                                     Qb.data_ptr(), qst2, st.data_ptr(), float(n), s), a.reps)
        report(f"rowpass_spectrum ypair={int(pair)}", tz, K * (8 * M + 5 * M))
        if pair:
            tc = timeit(lambda: K_.fft4_resample_colpass(x.data_ptr(), xp.data_ptr(), n, af.data_ptr(), K,
                                                         Y.data_ptr(), g, tab.data_ptr(), s), a.reps)
            report("colpass ypair=1", tc, K * 8 * M)
    g.ypair = False
    del Pb, Qb
    # harmonic peaks on normal noise (threshold 9 -> few peaks)
    P.normal_()
    nb = M + 1
    cap = 1 << 20
    out = torch.empty(cap * 3, dtype=torch.int32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    starts = [1, 2, 4, 8, 16]
    ends = [nb] * 5

    def harm():
        cnt.zero_()
        K_.harmonic_peaks_batch(P.data_ptr(), nb, nb, K, 3, starts, ends, 9.0, cap, out.data_ptr(), cnt.data_ptr(), s)

    hdef = K_.harmonic_flags()
    for hf in (hdef & ~1, hdef):
        K_.harmonic_set_flags(hf)
        th = timeit(harm, a.reps)
        report(f"harmonic_peaks (3 levels, fp32 staging) flags={hf}", th, K * 4 * M)
    qst = (nb + 63) // 64 * 64
    Q = torch.empty(K * qst, dtype=torch.uint8, device=dev)
    K_.quantize_q8(P.data_ptr(), nb, nb, K, Q.data_ptr(), qst, s)

    def harmq():
        cnt.zero_()
        K_.harmonic_peaks_batch(P.data_ptr(), nb, nb, K, 3, starts, ends, 9.0, cap, out.data_ptr(), cnt.data_ptr(), s,
                                Q.data_ptr(), qst)

    th = timeit(harmq, a.reps)
    report("harmonic_peaks (3 levels, screened)", th, K * M)
    K_.harmonic_set_flags(hdef)


if __name__ == "__main__":
    main()
