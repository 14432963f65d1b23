#!/usr/bin/env python3
"""Per-trial times of the two fused FFT passes of the headline search path
(pass A with row-pair Y, the fused spectrum pass) at K trials of 2^23 points,
for one fft4 flag set.   python tools/kbench_fused.py --flags F [--K 32]"""
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
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags", type=int, default=-1)
    ap.add_argument("--K", type=int, default=32)
    ap.add_argument("--log2n", type=int, default=23)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    if a.flags >= 0:
        K_.fft4_set_flags(a.flags)
    dev = torch.device("cuda")
    n = 1 << a.log2n
    M = n // 2
    K = a.K
    s = torch.cuda.current_stream().cuda_stream
    g = K_.fft4_geometry(M)
    g.ypair = K_.fft4_pair_y(g)
    x = torch.randn(n, device=dev)
    tab = torch.from_numpy(K_.fft4_tables(g)).to(dev)
    accs = 200.0 + 1.464 * np.arange(K)
    af = torch.tensor([a_ * 64e-6 / (2 * 299792458.0) for a_ in accs], dtype=torch.float64, device=dev)
    xp = torch.empty(g.insize, device=dev)
    K_.fft4_pad_input(x.data_ptr(), n, xp.data_ptr(), g, s)
    Y = torch.empty(K * g.ystride * 2, device=dev)
    pst = (M + 1 + 63) // 64 * 64
    qst = (M + 1 + K_.spec_q_shift + 63) // 64 * 64
    Pb = torch.empty(K * pst, device=dev)
    Qb = torch.empty(K * qst, dtype=torch.uint8, device=dev)
    st = torch.tensor([1.0, 2.0, 0.5, 0.0], device=dev)
    col = lambda: K_.fft4_resample_colpass(x.data_ptr(), xp.data_ptr(), n, af.data_ptr(), K, Y.data_ptr(), g,
                                           tab.data_ptr(), s)
    spec = lambda: K_.fft4_rowpass_spectrum(Y.data_ptr(), K, g, tab.data_ptr(), Pb.data_ptr(), pst, Qb.data_ptr(), qst,
                                            st.data_ptr(), float(n), s)
    tc = timeit(col, a.reps)
    tsp = timeit(spec, a.reps)
    both = timeit(lambda: (col(), spec()), a.reps)
    f = K_.fft4_flags()
    print(f"flags={f} log2n={a.log2n} K={K}: pass A {tc / K:.2f} us/trial, spectrum pass {tsp / K:.2f} us/trial, "
          f"both {both / K:.2f} us/trial", flush=True)


if __name__ == "__main__":
    main()
