#!/usr/bin/env python3
"""Pass A (one-exchange fused resample + column pass) phase costs at the
headline size: the full kernel and variants with its global loads, its FFT
arithmetic/exchange or its stores removed (timing flags), so the overlap of
the phases can be read off.  HIP-event timing, K trials per launch."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from peasoup_amd import _C  # noqa: E402

K_ = _C.kernels
SKIP_COMPUTE, SKIP_LOAD, SKIP_STORE = 8, 64, 128


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
    ap.add_argument("--extra", default="0", help="comma list of extra flag bits OR-ed onto the default")
    ap.add_argument("--only-full", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    n = 1 << a.log2n
    M, K = n // 2, a.K
    s = torch.cuda.current_stream().cuda_stream
    base = K_.fft4_flags()
    g = K_.fft4_geometry(M)
    x = torch.randn(n, device=dev)
    tab = torch.from_numpy(K_.fft4_tables(g)).to(dev)
    accs = 200.0 + 1.464 * np.arange(K)
    af = torch.tensor([v * 64e-6 / (2 * 299792458.0) for v in accs], dtype=torch.float64, device=dev)
    xp = torch.empty(g.insize, device=dev)
    Y = torch.empty(K * g.ystride * 2, device=dev)
    K_.fft4_pad_input(x.data_ptr(), n, xp.data_ptr(), g, s)
    for extra in [int(v) for v in a.extra.split(",")]:
        for name, f in (("full", 0), ("no loads", SKIP_LOAD), ("no stores", SKIP_STORE), ("no compute", SKIP_COMPUTE),
                        ("loads only", SKIP_COMPUTE | SKIP_STORE), ("stores only", SKIP_COMPUTE | SKIP_LOAD),
                        ("compute only", SKIP_LOAD | SKIP_STORE))[: 1 if a.only_full else 7]:
            K_.fft4_set_flags(base | extra | f)
            K_.fft4_pad_input(x.data_ptr(), n, xp.data_ptr(), g, s)  # the input layout follows the flags
            t = timeit(lambda: K_.fft4_resample_colpass(x.data_ptr(), xp.data_ptr(), n, af.data_ptr(), K, Y.data_ptr(),
                                                        g, tab.data_ptr(), s), a.reps)
            print(f"extra={extra:<8d} {name:14s} {t:9.1f} us/launch {t / K:7.2f} us/trial", flush=True)
    K_.fft4_set_flags(base)


if __name__ == "__main__":
    main()
