#!/usr/bin/env python3
"""kFft4WideStockham: the fused spectrum pass's P and Q with the lane-pair
16-byte Y stores in the Stockham pass A equal the default's bit for bit.
    python tools/expt/wide_stockham_check.py FLAGS_A FLAGS_B"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from peasoup_amd import _C, ops  # noqa: E402


def main():
    fa, fb = int(sys.argv[1]), int(sys.argv[2])
    for log2n in (17, 20, 21, 22, 25):
        n = 1 << log2n
        x = torch.randn(n, device="cuda")
        st = torch.tensor([1.0, 2.0, 0.5, 0.0], dtype=torch.float32, device="cuda")
        accs = [-410.0, -7.0, 0.0, 250.0, 499.0]
        out = []
        for f in (fa, fb):
            _C.kernels.fft4_set_flags(f)
            Pb, Q, g = ops.fft4_spectrum_pass(x, accs, 64e-6, st, float(n))
            out.append((Pb.cpu().numpy(), Q.cpu().numpy()))
        same = np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
        print(f"2^{log2n}: P, Q identical: {same}", flush=True)
        assert same
    _C.kernels.fft4_set_flags(fa)


if __name__ == "__main__":
    main()
