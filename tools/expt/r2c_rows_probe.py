#!/usr/bin/env python3
"""Time r2c_interbin_normalise_rows alone at 2^26 points (M = 2^25 = 4096 rows
x 8192): all bins vs a search limit, with and without the screening bytes.
    python tools/expt/r2c_rows_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from peasoup_amd import _C  # noqa: E402


def main():
    dev = torch.device("cuda")
    n2, n1 = 4096, 8192
    M = n1 * n2
    zp = n1 + 8
    K = 4
    s = torch.cuda.current_stream().cuda_stream
    Z = torch.randn(K * n2 * zp * 2, device=dev)
    pst = (M + 1 + 63) // 64 * 64
    P = torch.empty(K * pst, device=dev)
    Q = torch.empty(K * pst, dtype=torch.uint8, device=dev)
    st = torch.tensor([1.0, 2.0, 0.5, 0.0], device=dev)
    for nbo in (M + 1, 4_700_000):
        for q in (0, Q.data_ptr()):
            fn = lambda: _C.kernels.r2c_interbin_normalise_rows(Z.data_ptr(), zp, n2 * zp, 12, n1, P.data_ptr(),  # noqa
                                                                pst, K, nbo, st.data_ptr(), 1.0, s, q, pst)
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = 1e3 * e0.elapsed_time(e1) / 5 / K
            print(f"nbins_out {nbo}: Q {'on' if q else 'off'}: {us:.1f} us per trial", flush=True)


if __name__ == "__main__":
    main()
