#!/usr/bin/env python3
"""Phase timeline of the fused pass B (fft4_rowpass_r2c) next to the unfused
pass B, from per-workgroup shader-clock stamps (fft4_set_trace).  K = 32
trials at 2^23."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from peasoup_amd import _C  # noqa: E402
from fft4_trace import report  # noqa: E402

K_ = _C.kernels
FUSED_NAMES = ["start", "loads issued", "stage0", "exch1", "stage1", "exch2", "stage2", "exch3", "stage3",
               "hand-over", "-", "end"]


def main():
    K_.fft4_set_flags(K_.fft4_flags() | 2097152)
    dev = torch.device("cuda")
    n = 1 << 23
    M = n // 2
    K = 32
    s = torch.cuda.current_stream().cuda_stream
    g = K_.fft4_geometry(M)
    x = torch.randn(n, device=dev)
    tab = torch.from_numpy(K_.fft4_tables(g)).to(dev)
    xp = torch.empty(g.insize, device=dev)
    K_.fft4_pad_input(x.data_ptr(), n, xp.data_ptr(), g, s)
    accs = 200.0 + 1.464 * np.arange(K)
    af = torch.tensor([a_ * 64e-6 / (2 * 299792458.0) for a_ in accs], dtype=torch.float64, device=dev)
    Y = torch.empty(K * g.ystride * 2, device=dev)
    X = torch.empty(K * g.xstride * 2, device=dev)
    pst = (M + 4 + 7) // 8 * 8
    Pb = torch.empty(K * pst, device=dev)
    st = torch.tensor([0.0, 1.0, 1.0, 0.0], device=dev)
    K_.fft4_resample_colpass(x.data_ptr(), xp.data_ptr(), n, af.data_ptr(), K, Y.data_ptr(), g, tab.data_ptr(), s)
    runs = (("rowpass", (g.n1 // 8) * K, lambda: K_.fft4_rowpass(Y.data_ptr(), X.data_ptr(), K, g, tab.data_ptr(), s)),
            ("rowpass_r2c", (g.n2 // 16) * K,
             lambda: K_.fft4_rowpass_r2c(Y.data_ptr(), Pb.data_ptr(), pst, K, g, tab.data_ptr(), st.data_ptr(),
                                         float(n), M + 1, s)))
    for name, nblk, fn in runs:
        tr = torch.zeros(nblk * 12, dtype=torch.int64, device=dev)
        fn()
        fn()
        torch.cuda.synchronize()
        tr.zero_()
        K_.fft4_set_trace(tr.data_ptr())
        fn()
        torch.cuda.synchronize()
        K_.fft4_set_trace(0)
        report(name, tr.view(nblk, 12).cpu().numpy(), FUSED_NAMES)


if __name__ == "__main__":
    main()
