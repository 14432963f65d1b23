#!/usr/bin/env python3
"""Per-trial cost of pass A and the fused spectrum pass against the
acceleration: K = 85 trials (one config-3 slice of an 8-rank run) taken from
the ends and the middle of the +-500 m/s^2 legacy plan at 2^23, timed alone
with HIP events.   python tools/expt/accel_cost.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from peasoup_amd import _C  # noqa: E402

K_ = _C.kernels


def main():
    dev = torch.device("cuda")
    log2n = 23
    n = 1 << log2n
    M = n // 2
    tsamp = 64e-6
    plan = _C.AccelPlan(-500.0, 500.0, 1.1, 64.0, n, tsamp, 1550.0 - 200.0, -6.25, _C.AccelConvention.Legacy)
    accs = np.array(plan.generate(0.0))
    K = 85
    s = torch.cuda.current_stream().cuda_stream
    g = K_.fft4_geometry(M)
    g.ypair = K_.fft4_pair_y(g)
    x = torch.randn(n, device=dev)
    tab = torch.from_numpy(K_.fft4_tables(g)).to(dev)
    xp = torch.empty(g.insize, device=dev)
    K_.fft4_pad_input(x.data_ptr(), n, xp.data_ptr(), g, s)
    Y = torch.empty(K * g.ystride * 2, device=dev)
    pst = (M + 1 + 63) // 64 * 64
    qst = (M + 1 + K_.spec_q_shift + 63) // 64 * 64
    Pb = torch.empty(K * pst, device=dev)
    Qb = torch.empty(K * qst, dtype=torch.uint8, device=dev)
    st = torch.tensor([1.0, 2.0, 0.5, 0.0], device=dev)
    print(f"{len(accs)} trials, slices of {K}")
    for name, sl in (("first", slice(0, K)), ("middle", slice(len(accs) // 2 - K // 2, len(accs) // 2 - K // 2 + K)),
                     ("last", slice(len(accs) - K, len(accs)))):
        a = accs[sl]
        af = torch.tensor([a_ * tsamp / (2 * 299792458.0) for a_ in a], dtype=torch.float64, device=dev)
        col = lambda: K_.fft4_resample_colpass(x.data_ptr(), xp.data_ptr(), n, af.data_ptr(), K, Y.data_ptr(), g,  # noqa: E731
                                               tab.data_ptr(), s)
        spec = lambda: K_.fft4_rowpass_spectrum(Y.data_ptr(), K, g, tab.data_ptr(), Pb.data_ptr(), pst,  # noqa: E731
                                                Qb.data_ptr(), qst, st.data_ptr(), float(n), s)
        res = []
        for fn in (col, spec):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res.append(1e3 * e0.elapsed_time(e1) / 5 / K)
        print(f"{name:>6s} acc [{a[0]:8.2f}, {a[-1]:8.2f}]: pass A {res[0]:.2f} us/trial, spectrum {res[1]:.2f} us/trial")


if __name__ == "__main__":
    main()
