#!/usr/bin/env python3
"""rocFFT row pass of a four-step FFT too long for the fused passes: C2C of
length n1 over the n2 rows of Y (row pitch n1 + 8), written either in natural
bin order (output stride n2: X[k1 n2 + k2]) or row-contiguous; time per
transform set, HIP events.   python tools/expt/rows_probe.py [log2n]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from peasoup_amd import _C  # noqa: E402


def main():
    log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 26
    M = 1 << (log2n - 1)
    n2 = 4096
    n1 = M // n2
    yp = n1 + 8
    dev = torch.device("cuda")
    s = torch.cuda.current_stream().cuda_stream
    Y = torch.randn(n2 * yp * 2, device=dev)
    X = torch.empty(M * 2 + 16, device=dev)
    for name, kw in (("natural (out stride n2)", dict(in_dist=yp, out_dist=1, out_stride=n2)),
                     ("row-contiguous", dict(in_dist=yp, out_dist=n1, out_stride=1))):
        plan = _C.FftPlan(_C.FftType.C2C_FWD, n1, n2, inplace=False, **kw)
        plan.execute(Y.data_ptr(), X.data_ptr(), s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            plan.execute(Y.data_ptr(), X.data_ptr(), s)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        gb = (n2 * n1 * 8 * 2) / 1e9
        print(f"2^{log2n}: n1 {n1} x {n2} rows, {name}: {1e3 * ms:.1f} us ({gb / ms * 1e3 / 1e3:.2f} TB/s of in+out), "
              f"work {plan.work_bytes} B", flush=True)
    # check one row against torch
    yr = torch.view_as_complex(Y[: 2 * n1].view(n1, 2).contiguous())
    ref = torch.fft.fft(yr)
    plan = _C.FftPlan(_C.FftType.C2C_FWD, n1, n2, inplace=False, in_dist=yp, out_dist=1, out_stride=n2)
    plan.execute(Y.data_ptr(), X.data_ptr(), s)
    torch.cuda.synchronize()
    Xc = torch.view_as_complex(X[: 2 * M].view(M, 2))
    got = Xc[0::n2][:n1]
    print("row 0 max rel err", float((got - ref).abs().max() / ref.abs().max()))


if __name__ == "__main__":
    main()
