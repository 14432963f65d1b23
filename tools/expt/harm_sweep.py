#!/usr/bin/env python3
"""Harmonic-sum kernel tuning sweep at the headline size (2^23-point series,
K trials of 2^22 + 1 interbinned bins, 8-harmonic sum): block order,
nontemporal fundamental loads and an occupancy cap (extra dynamic LDS per
workgroup, so fewer tiles -- a smaller gather footprint -- are in flight per
XCD).  HIP-event timing, one stream.

    python tools/expt/harm_sweep.py [--K 32] [--reps 10]
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
    nb = M + 1
    pstride = (nb + 63) // 64 * 64
    K = a.K
    s = torch.cuda.current_stream().cuda_stream
    P = torch.randn(K * pstride, device=dev)
    cap = 1 << 20
    out = torch.empty(cap * 3, dtype=torch.int32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    starts = [1, 2, 4, 8, 16]
    ends = [nb] * 5

    def harm():
        cnt.zero_()
        K_.harmonic_peaks_batch(P.data_ptr(), nb, pstride, K, 3, starts, ends, 4.5, cap, out.data_ptr(),
                                cnt.data_ptr(), s)

    ref = None
    # static LDS is ~28.8 KiB: +50 KiB -> 2 workgroups/CU, +25 -> 3, +12 -> 4
    for name, fl in [("xcd", 1), ("xcd two-phase", 1 | 32), ("xcd", 1), ("xcd two-phase", 1 | 32),
                     ("plain two-phase", 32), ("xcd two-phase 6wg/CU", 1 | 32 | (10 << 8))]:
        K_.harmonic_set_flags(fl)
        us = timeit(harm, a.reps)
        torch.cuda.synchronize()
        c = int(cnt.item())
        got = sorted(map(tuple, out[: 3 * min(c, cap)].view(-1, 3).cpu().tolist()))
        if ref is None:
            ref = got
        same = "same peaks" if got == ref else "PEAKS DIFFER"
        print(f"harmonic_peaks {name:16s} flags={fl:6d} {us:9.1f} us/launch {us / K:7.2f} us/trial  "
              f"{K * 4 * nb / us / 1e3:7.0f} GB/s  peaks={c} {same}", flush=True)
    K_.harmonic_set_flags(1)


if __name__ == "__main__":
    main()
