#!/usr/bin/env python3
"""Phase timeline of the fft4 passes from per-workgroup shader-clock stamps
(fft4_set_trace): mean cycles between consecutive events, workgroup lifetime,
and how many workgroups overlap per CU slot.  K = 32 trials at 2^23."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from peasoup_amd import _C  # noqa: E402

K_ = _C.kernels
NAMES = ["start", "loads issued", "stage0", "exch1", "stage1", "exch2", "stage2", "exch3", "stage3", "fft done", "-",
         "end"]
ONEX_NAMES = ["start", "loads issued", "dftP+tw", "exchange", "dftG", "-", "-", "-", "-", "-", "-", "end"]


def report(name, ev, names=NAMES):
    ev = ev.astype(np.int64)
    ok = (ev[:, 0] > 0) & (ev[:, 11] > 0)
    ev = ev[ok]
    t0 = ev[:, 0].min()
    life = ev[:, 11] - ev[:, 0]
    print(f"{name}: {ok.sum()} workgroups, span {(ev[:, 11].max() - t0):.3e} cycles, "
          f"mean lifetime {life.mean():.0f} cycles (median {np.median(life):.0f})")
    prev = 0
    for e in range(1, 12):
        if (ev[:, e] == 0).all() or names[e] == "-":
            continue
        d = ev[:, e] - ev[:, prev]
        print(f"   {names[prev]:>13s} -> {names[e]:<13s} {d.mean():8.0f} cycles ({100 * d.mean() / life.mean():4.1f}%)")
        prev = e


def main():
    flags = int(sys.argv[1]) if len(sys.argv) > 1 else -1  # fft4 flag set (-1: the default)
    log2n = int(sys.argv[2]) if len(sys.argv) > 2 else 23
    if flags >= 0:
        K_.fft4_set_flags(flags)
    dev = torch.device("cuda")
    n = 1 << log2n
    M = n // 2
    K = int(sys.argv[3]) if len(sys.argv) > 3 else (32 if log2n <= 23 else 8)
    s = torch.cuda.current_stream().cuda_stream
    g = K_.fft4_geometry(M)
    g.ypair = K_.fft4_pair_y(g)  # pass A hands the spectrum pass row-pair Y (the engine's fused path)
    x = torch.randn(n, device=dev)
    tab = torch.from_numpy(K_.fft4_tables(g)).to(dev)
    xp = torch.empty(g.insize, device=dev)
    K_.fft4_pad_input(x.data_ptr(), n, xp.data_ptr(), g, s)
    accs = 200.0 + 1.464 * np.arange(K)  # consecutive legacy-plan steps at 2^23 x 64 us (as in a real batch)
    af = torch.tensor([a_ * 64e-6 / (2 * 299792458.0) for a_ in accs], dtype=torch.float64, device=dev)
    Y = torch.empty(K * g.ystride * 2, device=dev)
    X = torch.empty(K * g.xstride * 2, device=dev)
    nblk = (g.n1 // 8) * K
    tr = torch.zeros(nblk * 12, dtype=torch.int64, device=dev)
    col = lambda: K_.fft4_resample_colpass(x.data_ptr(), xp.data_ptr(), n, af.data_ptr(), K, Y.data_ptr(), g,
                                           tab.data_ptr(), s)
    row = lambda: K_.fft4_rowpass(Y.data_ptr(), X.data_ptr(), K, g, tab.data_ptr(), s)
    pst = (M + 1 + 63) // 64 * 64
    qst = (M + 1 + K_.spec_q_shift + 63) // 64 * 64
    Pb = torch.empty(K * pst, device=dev)
    Qb = torch.empty(K * qst, dtype=torch.uint8, device=dev)
    st = torch.tensor([1.0, 2.0, 0.5, 0.0], device=dev)
    spec = lambda: K_.fft4_rowpass_spectrum(Y.data_ptr(), K, g, tab.data_ptr(), Pb.data_ptr(), pst, Qb.data_ptr(), qst,
                                            st.data_ptr(), float(n), s)
    for name, fn in (("colpass", col), ("rowpass_spectrum", spec)):
        fn()
        fn()
        torch.cuda.synchronize()
        tr.zero_()
        K_.fft4_set_trace(tr.data_ptr())
        fn()
        torch.cuda.synchronize()
        K_.fft4_set_trace(0)
        onex = name == "colpass" and (K_.fft4_flags() & 131072) != 0 and g.n2 == 2048
        report(name, tr.view(nblk, 12).cpu().numpy(), ONEX_NAMES if onex else NAMES)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"   {name}: {1e3 * e0.elapsed_time(e1) / 10 / K:.2f} us per trial (K = {K}, untraced)")


if __name__ == "__main__":
    main()
