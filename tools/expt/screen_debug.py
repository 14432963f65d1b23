#!/usr/bin/env python3
"""Screened vs fp32 harmonic sum on r2c-produced spectra under search-engine
parameters (2^21 series, 17 trials, per-level end bins from max_freq), and the
engine itself with host / device clustering.  Prints any record the screen
misses with its terms, screening bytes and integer bound."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import peasoup_amd._C as C  # noqa: E402
from peasoup_amd import ops  # noqa: E402

dev = "cuda"
K = C.kernels


def lims(thresh, nlev):
    scale = [1.0, 0.70710678118654752440, 0.5, 0.35355339059327376220, 0.25, 0.17677669529663688110]
    out = []
    for h in range(6):
        t = thresh / scale[h]
        lo = np.float32(t - abs(t) * 1e-5 - 1e-30)
        if float(lo) > t - abs(t) * 1e-5 - 1e-30:
            lo = np.nextafter(lo, np.float32(-np.inf))
        n = 2.0 ** h
        x = 4.0 * (float(lo) - n / 8.0 - 0.25) + 127.0 * n
        out.append(int(np.floor(x)) - 1)
    return out


def terms(i, h):
    idx = [i]
    for hh in range(1, h + 1):
        ms = [1] if hh == 1 else ([3, 1] if hh == 2 else list(range(1, 1 << hh, 2)))
        for m in ms:
            idx.append((i * m + (1 << (hh - 1))) >> hh)
    return idx


def main():
    rng = np.random.default_rng(5)
    n = 1 << 21
    t = np.arange(n) * 64e-6
    x = rng.normal(0.0, 1.0, n)
    ph = (t / 0.0123) % 1.0
    x += 4.0 * (np.minimum(ph, 1 - ph) < 0.02)
    xt = torch.from_numpy(x.astype(np.float32)).to(dev)
    accs = [float(a) for a in np.linspace(-40, 40, 17)]
    M = n // 2
    # whitening-like stats: mean / sigma of the interbinned amplitude
    st0 = torch.tensor([0.0, 0.0, 1.0, 0.0], dtype=torch.float32, device=dev)
    P0 = ops.fft4_resample_interbin(xt, accs[:1], 64e-6, st0, 1.0)
    a = P0[0].double()
    st = torch.tensor([float(a.mean()), 0.0, float(a.std()), 0.0], dtype=torch.float32, device=dev)
    bw = 1.0 / (n * 64e-6)
    nlev, thresh = 4, 9.0
    starts, ends = [], []
    for h in range(nlev + 1):
        starts.append(int(2 * M * (0.1 / (bw * (M + 1))) * 2 ** h))
        ends.append(min(M + 1, int(1100.0 / bw * 2 ** h)))
    print("starts", starts, "ends", ends)
    P, Q = ops.fft4_resample_interbin(xt, accs, 64e-6, st, 1.0, nbins_out=max(ends), screen=True)
    Pn = P.cpu().numpy()
    Qn = Q.cpu().numpy()
    a = ops.harmonic_peaks(P, nlev, starts, ends, thresh, nbins=M + 1)
    b = ops.harmonic_peaks(P, nlev, starts, ends, thresh, nbins=M + 1, Q=Q)
    ra = sorted(zip(*[v.tolist() for v in a]))
    rb = sorted(zip(*[v.tolist() for v in b]))
    print("records fp32", len(ra), "screened", len(rb))
    miss = sorted(set(ra) - set(rb))
    extra = sorted(set(rb) - set(ra))
    print("missing", len(miss), "extra", len(extra))
    L = lims(thresh, nlev)
    print("lim", L)
    for (k, h, i, snr) in miss[:10]:
        ix = terms(i, h)
        w = [int(Qn[k, j]) for j in ix]
        p = [float(Pn[k, j]) for j in ix]
        print(f"  trial {k} level {h} bin {i} snr {snr:.4f}: sum w {sum(w)} vs lim {L[h]}; max w {max(w)}")
        print("    p", [round(v, 3) for v in p])
        print("    w", w)
    for cl in ("0", "1"):
        os.environ["PSOUP_GPU_CLUSTER"] = cl
        out = []
        old = K.harmonic_flags()
        try:
            for flags in (old, old | 4):
                K.harmonic_set_flags(flags)
                p = C.SearchParams()
                p.fft_size, p.tsamp, p.nharmonics = 1 << 21, 64e-6, 4
                eng = C.SearchEngine(p, torch.cuda.current_stream().cuda_stream)
                u8 = torch.from_numpy(np.clip(np.rint(128 + 6 * x), 0, 255).astype(np.uint8)).to(dev)
                c = eng.search_trial(u8.data_ptr(), n, 10.0, 3, accs)
                ctr = eng.counters()
                out.append(([(v.acc, v.nh, v.snr, v.freq) for v in c], ctr.get("peaks", -1)))
        finally:
            K.harmonic_set_flags(old)
        print(f"engine cluster={cl}: screened {len(out[0][0])} cands / {out[0][1]} peaks, "
              f"fp32 {len(out[1][0])} cands / {out[1][1]} peaks, equal {out[0][0] == out[1][0]}")


if __name__ == "__main__":
    main()
