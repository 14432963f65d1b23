"""NumPy reference implementations (float32 semantics) of every device stage.

Each function mirrors the reference CUDA code it replaces (cited per
function) and is the oracle for the HIP-kernel numerics tests.  The whole
chain also forms a CPU reference search (``search_trial``) used to validate
the algorithm on tutorial.fil without a GPU.
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence, Tuple

import numpy as np

C_LIGHT = 299792458.0
LEVEL_SCALE = [1.0, 1.0 / math.sqrt(2.0), 0.5, 1.0 / math.sqrt(8.0), 0.25, 1.0 / math.sqrt(32.0)]


# ------------------------------------------------------------ dedispersion --
def delay_table(nchans: int, tsamp: float, fch1: float, foff: float) -> np.ndarray:
    f0, df, dt = np.float32(fch1), np.float32(foff), np.float32(tsamp)
    c = np.arange(nchans, dtype=np.float32)
    a = np.float32(1.0) / (f0 + c * df)
    b = np.float32(1.0) / f0
    return (4.15e3 / float(dt) * (a * a - b * b).astype(np.float64)).astype(np.float32)


def dm_offsets(dms: Sequence[float], delays: np.ndarray) -> np.ndarray:
    d = np.asarray(dms, dtype=np.float32)[:, None] * delays[None, :]
    return (d + np.float32(0.5)).astype(np.int32)


def dedisperse(values: np.ndarray, offsets: np.ndarray, nbits: int, killmask=None,
               out_nsamps: int = None) -> np.ndarray:
    """values [nsamps, nchans] (raw) -> uint8 [ndm, out_nsamps] (dedisp 8-bit scaling)."""
    nsamps, nchans = values.shape
    kill = np.ones(nchans, bool) if killmask is None else np.asarray(killmask) != 0
    if out_nsamps is None:
        out_nsamps = nsamps - int(offsets.max())
    scale = np.float32(192.0 / (((1 << nbits) - 1) * nchans))
    x = values.T.astype(np.int64)
    out = np.empty((offsets.shape[0], out_nsamps), dtype=np.uint8)
    for d in range(offsets.shape[0]):
        s = np.zeros(out_nsamps, dtype=np.int64)
        for c in np.nonzero(kill)[0]:
            o = int(offsets[d, c])
            s += x[c, o:o + out_nsamps]
        v = np.clip(s.astype(np.float32) * scale, 0, 255)
        out[d] = v.astype(np.uint8)
    return out


# --------------------------------------------------------------- spectra ----
def convert_pad(trial_u8: np.ndarray, n: int) -> np.ndarray:
    nvalid = min(len(trial_u8), n)
    out = np.empty(n, dtype=np.float32)
    out[:nvalid] = trial_u8[:nvalid]
    if n > nvalid:
        out[nvalid:] = np.float32(float(trial_u8[:nvalid].astype(np.int64).sum()) / nvalid)
    return out


def amplitude(X: np.ndarray) -> np.ndarray:
    return np.abs(X.astype(np.complex64)).astype(np.float32)


def interbin(X: np.ndarray) -> np.ndarray:
    X = X.astype(np.complex64)
    prev = np.concatenate([[0j], X[:-1]]).astype(np.complex64)
    a = (X.real * X.real + X.imag * X.imag).astype(np.float32)
    d = (X - prev)
    b = (0.5 * (d.real * d.real + d.imag * d.imag).astype(np.float64)).astype(np.float32)
    return np.sqrt(np.maximum(a, b)).astype(np.float32)


def median_scrunch5(x: np.ndarray) -> np.ndarray:
    n = len(x)
    if n < 5:
        if n == 1:
            return x[:1].copy()
        if n == 2:
            return np.array([np.float32(0.5) * (x[0] + x[1])], np.float32)
        if n == 3:
            return np.array([np.median(x)], np.float32)
        s = np.sort(x)
        return np.array([np.float32(0.5) * (s[1] + s[2])], np.float32)
    m = n // 5
    return np.median(x[: 5 * m].reshape(m, 5), axis=1).astype(np.float32)


def linear_stretch(x: np.ndarray, out_count: int) -> np.ndarray:
    in_count = len(x)
    step = np.float32(in_count - 1) / np.float32(out_count - 1)
    xi = np.arange(out_count, dtype=np.uint32).astype(np.float32) * step
    j = np.minimum(xi.astype(np.uint32), in_count - 1)
    frac = (xi - j.astype(np.float32)).astype(np.float32)
    a = x[j]
    nxt = x[np.minimum(j + 1, in_count - 1)]
    use = (frac > np.float32(1e-5)) & (j + 1 < in_count)
    return np.where(use, a + frac * (nxt - a), a).astype(np.float32)


def running_median(amp: np.ndarray, bin_width: float, b5: float = 0.05, b25: float = 0.5) -> np.ndarray:
    """Dereddener::calculate_median (dereddener.hpp:44-62)."""
    nb = len(amp)
    m5 = median_scrunch5(amp)
    m25 = median_scrunch5(m5)
    m125 = median_scrunch5(m25)
    pos5 = int(np.float32(b5) / np.float32(bin_width))
    pos25 = int(np.float32(b25) / np.float32(bin_width))
    s5, s25, s125 = linear_stretch(m5, nb), linear_stretch(m25, nb), linear_stretch(m125, nb)
    k = np.arange(nb)
    return np.where(k >= pos25, s125, np.where(k >= pos5, s25, s5)).astype(np.float32)


def deredden(X: np.ndarray, median: np.ndarray, zapmask: np.ndarray = None) -> np.ndarray:
    out = (X / median.astype(np.complex64)).astype(np.complex64)
    out[:5] = 0
    if zapmask is not None:
        out[zapmask] = 1 + 0j
    return out


def zap_mask(freqs, widths, bin_width: float, nbins: int) -> np.ndarray:
    m = np.zeros(nbins, bool)
    for f, w in zip(freqs, widths):
        lo = int(math.floor((np.float32(f) - np.float32(w)) / np.float32(bin_width)))
        hi = int(math.ceil((np.float32(f) + np.float32(w)) / np.float32(bin_width)))
        lo = max(lo, 0)
        if lo >= nbins:
            continue
        hi = min(hi, nbins - 1)
        m[lo:hi] = True
    return m


def stats(P: np.ndarray) -> Tuple[float, float, float]:
    s = float(P.astype(np.float64).sum())
    s2 = float((P.astype(np.float64) ** 2).sum())
    n = np.float32(len(P))
    mean = np.float32(s) / n
    rms = np.sqrt(np.float32(s2) / n)
    std = np.sqrt(max(rms * rms - mean * mean, np.float32(0)))
    return float(mean), float(rms), float(std)


def whiten(trial_u8: np.ndarray, n: int, tsamp: float, zapmask=None, with_stats=True):
    """Worker::start per-DM whitening (pipeline_multi.cu:156-204)."""
    x = convert_pad(trial_u8, n)
    X = np.fft.rfft(x.astype(np.float64)).astype(np.complex64)
    bw = np.float32(1.0 / np.float32(np.float32(n) * np.float32(tsamp)))
    med = running_median(amplitude(X), float(bw))
    X = deredden(X, med, zapmask)
    st = stats(interbin(X)) if with_stats else None
    series = (np.fft.irfft(X.astype(np.complex128), n) * n).astype(np.float32)
    return series, st


# ---------------------------------------------------------- acceleration ---
def accel_factor(acc: float, tsamp: float) -> float:
    return (float(np.float32(acc)) * float(np.float32(tsamp))) / (2 * C_LIGHT)


def resample_ii(x: np.ndarray, af: float) -> np.ndarray:
    n = len(x)
    i = np.arange(n, dtype=np.float64)
    j = np.rint(i + i * af * (i - n))
    j = np.clip(j, 0, n - 1).astype(np.int64)
    return x[j]


def resample_v1(x: np.ndarray, af: float) -> np.ndarray:
    n = len(x)
    h = n / 2.0
    i = np.arange(n, dtype=np.float64)
    j = np.clip(np.rint(i + af * ((i - h) ** 2 - h * h)), 0, n - 1).astype(np.int64)
    return x[j]


def harmonic_sums(P: np.ndarray, nlevels: int) -> List[np.ndarray]:
    """harmonic_sum_kernel (kernels.cu:33-99) -> [level1..levelH] arrays."""
    n = len(P)
    i = np.arange(n, dtype=np.int64)
    val = P.astype(np.float32).copy()
    out = []
    orders = {1: [1], 2: [3, 1], 3: [1, 3, 5, 7], 4: list(range(1, 16, 2)), 5: list(range(1, 32, 2))}
    for h in range(1, nlevels + 1):
        for m in orders[h]:
            val = (val + P[(i * m + (1 << (h - 1))) >> h]).astype(np.float32)
        out.append((val.astype(np.float64) * LEVEL_SCALE[h]).astype(np.float32))
    return out


def peak_bounds(nbins: int, bin_width: float, nh: int, min_freq: float, max_freq: float):
    nyquist = np.float32(bin_width) * np.float32(nbins)
    orig = int(2.0 * (nbins - 1.0))
    p2 = 2.0 ** nh
    max_bin = int(float(np.float32(max_freq) / np.float32(bin_width)) * p2)
    start = int(float(np.float32(orig) * (np.float32(min_freq) / nyquist)) * p2)
    factor = 1.0 / nbins * float(nyquist) / 2.0 ** nh
    return max(start, 0), min(nbins, max_bin), factor


def unique_peaks(idxs: np.ndarray, snrs: np.ndarray, min_gap: int = 30):
    out = []
    ii, n = 0, len(idxs)
    while ii < n:
        cpeak, cidx, last = snrs[ii], idxs[ii], idxs[ii]
        ii += 1
        while ii < n and idxs[ii] - last < min_gap:
            if snrs[ii] > cpeak:
                cpeak, cidx, last = snrs[ii], idxs[ii], idxs[ii]
            ii += 1
        out.append((int(cidx), float(cpeak)))
    return out


def spectrum_peaks(series: np.ndarray, af: float, mean: float, std: float, n: int, bin_width: float,
                   nharm: int, thresh: float, min_freq: float, max_freq: float):
    """One acceleration trial: resample, R2C, interbin, normalise, harmonic sums,
    peaks -> list of (nh, idx, snr, freq)."""
    r = resample_ii(series, af)
    X = np.fft.rfft(r.astype(np.float64)).astype(np.complex64)
    P = interbin(X)
    P = ((P - np.float32(np.float32(mean) * np.float32(n))) / np.float32(np.float32(std) * np.float32(n))).astype(np.float32)
    levels = [P] + harmonic_sums(P, nharm)
    res = []
    for h, L in enumerate(levels):
        s, e, fac = peak_bounds(len(P), bin_width, h, min_freq, max_freq)
        seg = L[s:e]
        idx = np.nonzero(seg > np.float32(thresh))[0] + s
        for pi, ps in unique_peaks(idx, L[idx]):
            res.append((h, pi, ps, float(np.float32(pi * fac))))
    return res


# ---------------------------------------------------------------- folding --
def fold_series(x: np.ndarray, period: float, tsamp: float, nbins: int = 64, nints: int = 16) -> np.ndarray:
    """fold_time_series_kernel (kernels.cu:597-633): counts start at 1."""
    n = len(x)
    nps = n // nints
    out = np.zeros((nints, nbins), np.float64)
    cnt = np.ones((nints, nbins), np.int64)
    j = np.arange(nps * nints, dtype=np.float64)
    ph = np.modf(j * (tsamp / period))[0]
    b = np.floor(ph * nbins).astype(np.int64)
    s = (np.arange(nps * nints) // nps)
    np.add.at(out, (s, b), x[: nps * nints].astype(np.float64))
    np.add.at(cnt, (s, b), 1)
    return (out / cnt).astype(np.float32)


def shift_table(nbins: int = 64, nints: int = 16) -> np.ndarray:
    two_pi = np.float32(2 * 3.14159265359)
    s = np.arange(nbins)[:, None, None]
    i = np.arange(nints)[None, :, None].astype(np.float32)
    b = np.arange(nbins)[None, None, :]
    shift = (i / np.float32(nints)) * (s - nbins // 2).astype(np.float32)
    ramp = (b.astype(np.float32) * two_pi / np.float32(nbins)).astype(np.float32)
    ramp = np.where(b > nbins // 2, ramp - two_pi, ramp).astype(np.float32)
    ph = (-1.0 * ramp * shift).astype(np.float32)
    return np.exp(1j * ph.astype(np.float64)).astype(np.complex64)


def fold_optimise(fold: np.ndarray, nbins: int = 64, nints: int = 16):
    """FoldOptimiser::optimise (folder.hpp:235-334) with numpy FFTs:
    returns (opt_template, opt_shift, opt_bin_raw, opt_fold, opt_prof)."""
    F = np.fft.fft(fold.astype(np.complex64), axis=1)
    sh = shift_table(nbins, nints)
    post = F[None, :, :] * sh                      # [shift][int][bin]
    prof = post.sum(axis=1)                        # [shift][bin]
    ntmpl = nbins - 1
    box = (np.arange(nbins)[None, :] <= np.arange(ntmpl)[:, None]).astype(np.complex64)
    T = np.fft.fft(box, axis=1)                    # [template][bin]
    arr = prof[None, :, :] * T[:, None, :] / np.sqrt(np.arange(1, ntmpl + 1, dtype=np.float32))[:, None, None]
    arr[:, :, 0] = 0
    inv = np.fft.ifft(arr, axis=2) * nbins         # unnormalised inverse
    mag = np.abs(inv).astype(np.float32)
    am = int(np.argmax(mag))
    t = am // (nbins * nbins)
    s = (am // nbins) % nbins
    j = am % nbins
    opt_fold = (np.fft.ifft(post[s], axis=1) * nbins).real.astype(np.float32)
    opt_prof = (np.fft.ifft(prof[s]) * nbins).real.astype(np.float32)
    return t, s, j, opt_fold, opt_prof


def calculate_sn(prof: np.ndarray, bin: int, width: int) -> Tuple[float, float]:
    nbins = len(prof)
    edge = int(width * 0.3 + 0.5)
    wb2 = int(width / 2.0 + 0.5)
    rprof = np.array([prof[(bin - nbins // 2 + ii) % nbins] for ii in range(nbins)], np.float32)
    b = nbins // 2 - 1
    up, lo = b + (wb2 + edge), b - (wb2 + edge)
    on = np.array([rprof[i] for i in range(nbins) if lo <= i <= up], np.float32)
    off = np.array([rprof[i] for i in range(nbins) if not (lo <= i <= up)], np.float32)
    on_mean = np.float32(on.astype(np.float64).sum() / len(on))
    off_mean = np.float32(off.astype(np.float64).sum() / len(off))
    acc = np.float32(0)
    for v in off:
        acc = np.float32(float(acc) + (float(v) - float(off_mean)) ** 2)
    off_std = np.sqrt(acc / np.float32(len(off)))
    with np.errstate(divide="ignore", invalid="ignore"):
        sn1 = np.float32((on_mean - off_mean) * math.sqrt(width) / off_std)
        r = ((rprof - off_mean) / off_std).astype(np.float32)
        sn2 = np.float32(r.astype(np.float64).sum() / math.sqrt(width)) if width > 0 else np.float32(np.inf)
    if sn1 > 99999:
        sn1 = np.float32(0)
    if sn2 > 99999:
        sn2 = np.float32(0)
    return float(sn1), float(sn2)


def coincidence_mask(arrays: Sequence[np.ndarray], thresh: float, beam_thresh: int) -> np.ndarray:
    cnt = np.zeros(len(arrays[0]), np.int64)
    for a in arrays:
        cnt += (a > np.float32(thresh))
    return (cnt < beam_thresh).astype(np.float32)


# ----------------------------------------------------------------- FFA ------
def ffa_transform(X: np.ndarray) -> np.ndarray:
    """Radix-2 FFA (Staelin) of an [m, P] fold matrix, m a power of two:
    out[s] = H[s//2] + roll(T[s//2], -((s+1)//2)) over the two transformed
    halves; row s is the fold at period P + s/(m-1) bins (ffa.hip convention).
    Evaluated in float64 (the oracle)."""
    X = np.asarray(X, dtype=np.float64)
    m = X.shape[0]
    if m == 1:
        return X.copy()
    h = m // 2
    H, T = ffa_transform(X[:h]), ffa_transform(X[h:])
    out = np.empty_like(X)
    for s in range(m):
        j = s // 2
        out[s] = H[j] + np.roll(T[j], -((s + 1) // 2))
    return out


def ffa_fold_matrix(ds: np.ndarray, P: int) -> np.ndarray:
    """[m2, P]: floor(len/P) rows of the series, zero rows up to a power of two."""
    m = len(ds) // P
    m2 = 1 << int(np.ceil(np.log2(max(1, m))))
    X = np.zeros((m2, P), dtype=np.float64)
    X[:m] = np.asarray(ds[: m * P], dtype=np.float64).reshape(m, P)
    return X


def boxcar_best_snr(profile: np.ndarray, widths, var: float) -> float:
    """Max over widths and circular phases of boxcar_sum / sqrt(w var)."""
    p = np.asarray(profile, dtype=np.float64)
    P = len(p)
    ext = np.concatenate([p, p])
    c = np.concatenate([[0.0], np.cumsum(ext)])
    best = -np.inf
    for w in widths:
        if w >= P:
            break
        s = (c[w: w + P] - c[:P]).max()
        best = max(best, s / np.sqrt(w * var))
    return best


def ffa_downsample(x: np.ndarray, f: float) -> np.ndarray:
    """Piecewise-constant integration over [j f, (j+1) f)."""
    x = np.asarray(x, dtype=np.float64)
    n = len(x)
    nout = int(np.floor(n / f))
    c = np.concatenate([[0.0], np.cumsum(x)])

    def integ(t):
        i = np.minimum(np.floor(t).astype(np.int64), n)
        frac = t - i
        return c[i] + np.where(i < n, x[np.minimum(i, n - 1)] * frac, 0.0)

    j = np.arange(nout + 1, dtype=np.float64) * f
    I = integ(j)
    return I[1:] - I[:-1]
