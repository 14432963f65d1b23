"""The screened harmonic sum's no-miss bound, checked on the host (no GPU):
for every level h, an fp32 sum of the bin's 2^h terms (in the reference
order) above the pre-threshold lo[h] must give an integer sum of screening
bytes above lim[h], unless a term's byte is out of range (>= 254), which
forces the exact path.  Mirrors device_common.hpp dev::q8 and the host bound
of harmonic_peaks_batch (harmsum.hip)."""
import numpy as np

SCALE = [1.0, 0.70710678118654752440, 0.5, 0.35355339059327376220, 0.25, 0.17677669529663688110]


def q8(p):
    v = np.rint(p.astype(np.float32) * np.float32(4.0)) + np.float32(128.0)
    with np.errstate(invalid="ignore"):
        return np.where(np.isnan(v) | (v >= 255), 254, np.where(v <= 0, 255, v - 1)).astype(np.int64)


def pre_lo(thresh, h):
    t = thresh / SCALE[h]
    lo = t - abs(t) * 1e-5 - 1e-30
    f = np.float32(lo)
    if float(f) > lo:
        f = np.nextafter(f, np.float32(-np.inf))
    return f


def lim(thresh, h):
    n = 2.0 ** h
    return int(np.floor(4.0 * (float(pre_lo(thresh, h)) - n / 8.0 - 0.25) + 127.0 * n)) - 1


def seq_sum(terms):
    """fp32 running sum in order (the kernel's accumulation)."""
    acc = terms[:, 0].astype(np.float32)
    for j in range(1, terms.shape[1]):
        acc = (acc + terms[:, j]).astype(np.float32)
    return acc


def test_screen_never_misses_a_bin_above_the_pre_threshold():
    rng = np.random.default_rng(2024)
    for h in range(6):
        n = 1 << h
        for thresh in (5.0, 6.0, 9.0, 12.5):
            lo = pre_lo(thresh, h)
            L = lim(thresh, h)
            # terms around the level's mean share of the threshold, on and between
            # the byte grid (k/4 +- 1/8), plus wide noise and near-range values
            share = float(lo) / n
            parts = [
                share + rng.uniform(-0.5, 0.5, (20000, n)),
                np.round(share * 4 + rng.integers(-3, 4, (20000, n))) / 4 + rng.choice([-0.125, 0.125], (20000, n)),
                rng.uniform(-31.8, 31.6, (20000, n)),
                rng.exponential(1.0, (20000, n)) - 1.0 + share,
            ]
            terms = np.concatenate(parts).astype(np.float32)
            s = seq_sum(terms)
            w = q8(terms)
            passes = (w.sum(axis=1) > L) | (w.max(axis=1) >= 254)
            above = s > lo
            assert above.sum() > 100, (h, thresh)
            missed = above & ~passes
            assert not missed.any(), (h, thresh, terms[missed][:3], s[missed][:3])
            # and the screen is tight: most bins well below the pre-threshold are dropped
            far = s < lo - n * 0.5 - 1.0
            assert passes[far & (w.max(axis=1) < 254)].mean() < 0.01


def test_q8_codes():
    p = np.array([0.0, 0.124, 0.126, -31.7, -31.9, 31.5, 31.7, 1e9, -1e9, np.nan, np.inf, -np.inf],
                 dtype=np.float32)
    w = q8(p)
    assert list(w) == [127, 127, 128, 0, 255, 253, 254, 254, 255, 254, 254, 255]
    inr = w < 254
    assert np.all(np.abs(p[inr] - (w[inr] - 127) / 4.0) <= 0.125)
