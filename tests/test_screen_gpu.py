"""Screened harmonic sum (harmsum.hip harmonic_peaks_q8_kernel): integer sums
of the screening bytes dev::q8(P) decide which bins are summed exactly from P.
The records must equal the fp32 kernel's (reference semantics
src/kernels.cu:33-99 + peakfinder.hpp:77-94) for every level, including
saturated, large negative and NaN bins and the pre-threshold disabled."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def _q8_ref(P):
    """device_common.hpp dev::q8: v = rint(4p) + 128; bytes 0..253 = v - 1,
    254 = v >= 255 or NaN, 255 = v <= 0."""
    with np.errstate(invalid="ignore"):
        v = np.rint(P.astype(np.float32) * np.float32(4.0)) + np.float32(128.0)
        q = np.where(np.isnan(v) | (v >= 255), 254, np.where(v <= 0, 255, v - 1))
    return q.astype(np.uint8)


def _records(r):
    return sorted(zip(*[t.tolist() for t in r]))


@pytest.mark.parametrize("nlev,thresh", [(0, 5.0), (1, 6.0), (2, 7.5), (3, 9.0), (3, 11.5), (4, 10.0), (5, 10.0)])
def test_screened_harmonic_peaks_equal_exact(nlev, thresh):
    import peasoup_amd._C as C
    from peasoup_amd import ops

    rng = np.random.default_rng(80 + nlev)
    n, Kb = 200003, 8  # rows not a multiple of 16: the clamped tail chunks
    P = (rng.exponential(1.0, (Kb, n)) - 1.0).astype(np.float32)
    for k in range(Kb):  # harmonic families with amplitudes around the threshold
        for f0 in rng.uniform(40.0, n / 40.0, 3):
            amp = rng.uniform(0.4, 2.5) * thresh
            for hm in range(1, 33):
                b = int(f0 * hm)
                if b < n:
                    P[k, b] += amp / np.sqrt(hm)
    P[0, 1000:1010] = 40.0  # saturated screening bytes
    P[1, 5000] = 1e6
    P[2, 7000:7100] = -50.0  # below the byte range
    P[3, 90001] = np.nan
    starts = [3, 5, 9, 17, 33, 65]
    ends = [n, n - 7, n, n - 100, n, n]
    Pt = torch.from_numpy(P).to(dev)
    Q = ops.quantize_q8(Pt)
    assert np.array_equal(Q.cpu().numpy()[:, :n], _q8_ref(P))
    old = C.kernels.harmonic_flags()
    try:
        # bit 1: pre-threshold off (every bin takes the exact path); bit 16
        # toggled: the other tile size up to 3 levels (8 / 16 bins per thread)
        for flags in (old, old | 2, old ^ 65536, (old ^ 65536) | 2):
            C.kernels.harmonic_set_flags(flags)
            a = _records(ops.harmonic_peaks(Pt, nlev, starts, ends, thresh))
            b = _records(ops.harmonic_peaks(Pt, nlev, starts, ends, thresh, Q=Q))
            assert a == b and len(a) > 20, (len(a), len(b))
    finally:
        C.kernels.harmonic_set_flags(old)


@pytest.mark.parametrize("log2n", [17, 21, 23])
def test_tiled_r2c_writes_screening_bytes(log2n):
    """The tiled r2c kernel's screening bytes are dev::q8 of the P it stores
    (every stored bin; pruned rows included)."""
    from peasoup_amd import ops

    rng = np.random.default_rng(log2n)
    n = 1 << log2n
    x = torch.from_numpy(rng.standard_normal(n).astype(np.float32)).to(dev)
    # P ~ 20 x the amplitude of unit noise: bytes both inside and beyond the byte range
    st = torch.tensor([0.0, 0.0, 0.05 / np.sqrt(n), 0.0], dtype=torch.float32, device=dev)
    accs = [-300.0, 0.0, 250.0]
    for nbo in (None, int(0.4 * n)):
        P, Q = ops.fft4_resample_interbin(x, accs, 64e-6, st, float(n), nbins_out=nbo, screen=True)
        m = n // 2 + 1 if nbo is None else nbo
        exp = _q8_ref(P.cpu().numpy()[:, :m])
        got = Q.cpu().numpy()[:, :m]
        assert np.array_equal(got, exp)
        assert (got == 254).any() and (got < 254).any()
        P0 = ops.fft4_resample_interbin(x, accs, 64e-6, st, float(n), nbins_out=nbo)
        assert torch.equal(P, P0)


def test_engine_screen_equals_exact():
    """SearchEngine on the unfused spectrum path with the screened harmonic
    sum, without it (harmonic flag 4) and with the exact sums recomputed from
    the spectrum instead of a stored P (flag 8) gives identical candidates;
    the fused spectrum pass (flag 64, the default) the same candidates with
    S/N equal to FFT rounding (its mirror bins come from another transform)."""
    import peasoup_amd._C as C

    rng = np.random.default_rng(5)
    n = (1 << 21) + 100
    t = np.arange(n) * 64e-6
    x = rng.normal(128, 6, n)
    ph = (t / 0.0123) % 1.0
    x += 25.0 * (np.minimum(ph, 1 - ph) < 0.02)
    trial = torch.from_numpy(np.clip(np.rint(x), 0, 255).astype(np.uint8)).to(dev)
    accs = [float(a) for a in np.linspace(-40, 40, 17)]
    out = []
    old = C.kernels.harmonic_flags()
    unf = old & ~64
    try:
        # P stored / screen off / bins recomputed / fused (default)
        for flags in (unf & ~8, unf | 4, unf | 8, old | 64):
            C.kernels.harmonic_set_flags(flags)
            p = C.SearchParams()
            p.fft_size, p.tsamp, p.nharmonics = 1 << 21, 64e-6, 4
            eng = C.SearchEngine(p, torch.cuda.current_stream().cuda_stream)
            c = eng.search_trial(trial.data_ptr(), n, 10.0, 3, accs)
            out.append([(x.dm_idx, x.acc, x.nh, x.snr, x.freq, x.count_assoc()) for x in c])
    finally:
        C.kernels.harmonic_set_flags(old)
    assert out[0] == out[1] == out[2] and len(out[0]) > 0
    fused = sorted(out[3], key=lambda r: (r[0], r[1], r[2], r[4]))
    ref = sorted(out[0], key=lambda r: (r[0], r[1], r[2], r[4]))
    assert [(r[0], r[1], r[2], r[4], r[5]) for r in fused] == [(r[0], r[1], r[2], r[4], r[5]) for r in ref]
    assert all(abs(a[3] - b[3]) <= 1e-4 * abs(b[3]) for a, b in zip(fused, ref))
