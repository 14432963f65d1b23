"""Fused spectrum pass (fft4step.hip fft4_rowpass_spectrum_kernel): pass B of
the four-step FFT forms the normalised interbinned spectrum P (blocked
layout) and its screening bytes Q directly from the pass-A intermediate,
without the complex spectrum reaching memory.

Checked against the unfused path (pass B -> tiled r2c + interbin + normalise,
itself checked against the rocFFT/NumPy oracles in test_kernels_gpu.py): the
mirror bins come from a different (conjugated, pre-twiddled) transform of the
same rows, so values agree to FFT rounding, not bit for bit.  Q must be
dev::q8 of the stored P exactly, and the screened harmonic sum over (P, Q)
must give the records of the fp32 kernel over the same P in natural order."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def _q8_ref(P):
    with np.errstate(invalid="ignore"):
        v = np.rint(P.astype(np.float32) * np.float32(4.0)) + np.float32(128.0)
        q = np.where(np.isnan(v) | (v >= 255), 254, np.where(v <= 0, 255, v - 1))
    return q.astype(np.uint8)


def _series(log2n, seed, pulsar=False):
    rng = np.random.default_rng(seed)
    n = 1 << log2n
    x = rng.standard_normal(n).astype(np.float32)
    if pulsar:
        t = np.arange(n) * 64e-6
        ph = (t / 0.0123) % 1.0
        x += (2.0 * (np.minimum(ph, 1 - ph) < 0.03)).astype(np.float32)
    return torch.from_numpy(x).to(dev)


@pytest.mark.parametrize("log2n", [17, 19, 20, 21, 23])
def test_spectrum_pass_matches_unfused(log2n):
    from peasoup_amd import ops

    x = _series(log2n, 300 + log2n)
    n = x.numel()
    accs = [-300.0, 0.0, 410.0] if log2n == 23 else [-410.0, -300.0, -7.0, 0.0, 3.0, 120.0, 250.0, 499.0, 410.0]
    st = torch.tensor([1.0, 2.0, 0.5, 0.0], dtype=torch.float32, device=dev)
    Pu = ops.fft4_resample_interbin(x, accs, 64e-6, st, float(n)).cpu().numpy()
    Pb, Q, g = ops.fft4_spectrum_pass(x, accs, 64e-6, st, float(n))
    Pn = ops.spec_unblock(Pb, g).cpu().numpy()
    M = g.n1 * g.n2
    assert Pn.shape == Pu.shape == (len(accs), M + 1)
    scale = np.abs(Pu).max()
    assert np.abs(Pn - Pu).max() / scale < 1e-4
    assert np.sqrt(np.mean((Pn - Pu) ** 2)) / np.sqrt(np.mean(Pu ** 2)) < 1e-5
    # every bin written exactly once: the blocked slots are a permutation
    b = torch.arange(M + 1, device=dev, dtype=torch.int64)
    idx = ops.spec_pblk_index(b, g.log2_xrow, g.n1)
    assert torch.unique(idx).numel() == M + 1 and int(idx.max()) == M
    # screening bytes: q8 of the stored P, bin b at column spec_q_shift + b
    import peasoup_amd._C as C

    sh = C.kernels.spec_q_shift
    assert np.array_equal(Q.cpu().numpy()[:, sh:sh + M + 1], _q8_ref(Pn))
    # the row-pair Y hand-over (both pass-A kernels) changes only the layout:
    # the same bits as the tiled Y
    assert g.ypair, "the default pass A hands over row-pair Y at every length"
    Pt, Qt, gt = ops.fft4_spectrum_pass(x, accs, 64e-6, st, float(n), pair_y=False)
    assert not gt.ypair
    assert torch.equal(Pt, Pb) and torch.equal(Qt, Q)
    # only the searched bins (the engine passes its highest harmonic bin): those equal
    # the full pass, nothing at or above the 4-bin group holding the bound
    nb = int(0.14 * M) + 3
    Ps, Qs, _ = ops.fft4_spectrum_pass(x, accs, 64e-6, st, float(n), nbins=nb)
    Pns = ops.spec_unblock(Ps, g).cpu().numpy()
    assert np.array_equal(Pns[:, :nb], Pn[:, :nb])
    assert np.array_equal(Qs.cpu().numpy()[:, sh:sh + nb], Q.cpu().numpy()[:, sh:sh + nb])
    hi_ = (nb + 3) // 4 * 4 + 4
    assert not Pns[:, hi_:M].any() and not Qs.cpu().numpy()[:, sh + hi_:sh + M].any()


def test_spec_pblk_index_native_equals_python():
    import peasoup_amd._C as C
    from peasoup_amd import ops

    for log2_n2, n1 in ((11, 2048), (9, 1024), (8, 256)):
        M = n1 << log2_n2
        rng = np.random.default_rng(log2_n2)
        bs = np.unique(np.concatenate([np.arange(0, 70), np.arange(M - 70, M + 1), rng.integers(0, M + 1, 500)]))
        py = ops.spec_pblk_index(torch.from_numpy(bs.astype(np.int64)), log2_n2, n1).numpy()
        nat = np.array([C.kernels.spec_pblk_index(int(b), log2_n2, n1) for b in bs])
        assert np.array_equal(py, nat)


@pytest.mark.parametrize("log2n,nlev,thresh", [(20, 3, 6.0), (21, 4, 7.0), (21, 1, 5.5)])
def test_screened_sum_on_blocked_spectrum(log2n, nlev, thresh):
    """Records of the screened kernel reading the blocked P / shifted Q equal
    the fp32 kernel's over the same values in natural order."""
    from peasoup_amd import ops

    x = _series(log2n, 17 + log2n, pulsar=True)
    n = x.numel()
    accs = [float(a) for a in np.linspace(-60, 60, 16)]
    st = torch.tensor([0.0, 0.0, 0.5 / np.sqrt(n), 0.0], dtype=torch.float32, device=dev)
    Pb, Q, g = ops.fft4_spectrum_pass(x, accs, 64e-6, st, float(n))
    Pn = ops.spec_unblock(Pb, g).contiguous()
    M = g.n1 * g.n2
    starts = [3, 5, 9, 17, 33, 65]
    ends = [M + 1, M - 7, M + 1, M - 100, M + 1, M + 1]
    a = ops.harmonic_peaks(Pn, nlev, starts, ends, thresh)
    ra = sorted(zip(*[t.tolist() for t in a]))
    import peasoup_amd._C as C

    old = C.kernels.harmonic_flags()
    try:
        for flags in (old, old ^ 65536):  # bit 16 toggled: the other tile size (8 / 16 bins per thread, up to 3 levels)
            C.kernels.harmonic_set_flags(flags)
            b = ops.harmonic_peaks(Pb, nlev, starts, ends, thresh, nbins=M + 1, Q=Q, pblk=g)
            rb = sorted(zip(*[t.tolist() for t in b]))
            assert ra == rb and len(ra) > 20, (flags, len(ra), len(rb))
    finally:
        C.kernels.harmonic_set_flags(old)
