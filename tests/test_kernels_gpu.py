"""HIP kernel numerics vs the NumPy float32 references (MI355X)."""
import math

import numpy as np
import pytest
import torch

from peasoup_amd.utils import reference as ref
from peasoup_amd.utils import sigproc, synthetic

pytestmark = pytest.mark.gpu
dev = "cuda"


def test_single_hip_runtime_loaded():
    import peasoup_amd  # noqa: F401

    libs = {l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l}
    assert len(libs) == 1, libs


@pytest.mark.parametrize("nbits", [1, 2, 4, 8])
def test_unpack_transpose(nbits):
    from peasoup_amd import ops

    rng = np.random.default_rng(nbits)
    nsamps, nchans = 1000, 96 if nbits != 1 else 64
    vals = rng.integers(0, 1 << nbits, size=(nsamps, nchans), dtype=np.uint8)
    packed = torch.from_numpy(sigproc.pack_samples(vals, nbits)).to(dev)
    bias = 128 if nbits == 8 else 0
    out = ops.unpack_transpose(packed, nsamps, nchans, nbits, bias=bias, stride=1024)
    exp = (vals.T.astype(np.int16) - bias).astype(np.int8)
    assert np.array_equal(out[:, :nsamps].cpu().numpy(), exp)


def _geometry(C, nchans=64, nbits=2, nsamps=6000, dm_end=200.0, tsamp=0.00032, fch1=1510.0, foff=-1.09):
    hdr = synthetic.make_header(nchans=nchans, nbits=nbits, tsamp=tsamp, fch1=fch1, foff=foff, nsamples=nsamps)
    dms = C.generate_dm_list(0.0, dm_end, tsamp, 64.0, fch1, foff, nchans, 1.1)
    return hdr, dms


@pytest.mark.parametrize("nbits,nchans,kill", [(2, 64, False), (8, 128, True), (4, 64, True), (1, 64, False),
                                               (8, 384, True)])
def test_dedisperse_direct_mfma_valu_bit_exact(C, nbits, nchans, kill):
    """Direct, one-hot MFMA and packed-byte VALU kernels vs the NumPy
    reference; (8, 384) exercises the VALU kernel's 32-bit flush path."""
    rng = np.random.default_rng(7)
    hdr, dms = _geometry(C, nchans=nchans, nbits=nbits, nsamps=5000, dm_end=150.0)
    vals = rng.integers(0, 1 << nbits, size=(5000, nchans), dtype=np.uint8)
    killmask = [int(rng.random() > 0.2) for _ in range(nchans)] if kill else []
    g = C.DedispGeometry.make(hdr, 5000, dms, killmask)
    s = torch.cuda.current_stream().cuda_stream
    dfb = C.DeviceFilterbank(g, s)
    packed = torch.from_numpy(sigproc.pack_samples(vals, nbits)).to(dev)
    dfb.load_packed_device(packed.data_ptr())
    dd = C.Dedisperser(dfb, s)
    ndm = len(dms)
    stride = C.Dedisperser.row_stride(g.out_nsamps)
    outs = {}
    kinds = (C.DedispKernel.Direct, C.DedispKernel.Mfma, C.DedispKernel.Valu, C.DedispKernel.Auto)
    if nbits <= 2:  # the packed 2-bit kernel
        kinds = kinds + (C.DedispKernel.Packed2,)
    for k in kinds:
        o = torch.zeros(ndm * stride, dtype=torch.uint8, device=dev)
        dd.run(0, ndm, o.data_ptr(), stride, k)
        outs[k] = o.view(ndm, stride)[:, : g.out_nsamps].cpu().numpy()
    offs = np.array(g.offsets(0, ndm), dtype=np.int32).reshape(ndm, nchans)
    exp = ref.dedisperse(vals, offs, nbits, killmask or None, g.out_nsamps)
    for k in kinds:
        assert np.array_equal(outs[k], exp), k
    # sub-range (DM offset inside a tile)
    for k in kinds[1:]:
        o = torch.zeros(5 * stride, dtype=torch.uint8, device=dev)
        dd.run(3, 8, o.data_ptr(), stride, k)
        assert np.array_equal(o.view(5, stride)[:, : g.out_nsamps].cpu().numpy(), exp[3:8]), k


@pytest.mark.parametrize("nbits", [2, 4])
def test_dedisperse_1024ch_hybrid_mfma_bit_exact(C, nbits):
    """Config-4 geometry (1024 channels, 64 us, 1550 MHz - 400 MHz), 2^18
    output samples, 7 DM tiles from DM 0 to high DM: the LDS-fed one-hot MFMA
    kernel (low-spread tiles), the VALU kernels (byte and, for 2-bit data,
    packed 2-bit) and Auto (4-bit data: the MFMA / VALU hybrid split; 2-bit:
    the packed kernel throughout) all equal the direct kernel byte for byte."""
    rng = np.random.default_rng(21)
    nchans, tsamp, fch1, foff = 1024, 64e-6, 1550.0, -400.0 / 1024
    dms = C.generate_dm_list(0.0, 300.0, tsamp, 64.0, fch1, foff, nchans, 1.25)
    ndm = 320  # the first 10 tiles: ~2.1 -> 2.9 MFMA steps per channel (window-fitting to tile 10)
    delays = C.generate_delay_table(nchans, tsamp, fch1, foff)
    nsamps = (1 << 18) + C.compute_max_delay(dms, delays)
    hdr = synthetic.make_header(nchans=nchans, nbits=nbits, tsamp=tsamp, fch1=fch1, foff=foff, nsamples=nsamps)
    killmask = [int(rng.random() > 0.05) for _ in range(nchans)]
    g = C.DedispGeometry.make(hdr, nsamps, dms, killmask)
    s = torch.cuda.current_stream().cuda_stream
    dfb = C.DeviceFilterbank(g, s)
    packed = torch.randint(0, 256, (nsamps * nchans * nbits // 8,), dtype=torch.uint8, device=dev)
    dfb.load_packed_device(packed.data_ptr())
    dd = C.Dedisperser(dfb, s)
    split = dd.mfma_lds_split(0, ndm)
    if nbits == 4:
        assert 0 < split < ndm and split % 32 == 0, split  # both kernels run in Auto
    else:
        assert split == 0, split  # the packed 2-bit kernel beats the MFMA one at every spread
        split = 96  # (the LDS-fed MFMA kernel's leading tiles, run explicitly below)
    assert dd.mfma_lds_split(0, 8) == 0  # an 8-DM partial tile: the VALU kernel (MFMA computes all 32 DMs)
    stride = C.Dedisperser.row_stride(g.out_nsamps)
    outs = {}
    P2 = C.DedispKernel.Packed2 if nbits == 2 else C.DedispKernel.Valu
    for k in (C.DedispKernel.Direct, C.DedispKernel.Mfma, C.DedispKernel.Valu, C.DedispKernel.Auto, P2):
        o = torch.zeros(ndm * stride, dtype=torch.uint8, device=dev)
        dd.run(0, ndm, o.data_ptr(), stride, k)
        outs[k] = o.view(ndm, stride)[:, : g.out_nsamps]
    ref_ = outs[C.DedispKernel.Direct]
    for k in (C.DedispKernel.Mfma, C.DedispKernel.Valu, C.DedispKernel.Auto, P2):
        assert torch.equal(outs[k], ref_), k
    # MFMA-LDS on the low-DM tiles alone, and a range starting inside the split
    o = torch.zeros(split * stride, dtype=torch.uint8, device=dev)
    dd.run(0, split, o.data_ptr(), stride, C.DedispKernel.Mfma)
    assert torch.equal(o.view(split, stride)[:, : g.out_nsamps], ref_[:split])
    o = torch.zeros((ndm - 32) * stride, dtype=torch.uint8, device=dev)
    dd.run(32, ndm, o.data_ptr(), stride, C.DedispKernel.Auto)
    assert torch.equal(o.view(ndm - 32, stride)[:, : g.out_nsamps], ref_[32:])
    # ranges that do not start on a 32-DM tile (DM-sharded ranks: the bench's
    # [8r, 8r + 8), static shards cut anywhere): every kernel, no per-call plan
    for d0, d1 in ((8, 16), (24, 32), (40, 48), (1, 9), (5, 70), (13, 40), (33, 97), (100, 101),
                   (split - 3, split + 37), (250, ndm)):
        for k in (C.DedispKernel.Mfma, C.DedispKernel.Valu, C.DedispKernel.Auto, P2):
            o = torch.zeros((d1 - d0 + 2) * stride, dtype=torch.uint8, device=dev)  # a guard row each side
            dd.run(d0, d1, o.data_ptr() + stride, stride, k)
            got = o.view(d1 - d0 + 2, stride)
            assert torch.equal(got[1: d1 - d0 + 1, : g.out_nsamps], ref_[d0:d1]), (d0, d1, k)
            assert not got[0].any() and not got[d1 - d0 + 1].any(), (d0, d1, k)  # nothing stored outside
    # the fold stage's scattered DM list (unsorted, a repeat, > one 32-DM tile)
    lst = [int(v) for v in rng.choice(ndm, 40, replace=False)] + [7, 7]
    o = torch.zeros(len(lst) * stride, dtype=torch.uint8, device=dev)
    dd.run_list(lst, o.data_ptr(), stride)
    assert torch.equal(o.view(len(lst), stride)[:, : g.out_nsamps], ref_[lst])
    # a static shard's own tables (warm(d0, d1)): its ranges are exact, and a
    # range outside them rebuilds the whole list's and is exact too
    for d0, d1, out_of in ((70, 150, (0, 40)), (200, ndm, (5, 70)), (13, 40, (250, ndm))):
        sh = C.Dedisperser(dfb, s)
        sh.warm(d0, d1)
        for a, b in ((d0, d1), (d0 + 3, d1 - 1), out_of):
            for k in (C.DedispKernel.Mfma, C.DedispKernel.Valu, C.DedispKernel.Auto, P2):
                o = torch.zeros((b - a) * stride, dtype=torch.uint8, device=dev)
                sh.run(a, b, o.data_ptr(), stride, k)
                assert torch.equal(o.view(b - a, stride)[:, : g.out_nsamps], ref_[a:b]), (d0, d1, a, b, k)


def test_dedisperse_packed2_high_dm_bit_exact(C):
    """The 2-bit kernel at config-4 DMs up to ~2000 (wide per-tile spreads,
    windows near its LDS bound), with killed channels: equal to the direct
    kernel byte for byte, for whole tiles, unaligned ranges and Auto."""
    rng = np.random.default_rng(41)
    nchans, tsamp, fch1, foff = 1024, 64e-6, 1550.0, -400.0 / 1024
    dms = C.generate_dm_list(0.0, 2200.0, tsamp, 64.0, fch1, foff, nchans, 1.1)
    delays = C.generate_delay_table(nchans, tsamp, fch1, foff)
    nsamps = (1 << 18) + 5000 + C.compute_max_delay(dms, delays)
    hdr = synthetic.make_header(nchans=nchans, nbits=2, tsamp=tsamp, fch1=fch1, foff=foff, nsamples=nsamps)
    killmask = [int(rng.random() > 0.03) for _ in range(nchans)]
    g = C.DedispGeometry.make(hdr, nsamps, dms, killmask)
    s = torch.cuda.current_stream().cuda_stream
    dfb = C.DeviceFilterbank(g, s)
    packed = torch.randint(0, 256, (nsamps * nchans * 2 // 8,), dtype=torch.uint8, device=dev)
    dfb.load_packed_device(packed.data_ptr())
    dd = C.Dedisperser(dfb, s)
    ndm = len(dms)
    stride = C.Dedisperser.row_stride(g.out_nsamps)
    for d0, d1 in ((ndm - 64, ndm), (ndm // 2 + 5, ndm // 2 + 40), (700, 732), (0, 32)):
        outs = {}
        for k in (C.DedispKernel.Direct, C.DedispKernel.Packed2, C.DedispKernel.Auto):
            o = torch.zeros((d1 - d0) * stride, dtype=torch.uint8, device=dev)
            dd.run(d0, d1, o.data_ptr(), stride, k)
            outs[k] = o.view(d1 - d0, stride)[:, : g.out_nsamps]
        assert outs[C.DedispKernel.Direct].any()
        for k in (C.DedispKernel.Packed2, C.DedispKernel.Auto):
            assert torch.equal(outs[k], outs[C.DedispKernel.Direct]), (d0, d1, k)


@pytest.mark.parametrize("nbits", [2, 8])
def test_dedisperse_beyond_one_grid_bit_exact(C, nbits):
    """A series longer than one launch (65535 time tiles: 2048 samples for the
    2-bit kernel, 1024 for the byte-VALU and MFMA kernels -- 2^27-sample
    observations) runs as consecutive shifted ranges: equal to the direct
    kernel byte for byte, across the seam."""
    nchans, tsamp, fch1, foff = 16, 64e-6, 1550.0, -400.0 / 16
    dms = C.generate_dm_list(0.0, 60.0, tsamp, 64.0, fch1, foff, nchans, 1.1)[:8]
    delays = C.generate_delay_table(nchans, tsamp, fch1, foff)
    tile = 2048 if nbits == 2 else 1024
    nsamps = 65535 * tile + 70000 + C.compute_max_delay(dms, delays)
    hdr = synthetic.make_header(nchans=nchans, nbits=nbits, tsamp=tsamp, fch1=fch1, foff=foff, nsamples=nsamps)
    g = C.DedispGeometry.make(hdr, nsamps, dms, [1] * nchans)
    s = torch.cuda.current_stream().cuda_stream
    dfb = C.DeviceFilterbank(g, s)
    gen = torch.Generator(device=dev)
    gen.manual_seed(27)
    packed = torch.randint(0, 256, (nsamps * nchans * nbits // 8,), dtype=torch.uint8, device=dev, generator=gen)
    dfb.load_packed_device(packed.data_ptr())
    del packed
    dd = C.Dedisperser(dfb, s)
    stride = C.Dedisperser.row_stride(g.out_nsamps)
    assert g.out_nsamps > 65535 * tile
    kinds = (C.DedispKernel.Packed2,) if nbits == 2 else (C.DedispKernel.Valu, C.DedispKernel.Mfma)
    outs = {}
    for k in (C.DedispKernel.Direct,) + kinds:
        o = torch.zeros(len(dms) * stride, dtype=torch.uint8, device=dev)
        dd.run(0, len(dms), o.data_ptr(), stride, k)
        outs[k] = o.view(len(dms), stride)[:, : g.out_nsamps]
    torch.cuda.synchronize()
    seam = 65535 * tile
    assert outs[C.DedispKernel.Direct][:, seam - 4096: seam + 4096].any()
    for k in kinds:
        assert torch.equal(outs[k], outs[C.DedispKernel.Direct]), k


def test_mfma_resident_plan_ranges_and_side_stream(C):
    """Every range uses the resident plan (ragged per-tile step lists; a
    range inside a tile skips the tile's leading DMs): bit-exact, also on a
    side stream."""
    rng = np.random.default_rng(11)
    nchans, nsamps = 64, 6000
    hdr, dms = _geometry(C, nchans=nchans, nbits=2, nsamps=nsamps, dm_end=900.0)
    ndm = len(dms)
    assert ndm > 70, ndm
    vals = rng.integers(0, 4, size=(nsamps, nchans), dtype=np.uint8)
    g = C.DedispGeometry.make(hdr, nsamps, dms, [])
    s = torch.cuda.current_stream().cuda_stream
    dfb = C.DeviceFilterbank(g, s)
    dfb.load_packed_device(torch.from_numpy(sigproc.pack_samples(vals, 2)).to(dev).data_ptr())
    dd = C.Dedisperser(dfb, s)
    stride = C.Dedisperser.row_stride(g.out_nsamps)
    offs = np.array(g.offsets(0, ndm), dtype=np.int32).reshape(ndm, nchans)
    exp = ref.dedisperse(vals, offs, 2, None, g.out_nsamps)
    T = C.Dedisperser.tile_dms
    side = torch.cuda.Stream()
    for d0, d1 in [(0, T), (T, 2 * T), (2 * T, ndm), (0, ndm), (T, T + 5), (5, 2 * T), (ndm - 3, ndm)]:
        o = torch.zeros((d1 - d0) * stride, dtype=torch.uint8, device=dev)
        for k in (C.DedispKernel.Mfma, C.DedispKernel.Valu):
            o.zero_()
            side.wait_stream(torch.cuda.current_stream())
            dd.run(d0, d1, o.data_ptr(), stride, k, side.cuda_stream)
            side.synchronize()
            got = o.view(d1 - d0, stride)[:, : g.out_nsamps].cpu().numpy()
            assert np.array_equal(got, exp[d0:d1]), (d0, d1, k)


def test_convert_pad_and_truncate():
    from peasoup_amd import ops

    u = torch.randint(0, 256, (1000,), dtype=torch.uint8, device=dev)
    x = ops.convert_pad(u, 1536)
    exp = ref.convert_pad(u.cpu().numpy(), 1536)
    assert np.allclose(x.cpu().numpy(), exp)
    x = ops.convert_pad(u, 512)
    assert np.array_equal(x.cpu().numpy(), u[:512].cpu().numpy().astype(np.float32))


def test_spectrum_forms_and_running_median():
    from peasoup_amd import ops

    rng = np.random.default_rng(3)
    n = 1 << 16
    x = rng.standard_normal(n).astype(np.float32) + np.linspace(0, 5, n, dtype=np.float32)
    X = ops.rfft(torch.from_numpy(x).to(dev))
    Xn = X.cpu().numpy()
    assert np.allclose(Xn, np.fft.rfft(x.astype(np.float64)), rtol=1e-4, atol=1e-2)
    assert np.allclose(ops.form_amplitude(X).cpu().numpy(), ref.amplitude(Xn), rtol=1e-5, atol=1e-5)
    assert np.allclose(ops.form_interbin(X).cpu().numpy(), ref.interbin(Xn), rtol=1e-5, atol=1e-5)
    m5, m25, m125 = ops.running_median(X)
    amp = ref.amplitude(Xn)
    assert np.allclose(m5.cpu().numpy(), ref.median_scrunch5(amp), rtol=1e-6)
    assert np.allclose(m25.cpu().numpy(), ref.median_scrunch5(ref.median_scrunch5(amp)), rtol=1e-6)
    bw = float(np.float32(1.0 / np.float32(n * np.float32(0.00032))))
    zm = ref.zap_mask([10.0, 50.0], [0.3, 0.5], bw, len(Xn))
    bits = np.zeros((len(Xn) + 31) // 32, np.uint32)
    for k in np.nonzero(zm)[0]:
        bits[k >> 5] |= np.uint32(1 << (k & 31))
    zt = torch.from_numpy(bits.view(np.int32)).to(dev)
    Xd = ops.deredden(X.clone(), bw, zt).cpu().numpy()
    exp = ref.deredden(Xn, ref.running_median(amp, bw), zm)
    assert np.allclose(Xd, exp, rtol=2e-5, atol=1e-6)
    import peasoup_amd._C as C

    assert np.array_equal(np.array(C.build_zap_mask([10.0, 50.0], [0.3, 0.5], bw, len(Xn)), dtype=np.uint32), bits)
    P, st = ops.interbin_stats(torch.from_numpy(exp).to(dev))
    mean, rms, std = ref.stats(ref.interbin(exp))
    assert st[0].item() == pytest.approx(mean, rel=1e-5) and st[2].item() == pytest.approx(std, rel=1e-4)


def test_whitening_engine_matches_reference(C):
    """Whitener path of SearchEngine (convert/pad, R2C, median, deredden, zap, C2R)."""
    rng = np.random.default_rng(11)
    nsamps, n = 100000, 1 << 17
    trial = rng.integers(60, 200, size=nsamps, dtype=np.uint8)
    p = C.SearchParams()
    p.fft_size, p.tsamp = n, 0.00032
    p.zap_freqs, p.zap_widths = [50.0], [0.15]
    s = torch.cuda.current_stream().cuda_stream
    eng = C.SearchEngine(p, s)
    t = torch.from_numpy(trial).to(dev)
    eng.search_trial(t.data_ptr(), nsamps, 0.0, 0, [0.0])
    torch.cuda.synchronize()
    w = torch.empty(n, dtype=torch.float32, device=dev)
    stt = torch.empty(3, dtype=torch.float32, device=dev)
    eng.copy_whitened(w.data_ptr())
    eng.copy_stats(stt.data_ptr())
    bw = float(np.float32(1.0 / np.float32(np.float32(n) * np.float32(0.00032))))
    zm = ref.zap_mask([50.0], [0.15], bw, n // 2 + 1)
    exp, st = ref.whiten(trial, n, 0.00032, zm)
    got = w.cpu().numpy()
    scale = np.abs(exp).max()
    assert np.abs(got - exp).max() / scale < 2e-5
    assert stt[0].item() == pytest.approx(st[0], rel=1e-4) and stt[2].item() == pytest.approx(st[2], rel=1e-3)


def test_resample_batch_and_v1():
    from peasoup_amd import ops

    n = 1 << 18
    x = torch.arange(n, dtype=torch.float32, device=dev) % 451  # resampling_test.cpp sawtooth
    accs = [-500.0, -125.5, 0.0, 125.5, 499.0]
    tsamp = 64e-6
    out = ops.resample(x, accs, tsamp).cpu().numpy()
    xn = x.cpu().numpy()
    for k, a in enumerate(accs):
        exp = ref.resample_ii(xn, ref.accel_factor(a, tsamp))
        assert np.array_equal(out[k], exp), a
    v1 = ops.resample_v1(x, 125.5, tsamp).cpu().numpy()
    assert np.array_equal(v1, ref.resample_v1(xn, ref.accel_factor(125.5, tsamp)))
    # resample (II) and v1 agree up to index rounding ties (reference resampling_test.cpp)
    ii = ref.resample_ii(xn, ref.accel_factor(125.5, tsamp))
    assert np.mean(ii != v1) < 1e-3


@pytest.mark.parametrize("nlevels", [1, 2, 3, 4, 5])
def test_harmonic_sums_exact(nlevels):
    from peasoup_amd import ops

    rng = np.random.default_rng(nlevels)
    P = rng.standard_normal(200003).astype(np.float32)
    got = ops.harmonic_sums(torch.from_numpy(P).to(dev), nlevels).cpu().numpy()
    exp = ref.harmonic_sums(P, nlevels)
    for h in range(nlevels):
        assert np.array_equal(got[h], exp[h]), h


def test_harmonic_peaks_matches_threshold_of_sums():
    from peasoup_amd import ops

    rng = np.random.default_rng(2)
    n, Kb, nlev = 120001, 3, 4
    P = rng.standard_normal((Kb, n)).astype(np.float32) * 2.5
    starts = [17, 30, 60, 120, 240]
    ends = [n - 5, n - 100, n, n, n - 1]
    trial, level, idx, snr = ops.harmonic_peaks(torch.from_numpy(P).to(dev), nlev, starts, ends, 9.0)
    got = set(zip(trial.tolist(), level.tolist(), idx.tolist()))
    exp = set()
    for k in range(Kb):
        levels = [P[k]] + ref.harmonic_sums(P[k], nlev)
        for h, L in enumerate(levels):
            sel = np.nonzero(L[starts[h]:ends[h]] > 9.0)[0] + starts[h]
            exp |= {(k, h, int(i)) for i in sel}
    assert got == exp and len(exp) > 50


def test_interbin_normalise_batch():
    from peasoup_amd import ops

    rng = np.random.default_rng(4)
    X = (rng.standard_normal((3, 5001)) + 1j * rng.standard_normal((3, 5001))).astype(np.complex64)
    st = torch.tensor([1.5, 2.0, 0.75, 0.0], dtype=torch.float32, device=dev)
    P = ops.interbin_normalise(torch.from_numpy(X).to(dev), st, 16.0).cpu().numpy()
    mean, sd = np.float32(1.5) * np.float32(16.0), np.float32(0.75) * np.float32(16.0)
    for k in range(3):
        assert np.allclose(P[k], (ref.interbin(X[k]) - mean) / sd, rtol=1e-6, atol=1e-6)


def test_r2c_interbin_normalise_batch():
    """Fused real-FFT post-processing (N/2-point complex FFT) vs numpy rfft."""
    from peasoup_amd import ops

    rng = np.random.default_rng(5)
    n = 1 << 14
    x = rng.standard_normal((3, n)).astype(np.float32)
    st = torch.tensor([1.5, 2.0, 0.75, 0.0], dtype=torch.float32, device=dev)
    P = ops.r2c_interbin_normalise(torch.from_numpy(x).to(dev), st, 1.0).cpu().numpy()
    assert P.shape == (3, n // 2 + 1)
    for k in range(3):
        X = np.fft.rfft(x[k].astype(np.float64))
        exp = (ref.interbin(X.astype(np.complex64)) - 1.5) / 0.75
        assert np.allclose(P[k], exp, rtol=1e-4, atol=2e-3), np.abs(P[k] - exp).max()


def test_r2c_interbin_normalise_rows_matches_numpy(C):
    """The transposing post-processing of the long-series path: a row-major
    half spectrum Z'[k2][k1] = Z[k2 + n2 k1] (row pitch n1 + 8) in, natural
    P out, vs numpy rfft + interbin (every bin 0 .. M, bins M/2 and M
    included)."""
    rng = np.random.default_rng(11)
    n2, n1 = 128, 256
    M = n1 * n2
    n = 2 * M
    K = 2
    x = rng.standard_normal((K, n)).astype(np.float32)
    zp = n1 + 8
    Zr = np.zeros((K, n2, zp), dtype=np.complex64)
    for k in range(K):
        z = np.fft.fft(x[k, 0::2].astype(np.float64) + 1j * x[k, 1::2].astype(np.float64))
        Zr[k, :, :n1] = z.reshape(n1, n2).T.astype(np.complex64)  # Z'[k2][k1] = Z[k2 + n2 k1]
    Zd = torch.from_numpy(Zr.view(np.float32).reshape(-1)).to(dev)
    st = torch.tensor([1.5, 2.0, 0.75, 0.0], dtype=torch.float32, device=dev)
    pst = M + 1 + 7
    P = torch.zeros(K * pst, device=dev)
    qst = (M + 1 + 63) // 64 * 64
    Q = torch.zeros(K * qst, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    C.kernels.r2c_interbin_normalise_rows(Zd.data_ptr(), zp, n2 * zp, 7, n1, P.data_ptr(), pst, K, M + 1,
                                          st.data_ptr(), 1.0, s, Q.data_ptr(), qst)
    torch.cuda.synchronize()
    Pn = P.cpu().numpy().reshape(K, pst)
    Qn = Q.cpu().numpy().reshape(K, qst)[:, : M + 1]
    q_exp = (np.clip(np.rint(Pn[:, : M + 1] * 4.0) + 127.0, -1, 254).astype(np.int64) & 0xFF).astype(np.uint8)
    assert np.array_equal(Qn, q_exp)  # the screening bytes dev::q8 of every P
    for k in range(K):
        X = np.fft.rfft(x[k].astype(np.float64))
        exp = (ref.interbin(X.astype(np.complex64)) - 1.5) / 0.75
        assert np.allclose(Pn[k, : M + 1], exp, rtol=1e-4, atol=2e-3), np.abs(Pn[k, : M + 1] - exp).max()
    g = C.kernels.fft4_geometry_rows(1 << 25)
    assert g.ok and g.rows_ext and (g.n1, g.n2) == (8192, 4096)
    assert not C.kernels.fft4_geometry_rows(1 << 24).ok


def test_long_series_external_rows_match_rocfft_path(C):
    """2^26 points (rows of 8192: beyond the fused passes): the fused resample
    + pass A over columns of 4096, rocFFT over the rows and the transposing
    r2c (fft4_geometry_rows) find the candidates of the plain rocFFT path
    (fft_mode 1: resample kernel + N/2-point C2C), S/N within 1e-4."""
    n = 1 << 26
    g = torch.Generator(device=dev)
    g.manual_seed(26)
    t = torch.arange(n, device=dev, dtype=torch.float64) * 64e-6
    pulse = ((t / 0.0173) % 1.0) < 0.03
    x = 128 + 10 * torch.randn(n, device=dev, generator=g) + 6 * pulse.float()
    row = torch.clamp(torch.round(x), 0, 255).to(torch.uint8)
    del t, pulse, x
    s = torch.cuda.current_stream().cuda_stream
    accs = [-2.0, 0.0, 3.0]
    out = {}
    for mode in (2, 1):
        p = C.SearchParams()
        p.fft_size, p.tsamp, p.nharmonics, p.fft_mode = n, 64e-6, 3, mode
        e = C.SearchEngine(p, s)
        assert e.fft_mode == mode and e.rows_ext == (mode == 2)
        cands = e.search_trial(row.data_ptr(), n, 10.0, 0, accs)
        torch.cuda.synchronize()
        out[mode] = sorted(cands, key=lambda c: -c.snr)
        del e
    a, b = out[2], out[1]
    assert len(a) > 0 and abs(len(a) - len(b)) <= max(2, len(b) // 20), (len(a), len(b))
    for ca, cb in zip(a[:10], b[:10]):
        assert (round(ca.freq, 6), ca.nh, ca.acc) == (round(cb.freq, 6), cb.nh, cb.acc)
        assert abs(ca.snr - cb.snr) <= 1e-4 * abs(cb.snr) + 1e-3, (ca.snr, cb.snr)
    assert abs(1.0 / a[0].freq - 0.0173) < 1e-3 or any(abs(1.0 / c.freq - 0.0173) < 1e-4 for c in a[:5])


# Every prefix of the kernel-shape chain (kernels.hpp Fft4Flags): None = the
# default (1074216195 = 212227 | kFft4StripInput | kFft4PairY); 0 / 1 =
# natural layouts (2 x 4 / 8 transforms per thread); 259 = blocked; 1299 = +
# tiled Y; 3331 = + tiled X; 7427 = + paired XCD blocks; 15619 = + grouped XCD
# blocks; 81155 = + uniform pass-A twiddles (the Stockham pass A); 212227 = +
# the one-exchange pass A on the row-pitch input.  (kFft4PairY only changes
# the fused spectrum pass's input: tests/test_spectrum_gpu.py.)
FFT4_FLAG_SETS = [None, 0, 1, 259, 1299, 3331, 7427, 15619, 81155, 212227]


@pytest.fixture(params=FFT4_FLAG_SETS)
def fft4_flags(request):
    import peasoup_amd._C as C

    old = C.kernels.fft4_flags()
    if request.param is not None:
        C.kernels.fft4_set_flags(request.param)
    yield request.param
    C.kernels.fft4_set_flags(old)


@pytest.mark.parametrize("log2n", [15, 17, 20, 23, 25])
def test_fft4_resample_spectrum_matches_numpy(log2n, fft4_flags):
    """Fused resample + four-step FFT vs (bit-exact GPU resample) + numpy fp64 FFT."""
    from peasoup_amd import ops

    rng = np.random.default_rng(log2n)
    n = 1 << log2n
    x = torch.from_numpy(rng.standard_normal(n).astype(np.float32)).to(dev)
    accs = [-480.0, 0.0, 37.5, 500.0] if log2n < 23 else ([-500.0, 250.0] if log2n == 23 else [310.0])
    Z = ops.fft4_resample_spectrum(x, accs, 64e-6).cpu().numpy()
    R = ops.resample(x, accs, 64e-6).cpu().numpy().astype(np.float64)
    for k in range(len(accs)):
        z = R[k, 0::2] + 1j * R[k, 1::2]
        ref_Z = np.fft.fft(z)
        err = np.abs(Z[k] - ref_Z)
        scale = np.sqrt(np.mean(np.abs(ref_Z) ** 2))
        assert err.max() / scale < 5e-5, (k, err.max() / scale)
        assert np.sqrt(np.mean(err ** 2)) / scale < 5e-6


def test_fold_optimise_matches_fft_reference():
    from peasoup_amd import ops

    rng = np.random.default_rng(9)
    folds = rng.standard_normal((6, 16, 64)).astype(np.float32)
    # add a drifting narrow pulse to some folds
    for f in range(3):
        for i in range(16):
            folds[f, i, (20 + (i * (f + 1)) // 4) % 64] += 8.0
    oi, of, op = ops.fold_optimise(torch.from_numpy(folds).to(dev))
    oi, of, op = oi.cpu().numpy(), of.cpu().numpy(), op.cpu().numpy()
    for f in range(6):
        t, s, j, ofold, oprof = ref.fold_optimise(folds[f])
        if f < 3:
            assert (oi[f, 0], oi[f, 1], oi[f, 2]) == (t, s, j)
            assert np.allclose(of[f], ofold, rtol=1e-3, atol=1e-2)
            assert np.allclose(op[f], oprof, rtol=1e-3, atol=1e-2)


def test_fold_series_against_reference(C):
    from peasoup_amd import ops

    n, tsamp, period = 1 << 18, 0.00032, 0.2513
    t = np.arange(n) * tsamp
    ph = (t / period) % 1.0
    x = (np.exp(-0.5 * ((ph - 0.3) / 0.02) ** 2) * 5 + np.random.default_rng(1).standard_normal(n)).astype(np.float32)
    res = ops.fold_series(torch.from_numpy(x).to(dev), [period], [0.0], tsamp)[0]
    fold_ref = ref.fold_series(x, period, float(np.float32(tsamp)))  # the folder's tsamp is float32
    t_, s_, j_, ofold, oprof = ref.fold_optimise(fold_ref)
    assert res.opt_width == t_ + 1
    sn1, sn2 = ref.calculate_sn(oprof, j_ - t_ // 2, t_)
    # float32 fold sums in a different order than the double-precision oracle
    assert res.folded_snr == pytest.approx(max(sn1, sn2), rel=1e-2)
    assert np.allclose(np.array(res.fold).reshape(16, 64), ofold, rtol=2e-3, atol=2e-2)


def test_calculate_sn_host(C):
    rng = np.random.default_rng(6)
    prof = rng.standard_normal(64).astype(np.float32)
    prof[40:44] += 10
    for b, w in ((41, 3), (5, 7), (60, 1)):
        a, c = C.fold_calculate_sn(list(prof), b, w)
        ea, ec = ref.calculate_sn(prof, b, w)
        assert a == pytest.approx(ea, rel=1e-5) and c == pytest.approx(ec, rel=1e-5)


def test_coincidence_and_correlation_ops():
    from peasoup_amd import ops

    rng = np.random.default_rng(8)
    beams = [rng.standard_normal(10000).astype(np.float32) * 3 for _ in range(5)]
    counts = None
    for b in beams:
        counts = ops.coincidence_counts(torch.from_numpy(b).to(dev), 4.0, counts)
    mask = ops.coincidence_mask(counts, 2).cpu().numpy()
    assert np.array_equal(mask, ref.coincidence_mask(beams, 4.0, 2))
    x = torch.from_numpy((rng.standard_normal(999) + 1j * rng.standard_normal(999)).astype(np.complex64)).to(dev)
    y = torch.from_numpy((rng.standard_normal(999) + 1j * rng.standard_normal(999)).astype(np.complex64)).to(dev)
    exp = np.conj(x.cpu().numpy()) * y.cpu().numpy()
    ops.cmul_(ops.conjugate(x), y)
    assert np.allclose(y.cpu().numpy(), exp, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("log2n", [16, 21])
def test_fft4_interbin_path_matches_rocfft_path(log2n, fft4_flags):
    """fft_mode 2 hot path (padded spectrum layout) == resample + C2C + r2c post."""
    from peasoup_amd import ops

    rng = np.random.default_rng(100 + log2n)
    n = 1 << log2n
    x = torch.from_numpy(rng.standard_normal(n).astype(np.float32)).to(dev)
    accs = [-300.0, 0.0, 410.0]
    st = torch.tensor([1.0, 2.0, 0.5, 0.0], dtype=torch.float32, device=dev)
    P2 = ops.fft4_resample_interbin(x, accs, 64e-6, st, float(n)).cpu().numpy()
    R = ops.resample(x, accs, 64e-6).contiguous()
    P1 = ops.r2c_interbin_normalise(R, st, float(n)).cpu().numpy()
    assert P2.shape == P1.shape == (3, n // 2 + 1)
    scale = np.abs(P1).max()
    assert np.abs(P2 - P1).max() / scale < 1e-4
    assert np.sqrt(np.mean((P2 - P1) ** 2)) / np.sqrt(np.mean(P1 ** 2)) < 1e-5


@pytest.mark.parametrize("log2n,frac", [(21, 0.1), (21, 0.37), (23, 0.1408), (21, 0.499)])
def test_fft4_pruned_spectrum_rows_match_full(log2n, frac):
    """Search path: pass B stores only the spectrum rows the tiled r2c reads
    for bins < nbins_out; those bins are bit-identical to the unpruned path."""
    from peasoup_amd import ops

    rng = np.random.default_rng(7 + log2n)
    n = 1 << log2n
    x = torch.from_numpy(rng.standard_normal(n).astype(np.float32)).to(dev)
    accs = [-250.0, 0.0, 120.0, 499.0, -499.0, 3.0, 7.0, -1.0]
    st = torch.tensor([1.0, 2.0, 0.5, 0.0], dtype=torch.float32, device=dev)
    nbo = int(frac * n)
    full = ops.fft4_resample_interbin(x, accs, 64e-6, st, float(n))
    pruned = ops.fft4_resample_interbin(x, accs, 64e-6, st, float(n), nbins_out=nbo)
    assert torch.equal(full[:, :nbo], pruned[:, :nbo])
    assert torch.count_nonzero(pruned[:, nbo:]) == 0


@pytest.mark.parametrize("nlev,thresh", [(1, 6.0), (3, 9.0), (3, 11.5), (5, 10.0)])
def test_harmonic_prethreshold_is_exact(nlev, thresh):
    """The conservative unscaled pre-threshold (fast no-peak path) never drops a
    peak: records equal the exact-path records and the threshold of the
    reference sums."""
    import peasoup_amd._C as C
    from peasoup_amd import ops

    rng = np.random.default_rng(40 + nlev)
    n, Kb = 70001, 8
    P = rng.standard_normal((Kb, n)).astype(np.float32) * 3.0
    starts = [3, 5, 9, 17, 33, 65]
    ends = [n] * 6
    Pt = torch.from_numpy(P).to(dev)
    runs = []
    old = C.kernels.harmonic_flags()
    try:
        # bit 1 disables the pre-threshold; bit 5 = two-phase staging (3 levels),
        # bits 8-15 = occupancy cap; the default is 1 | 8 | 32 | (10 << 8)
        for flags in (1, 3, 33, 35, 1 | 32 | (10 << 8), old):
            C.kernels.harmonic_set_flags(flags)
            trial, level, idx, snr = ops.harmonic_peaks(Pt, nlev, starts, ends, thresh)
            runs.append(sorted(zip(trial.tolist(), level.tolist(), idx.tolist(), snr.tolist())))
    finally:
        C.kernels.harmonic_set_flags(old)
    assert all(r == runs[0] for r in runs) and len(runs[0]) > 20
    exp = set()
    for k in range(Kb):
        levels = [P[k]] + ref.harmonic_sums(P[k], nlev)
        for h, L in enumerate(levels):
            sel = np.nonzero(L[starts[h]:ends[h]] > thresh)[0] + starts[h]
            exp |= {(k, h, int(i)) for i in sel}
    assert {r[:3] for r in runs[0]} == exp


def test_parallel_host_distillation_is_deterministic(C):
    """Peak-heavy batches (low threshold: tens of thousands of records) are
    clustered/distilled on the host pool; candidates equal the serial path."""
    rng = np.random.default_rng(21)
    nsamps, n = 200000, 1 << 17
    t = (np.arange(nsamps) * 0.00032) / 0.0731
    trial = np.clip(rng.normal(128, 6, nsamps) + 9.0 * ((t % 1.0) < 0.03), 0, 255).astype(np.uint8)
    tt = torch.from_numpy(trial).to(dev)
    accs = [float(a) for a in np.linspace(-40, 40, 48)]
    s = torch.cuda.current_stream().cuda_stream
    runs = []
    for ht in (1, 6):
        p = C.SearchParams()
        p.fft_size, p.tsamp, p.nharmonics, p.min_snr = n, 0.00032, 3, 2.5
        p.host_threads = ht
        eng = C.SearchEngine(p, s)
        cands = eng.search_trial(tt.data_ptr(), nsamps, 5.0, 0, accs)
        torch.cuda.synchronize()
        assert eng.counters()["peaks"] > 8192 * 2  # the parallel branch is taken
        runs.append([(c.acc, c.nh, c.snr, c.freq, len(c.assoc)) for c in cands])
    assert runs[0] == runs[1] and len(runs[0]) > 0


@pytest.mark.parametrize("batch,sub", [(4, 0), (7, 0), (16, 8), (64, 32)])
def test_results_independent_of_accel_batching(C, batch, sub):
    """Regression: with more acceleration trials than two batches the slots
    are re-issued before their peak records are processed (and the last
    batch is partial); candidates (incl. their accelerations) must not depend
    on the batch size or sub-batching."""
    rng = np.random.default_rng(33)
    nsamps, n = 1100000, 1 << 20
    tsamp = 64e-6
    t = np.arange(nsamps) * tsamp
    # accelerated pulsar (synthetic.py convention): phase = (t - a t^2 / 2c) / P;
    # over 67 s the drift is ~1.2 turns, so the acceleration is measurable
    a_true = 310.0
    ph = ((t - a_true * t * t / (2 * 299792458.0)) / 0.002) % 1.0
    trial = np.clip(rng.normal(128, 6, nsamps) + 2.0 * (np.minimum(ph, 1 - ph) < 0.04), 0, 255).astype(np.uint8)
    tt = torch.from_numpy(trial).to(dev)
    accs = [float(a) for a in np.linspace(-500, 500, 101)]
    s = torch.cuda.current_stream().cuda_stream
    runs = []
    for b, sb in ((200, 0), (batch, sub)):
        p = C.SearchParams()
        p.fft_size, p.tsamp, p.nharmonics, p.min_snr = n, tsamp, 3, 6.0
        p.accel_batch, p.sub_batch = b, sb
        eng = C.SearchEngine(p, s)
        cands = eng.search_trial(tt.data_ptr(), nsamps, 1.0, 0, accs)
        torch.cuda.synchronize()
        runs.append(sorted((c.acc, c.nh, c.snr, c.freq) for c in cands))
    assert runs[0] == runs[1] and len(runs[0]) > 0
    best = max(runs[1], key=lambda r: r[2])
    assert abs(best[0] - a_true) <= 30.0, best


def test_auto_short_list_balancing_matches_fixed_batch(C):
    """the auto path that cuts a short trial list into min_batches
    even batches (kc < K) gives the same candidates as fixed batches, and its
    buffers only hold the batch actually used."""
    rng = np.random.default_rng(34)
    nsamps, n, tsamp = 1100000, 1 << 20, 64e-6
    t = np.arange(nsamps) * tsamp
    ph = ((t - 250.0 * t * t / (2 * 299792458.0)) / 0.003) % 1.0
    trial = np.clip(rng.normal(128, 6, nsamps) + 2.0 * (np.minimum(ph, 1 - ph) < 0.04), 0, 255).astype(np.uint8)
    tt = torch.from_numpy(trial).to(dev)
    accs = [float(a) for a in np.linspace(-500, 500, 101)]
    s = torch.cuda.current_stream().cuda_stream
    runs = []
    for auto in (False, True):
        p = C.SearchParams()
        p.fft_size, p.tsamp, p.nharmonics, p.min_snr = n, tsamp, 3, 6.0
        if auto:
            # budget of exactly 64 trials: Y + blocked P + screening bytes per trial with the fused
            # spectrum pass (harmonic flag 64, the default), else Y + X + P + bytes (the search range
            # covers all bins)
            nb = n // 2 + 1
            if C.kernels.harmonic_flags() & 64:
                pst = (nb + 63) // 64 * 64
                per = n * 4 + pst * 4 + (pst + C.kernels.spec_q_shift + 63) // 64 * 64
            else:
                per = n * 4 + nb * 8 + nb * 4 + (nb + 63) // 64 * 64
            p.accel_batch, p.batch_bytes, p.min_batches = 0, 64 * per, 8
        else:
            p.accel_batch, p.sub_batch = 24, 0
        eng = C.SearchEngine(p, s)
        cands = eng.search_trial(tt.data_ptr(), nsamps, 1.0, 0, accs)
        torch.cuda.synchronize()
        if auto:
            assert eng.batch_size == 64
            assert eng.last_batch == 16  # 101 trials < 8 x 64: 8 even batches, floored at k_small = 16
        runs.append(sorted((c.acc, c.nh, c.snr, c.freq) for c in cands))
    assert runs[0] == runs[1] and len(runs[0]) > 0


@pytest.mark.parametrize("log2n", [17, 20, 23])
def test_whitener_real_ffts_on_fft4_match_numpy(C, log2n):
    """Whitener R2C/C2R on the four-step passes (K = 1) vs NumPy fp64 and the
    rocFFT fallback: unnormalised like rocFFT (C2R(R2C(x)) = N x)."""
    n = 1 << log2n
    rng = np.random.default_rng(log2n)
    x = rng.standard_normal(n).astype(np.float32)
    s = torch.cuda.current_stream().cuda_stream
    xs = torch.from_numpy(x).to(dev)
    ref_spec = np.fft.rfft(x.astype(np.float64))
    scale = np.abs(ref_spec).max()
    outs = {}
    for f4 in (True, False):
        w = C.Whitener(n, 64e-6, s, f4)
        assert w.uses_fft4 == f4
        X = torch.empty(n // 2 + 1, dtype=torch.complex64, device=dev)
        w.forward(xs.data_ptr(), X.data_ptr())
        torch.cuda.synchronize()
        Xn = X.cpu().numpy()
        y = torch.empty(n, dtype=torch.float32, device=dev)
        w.inverse(X.data_ptr(), y.data_ptr())  # (rocFFT's out-of-place C2R may overwrite X)
        torch.cuda.synchronize()
        assert np.abs(Xn - ref_spec).max() < 2e-6 * scale * log2n, f4
        assert np.allclose(y.cpu().numpy() / n, x, atol=2e-5 * log2n), f4
        outs[f4] = Xn
    assert np.abs(outs[True] - outs[False]).max() < 2e-6 * scale * log2n


@pytest.mark.parametrize("m,log2p", [(3, 14), (17, 16)])
def test_whitener_mixed_radix_ffts_match_numpy(C, m, log2p):
    """Lengths with an odd factor (n = m 2^k, e.g. the coincidencer's
    1114112-sample DM-0 series) run as m batched power-of-two four-step FFTs
    plus a length-m combination -- no rocFFT runtime compilation -- and match
    NumPy's rfft / unnormalised irfft."""
    n = m << log2p
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n).astype(np.float32)
    s = torch.cuda.current_stream().cuda_stream
    w = C.Whitener(n, 64e-6, s, True)
    assert w.mixed_radix and w.uses_fft4
    xs = torch.from_numpy(x).to(dev)
    X = torch.empty(n // 2 + 1, dtype=torch.complex64, device=dev)
    w.forward(xs.data_ptr(), X.data_ptr())
    torch.cuda.synchronize()
    ref = np.fft.rfft(x.astype(np.float64))
    scale = np.abs(ref).max()
    assert np.abs(X.cpu().numpy() - ref).max() < 2e-6 * scale * np.log2(n)
    y = torch.empty(n, dtype=torch.float32, device=dev)
    w.inverse(X.data_ptr(), y.data_ptr())
    torch.cuda.synchronize()
    assert np.allclose(y.cpu().numpy() / n, x, atol=2e-5 * np.log2(n))


def test_batched_whitening_matches_single_trial(C):
    """SearchEngine.prepare(count) + search_prepared(b) (one K = count
    four-step FFT pair for the whitening) gives the candidates, whitened
    series and stats of search_trial on each trial alone."""
    rng = np.random.default_rng(5)
    n, nsamps, count = 1 << 18, (1 << 18) + 300, 5
    rs = 1 << 19
    t = np.arange(nsamps) * 64e-6
    rows = np.zeros((count, rs), dtype=np.uint8)
    for b in range(count):
        x = rng.normal(128, 10, nsamps) + 25 * (((t / (0.0213 * (1 + 0.1 * b))) % 1.0) < 0.03)
        rows[b, :nsamps] = np.clip(np.rint(x), 0, 255).astype(np.uint8)
    d = torch.from_numpy(rows).to(dev)
    p = C.SearchParams()
    p.fft_size, p.tsamp, p.nharmonics = n, 64e-6, 3
    s = torch.cuda.current_stream().cuda_stream
    e1, e2 = C.SearchEngine(p, s), C.SearchEngine(p, s)
    assert e2.max_prepare >= count
    accs = [-20.0, 0.0, 35.0]
    e2.prepare(d.data_ptr(), rs, nsamps, count)
    key = lambda c: (round(c.freq, 7), c.acc, c.nh, c.snr)  # noqa: E731
    for b in range(count):
        single = e1.search_trial(d.data_ptr() + b * rs, nsamps, 10.0, b, accs)
        w1 = torch.empty(n, dtype=torch.float32, device=dev)
        e1.copy_whitened(w1.data_ptr())
        batched = e2.search_prepared(b, 10.0, b, accs)
        w2 = torch.empty(n, dtype=torch.float32, device=dev)
        e2.copy_whitened(w2.data_ptr())
        assert torch.equal(w1, w2), b
        assert sorted(map(key, single)) == sorted(map(key, batched)), b
        assert len(single) > 0


@pytest.mark.parametrize("log2n", [18, 20, 23])
def test_whitening_direct_sources_equal_padded_path(C, log2n):
    """kFft4WhitenStrips, forward: the batched whitener's pass A reads the
    8-bit rows staged into column strips (or the 8-bit rows themselves,
    kFft4WhitenU8, or the unpadded f32 rows, kFft4WhitenF32); inverse: the
    half spectra with the C2R pre-processing applied on the fly.  At column
    length 2048 the one-exchange pass A reads the strips.  All give
    bit-identical whitened series to the f32 copy + pad + c2r_pre kernels
    (rows shorter than n: the mean-padded tail)."""
    WS, U8, F32 = 16777216, 33554432, 67108864
    rng = np.random.default_rng(log2n)
    n, count = 1 << log2n, 3
    nsamps = n - 1000
    rs = n + 64
    rows = torch.from_numpy(rng.integers(90, 170, (count, rs), dtype=np.uint8)).to(dev)
    p = C.SearchParams()
    p.fft_size, p.tsamp, p.nharmonics = n, 64e-6, 3
    s = torch.cuda.current_stream().cuda_stream
    f0 = C.kernels.fft4_flags()
    assert f0 & WS
    out = {}
    try:
        for f in (f0 & ~WS, f0 & ~(U8 | F32), (f0 & ~F32) | U8, (f0 & ~U8) | F32):
            C.kernels.fft4_set_flags(f)
            e = C.SearchEngine(p, s)
            e.prepare(rows.data_ptr(), rs, nsamps, count)
            ws = []
            for b in range(count):
                e.search_prepared(b, 5.0, b, [0.0])
                w = torch.empty(n, dtype=torch.float32, device=dev)
                e.copy_whitened(w.data_ptr())
                ws.append(w)
            torch.cuda.synchronize()
            out[f] = ws
            del e
    finally:
        C.kernels.fft4_set_flags(f0)
    for b in range(count):
        for f in (f0 & ~(U8 | F32), (f0 & ~F32) | U8, (f0 & ~U8) | F32):
            assert torch.equal(out[f][b], out[f0 & ~WS][b]), (b, f)
        assert out[f0 & ~WS][b].abs().max() > 0


@pytest.mark.parametrize("log2n", [20, 21, 23])
def test_whitening_into_padded_input_equals_pad_kernel(C, monkeypatch, log2n):
    """fft4_c2r_post_pad: the whitener's inverse writes pass A's padded row
    input directly (no unpadded series, no pad kernel), and pass A's
    off-band fallback reads the padded copy; deredden_zap_stats: dereddening
    and the interbin statistics in one out-of-place pass.  The whitened
    series and every candidate of an accelerated search equal those of the
    two-kernel sequences (PSOUP_WHITEN_PAD_DIRECT=0,
    PSOUP_WHITEN_FUSED_STATS=0) bit for bit (2^23: the strip layout keeps
    the pad kernel)."""
    rng = np.random.default_rng(log2n)
    n, count = 1 << log2n, 3
    nsamps = n - 700
    rs = n + 64
    t = np.arange(nsamps) * 64e-6
    rows = np.zeros((count, rs), dtype=np.uint8)
    for b in range(count):
        x = rng.normal(128, 10, nsamps) + 30 * (((t / (0.0123 * (1 + 0.1 * b))) % 1.0) < 0.04)
        rows[b, :nsamps] = np.clip(np.rint(x), 0, 255).astype(np.uint8)
    d = torch.from_numpy(rows).to(dev)
    p = C.SearchParams()
    p.fft_size, p.tsamp, p.nharmonics = n, 64e-6, 3
    s = torch.cuda.current_stream().cuda_stream
    accs = list(np.linspace(-300, 300, 23))
    key = lambda c: (c.dm_idx, c.freq, c.acc, c.nh, c.snr)  # noqa: E731
    res = {}
    for direct in ("00", "10", "11"):
        monkeypatch.setenv("PSOUP_WHITEN_PAD_DIRECT", direct[0])
        monkeypatch.setenv("PSOUP_WHITEN_FUSED_STATS", direct[1])
        e = C.SearchEngine(p, s)
        e.prepare(d.data_ptr(), rs, nsamps, count)
        many = e.search_prepared_many([(b, 5.0 + b, b, accs) for b in range(count)])
        w = torch.empty(n, dtype=torch.float32, device=dev)
        e.copy_whitened(w.data_ptr())  # the current search's first series
        torch.cuda.synchronize()
        res[direct] = ([sorted(map(key, many[b])) for b in range(count)], w)
        del e
    for v in ("10", "11"):
        assert res["00"][0] == res[v][0] and sum(len(c) for c in res[v][0]) > 0, v
        assert torch.equal(res["00"][1], res[v][1]) and res[v][1].abs().max() > 0, v


def test_flat_multi_dm_batches_match_per_dm_search(C):
    """search_prepared_many: the trials of several DMs concatenated and cut
    into K-trial batches across DM boundaries (per-trial series index and
    whitening stats) give each DM exactly the candidates of its own search."""
    rng = np.random.default_rng(9)
    n, nsamps, count = 1 << 18, (1 << 18) + 300, 5
    rs = 1 << 19
    t = np.arange(nsamps) * 64e-6
    rows = np.zeros((count, rs), dtype=np.uint8)
    for b in range(count):
        x = rng.normal(128, 10, nsamps) + 25 * (((t / (0.0171 * (1 + 0.13 * b))) % 1.0) < 0.03)
        rows[b, :nsamps] = np.clip(np.rint(x), 0, 255).astype(np.uint8)
    d = torch.from_numpy(rows).to(dev)
    p = C.SearchParams()
    p.fft_size, p.tsamp, p.nharmonics, p.accel_batch = n, 64e-6, 3, 16
    s = torch.cuda.current_stream().cuda_stream
    e1, e2 = C.SearchEngine(p, s), C.SearchEngine(p, s)
    acc_lists = [list(np.linspace(-40, 40, k)) for k in (3, 37, 1, 16, 10)]
    e2.prepare(d.data_ptr(), rs, nsamps, count)
    many = e2.search_prepared_many([(b, 5.0 + b, b, acc_lists[b]) for b in range(count)])
    key = lambda c: (c.dm_idx, round(c.freq, 7), c.acc, c.nh, c.snr)  # noqa: E731
    total = 0
    for b in range(count):
        single = e1.search_trial(d.data_ptr() + b * rs, nsamps, 5.0 + b, b, acc_lists[b])
        assert sorted(map(key, single)) == sorted(map(key, many[b])), b
        total += len(single)
    assert total > 0


