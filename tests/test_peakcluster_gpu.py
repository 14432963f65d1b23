"""GPU peak clustering (kern::peak_cluster_batch) against the reference's
host scan (identify_unique_peaks, include/transforms/peakfinder.hpp:24-55),
and the search engine with device clustering against host clustering."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def _segment(rng, n, span, ties):
    idx = np.sort(rng.choice(span, n, replace=False)).astype(np.int32)
    # bumps (runs of crossings rising to a peak and falling) plus noise
    snr = 9.0 + 40.0 * rng.random(n)
    for c in rng.choice(span, max(1, n // 200), replace=False):
        snr += 200.0 * np.exp(-0.5 * ((idx - c) / (5 + 40 * rng.random())) ** 2)
    if ties:
        snr = np.round(snr * 2) / 2  # equal S/N neighbours: the strict '>' rule
    return idx, snr.astype(np.float32)


def chunked_records(segs, rng):
    """Records as harmonic_peaks_batch emits them: per segment, runs of
    idx-ascending crossings of one 64-bin group, each behind its descriptor
    {0x80000000 | count << 16 | segment, first idx, position}; chunks in any
    order (kernels.hpp kPeakChunk)."""
    chunks = []
    for s, (idx, snr) in segs.items():
        grp = idx >> 6
        cuts = np.flatnonzero(np.diff(grp)) + 1
        for a, b in zip(np.r_[0, cuts], np.r_[cuts, len(idx)]):
            chunks.append((s, idx[a:b], snr[a:b]))
    order = rng.permutation(len(chunks))
    rows, pos = [], 0
    for k in order:
        s, ci, cs = chunks[k]
        c = len(ci)
        rows.append(np.array([[0x80000000 | (c << 16) | s, int(ci[0]), pos + 1]], np.uint32))
        rows.append(np.stack([np.full(c, s, np.uint32), ci.view(np.uint32), cs.view(np.uint32)], axis=1))
        pos += 1 + c
    return np.concatenate(rows)


@pytest.mark.parametrize("gap", [30, 5, 1])
def test_peak_cluster_matches_host_scan(C, gap):
    K = C.kernels
    rng = np.random.default_rng(3 + gap)
    cap_seg = int(K.cluster_cap)
    sizes = [0, 1, 2, 31, 64, 65, 500, 4096, 4097, 5000, cap_seg, cap_seg + 1, 20000, 7, 0, 900, 12000, 3]
    segs = {}
    recs = []
    for s, n in enumerate(sizes):
        if n == 0:
            continue
        span = n * (1 + s % 4) + 10  # dense (most within the gap) to sparse
        idx, snr = _segment(rng, n, span, ties=s % 2 == 0)
        segs[s] = (idx, snr)
    allr = chunked_records(segs, rng)  # chunks land in any order
    n = len(allr)
    nseg = len(sizes)
    cap = n + 100
    peaks = torch.from_numpy(allr.reshape(-1).view(np.int32).copy()).to(dev)
    count = torch.tensor([n], dtype=torch.int32, device=dev)
    work = torch.empty(5 * nseg, dtype=torch.int32, device=dev)
    srt = torch.empty(4 * cap, dtype=torch.int32, device=dev)
    out = torch.empty(2 * cap, dtype=torch.int32, device=dev)
    tab = torch.empty(2 * nseg, dtype=torch.int32, device=dev)
    tot = torch.zeros(1, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    K.peak_cluster_batch(peaks.data_ptr(), count.data_ptr(), cap, nseg, gap, work.data_ptr(), srt.data_ptr(),
                         out.data_ptr(), tab.data_ptr(), tot.data_ptr(), s)
    torch.cuda.synchronize()
    tab_h = tab.cpu().numpy().view(np.uint32).reshape(nseg, 2)
    out_h = out.cpu().numpy().view(np.uint32).reshape(cap, 2)
    srt_h = srt.cpu().numpy().view(np.uint32).reshape(2 * cap, 2)[cap:]  # raw segments: the second half
    assert int(tot.item()) == sum(int(tab_h[s_, 1]) for s_ in range(nseg) if not tab_h[s_, 1] & 0x80000000)
    for s_, sz in enumerate(sizes):
        first, cnt = int(tab_h[s_, 0]), int(tab_h[s_, 1])
        if sz == 0:
            assert cnt == 0
            continue
        idx, snr = segs[s_]
        if sz > cap_seg:  # left to the host: the raw crossings of exactly this segment
            assert cnt == (sz | 0x80000000), (s_, hex(cnt))
            raw = srt_h[first:first + sz]
            assert np.array_equal(np.sort(raw[:, 0].astype(np.int32)), idx)
            continue
        exp_i, exp_s = C.identify_unique_peaks(idx.tolist(), snr.tolist(), gap)
        got = out_h[first:first + cnt]
        assert cnt == len(exp_i), (s_, sz, cnt, len(exp_i))
        assert np.array_equal(got[:, 0].astype(np.int32), np.array(exp_i, np.int32)), s_
        assert np.array_equal(got[:, 1].view(np.float32), np.array(exp_s, np.float32)), s_


def _search(C, trial, nsamps, accs, gpu_cluster):
    os.environ["PSOUP_GPU_CLUSTER"] = "1" if gpu_cluster else "0"
    try:
        p = C.SearchParams()
        p.fft_size, p.tsamp, p.nharmonics = 1 << 20, 64e-6, 4
        eng = C.SearchEngine(p, torch.cuda.current_stream().cuda_stream)
        c = eng.search_trial(trial.data_ptr(), nsamps, 10.0, 3, accs)
        ctr = eng.counters()
    finally:
        os.environ.pop("PSOUP_GPU_CLUSTER", None)
    return [(x.dm_idx, x.acc, x.nh, x.snr, x.freq) for x in c], ctr


def test_engine_gpu_clustering_equals_host(C):
    """A peak-heavy trial (bright narrow pulse train + strong undispersed
    periodic RFI): device clustering gives the candidate list of the host
    scan, field for field."""
    rng = np.random.default_rng(5)
    n = (1 << 20) + 512
    t = np.arange(n) * 64e-6
    x = rng.normal(128, 6, n)
    for per, amp in ((0.00731, 30.0), (0.02, 60.0), (0.0613, 25.0)):
        ph = (t / per) % 1.0
        x += amp * (np.minimum(ph, 1 - ph) < 0.015)
    trial = torch.from_numpy(np.clip(np.rint(x), 0, 255).astype(np.uint8)).to(dev)
    accs = [float(a) for a in np.linspace(-60, 60, 41)]
    host, ch = _search(C, trial, n, accs, False)
    gpu, cg = _search(C, trial, n, accs, True)
    assert ch["peaks"] > 100000, ch  # peak-heavy: the clustering matters
    assert cg["peaks"] == ch["peaks"]
    assert len(gpu) == len(host) and len(gpu) > 0
    assert gpu == host


def _search_regions(C, trial, nsamps, accs, rlog2, min_snr):
    p = C.SearchParams()
    p.fft_size, p.tsamp, p.nharmonics, p.min_snr = 1 << 20, 64e-6, 4, min_snr
    p.accel_batch, p.peak_region_log2 = 8, rlog2
    eng = C.SearchEngine(p, torch.cuda.current_stream().cuda_stream)
    c = eng.search_trial(trial.data_ptr(), nsamps, 10.0, 3, accs)
    return [(x.dm_idx, x.acc, x.nh, x.snr, x.freq) for x in c], eng.counters()


@pytest.mark.parametrize("min_snr", [6.0, 1.5])
def test_engine_record_regions_equal_one_counter(C, min_snr):
    """Threshold crossings in 64 record regions (SearchParams.peak_region_log2,
    one reservation counter each) give the candidates of the single counter;
    at S/N 1.5 the 8-trial batches overflow their regions (4096 records each)
    and are recomputed with the capacity the fullest region asked for."""
    rng = np.random.default_rng(9)
    n = (1 << 20) + 512
    t = np.arange(n) * 64e-6
    x = rng.normal(128, 6, n)
    for per, amp in ((0.00731, 30.0), (0.02, 60.0)):
        ph = (t / per) % 1.0
        x += amp * (np.minimum(ph, 1 - ph) < 0.015)
    trial = torch.from_numpy(np.clip(np.rint(x), 0, 255).astype(np.uint8)).to(dev)
    accs = [float(a) for a in np.linspace(-40, 40, 17)]
    one, c1 = _search_regions(C, trial, n, accs, 0, min_snr)
    reg, c6 = _search_regions(C, trial, n, accs, 6, min_snr)
    assert c6["peaks"] == c1["peaks"] and c1["peaks"] > 50000, (c1, c6)
    if min_snr < 4:
        assert c6["overflows"] > 0, (c6["peaks"], c6["overflows"])
    assert len(reg) == len(one) and len(one) > 0
    assert reg == one


def test_harmonic_regions_kernel_level(C):
    """harmonic_peaks_batch with 8 record regions: every region's records are
    whole chunks at absolute positions, the union equals the single-counter
    records, and peak_regions_total reports the sum -- or, when a region
    overflows, 8 x its count (more than the capacity)."""
    from peasoup_amd import ops

    K = C.kernels
    rng = np.random.default_rng(12)
    Kb, n = 16, 1 << 18
    P = torch.from_numpy((rng.exponential(1.0, (Kb, n)) - 1.0).astype(np.float32)).to(dev)
    starts, ends, thr = [3, 5, 9, 17], [n] * 4, 3.0
    Q = ops.quantize_q8(P)
    s = torch.cuda.current_stream().cuda_stream
    ref = ops.harmonic_peaks(P, 3, starts, ends, thr, Q=Q, capacity=1 << 22)
    nref = len(ref[0])
    stride = int(K.peak_region_stride)
    for cap, expect_overflow in ((8 * 4096 * 64, False), (8 * 256, True)):
        rec = torch.zeros((cap, 3), dtype=torch.int32, device=dev)
        cnt = torch.zeros(stride * 9, dtype=torch.int32, device=dev)
        K.harmonic_peaks_batch(P.data_ptr(), n, n, Kb, 3, starts, ends, thr, cap, rec.data_ptr(),
                               cnt.data_ptr() + 4 * stride, s, Q.data_ptr(), Q.shape[1], region_log2=3)
        K.peak_regions_total(cnt.data_ptr() + 4 * stride, 3, cap, cnt.data_ptr(), s)
        torch.cuda.synchronize()
        c = cnt.cpu().numpy().view(np.uint32)
        per = c[stride:stride * 9:stride]
        capr = cap // 8
        if expect_overflow:
            assert per.max() > capr and int(c[0]) == 8 * int(per.max()) > cap
            continue
        assert per.max() <= capr and int(c[0]) == int(per.sum())
        r = rec.cpu().numpy().view(np.uint32)
        got = []
        for g in range(8):
            reg = r[g * capr:g * capr + per[g]]
            i = 0
            while i < len(reg):  # the region is a sequence of whole chunks
                d = reg[i]
                assert d[0] & 0x80000000
                m = (d[0] >> 16) & 0x7F
                assert int(d[2]) == g * capr + i + 1  # absolute position of its first crossing
                body = reg[i + 1:i + 1 + m]
                assert np.all(body[:, 0] == (d[0] & 0xFFFF))
                got.extend(zip(body[:, 0].tolist(), body[:, 1].tolist(), body[:, 2].tolist()))
                i += 1 + m
        got.sort()
        seg = (ref[0] * 8 + ref[1]).cpu().numpy()
        exp = sorted(zip(seg.tolist(), ref[2].cpu().numpy().tolist(),
                         ref[3].cpu().numpy().view(np.uint32).tolist()))
        assert len(got) == nref and got == exp
