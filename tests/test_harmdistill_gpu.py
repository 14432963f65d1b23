"""Per-trial harmonic distillation on the device (kern::harm_distill_batch,
csrc/kernels/harmdistill.hip) against the host HarmonicDistiller
(include/transforms/distiller.hpp:63-108 semantics, csrc/src/candidates.cpp),
and the search engine with device distillation against host distillation."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"
RAW = 0x80000000
HOST = 0x80000000


def _trial(rng, n, nlev, df, ties=False):
    """n cluster peaks over levels 0..nlev: a few fundamentals with many
    (fractional) harmonics at every level -- the relation matters -- plus
    unrelated bins; per level ascending idx (the cluster kernel's order)."""
    per = np.full(nlev + 1, n // (nlev + 1))
    per[: n - per.sum()] += 1
    levels = []
    funds = rng.uniform(0.5, 60.0, 4)
    for h, m in enumerate(per):
        fac = df / 2 ** h
        idx = set()
        while len(idx) < m:
            if rng.random() < 0.6:
                f0 = funds[rng.integers(len(funds))]
                f = f0 * rng.integers(1, 17) / rng.integers(1, 2 ** h + 1)
                f *= 1.0 + rng.normal(0, 3e-5)  # inside/outside the 1e-4 tolerance
            else:
                f = rng.uniform(0.2, 900.0)
            b = int(round(f / fac))
            if 0 < b < (1 << 28):
                idx.add(b)
        idx = np.array(sorted(idx), np.int32)
        snr = (9.0 + 80.0 * rng.random(m)).astype(np.float32)
        if ties and m > 3:
            snr[2] = snr[0]
        levels.append((idx, snr))
    return levels


def test_harm_distill_matches_host(C):
    K = C.kernels
    rng = np.random.default_rng(11)
    nlev = 3
    df = 1.0 / ((1 << 20) * 64e-6)
    factor = [df / 2 ** h for h in range(6)]
    tol, max_harm = 1e-4, 16.0
    cap = int(K.harm_cap)
    sizes = [0, 1, 5, 64, 65, 200, 1024, 1025, 3000, cap, cap + 1, 300, 700, 2, 0, 129]
    raw_trial, tie_trial = 11, 12
    trials = []
    clust, segtab = [], np.zeros((len(sizes), 8, 2), np.uint32)
    off = 0
    for k, n in enumerate(sizes):
        lv = _trial(rng, n, nlev, df, ties=(k == tie_trial))
        trials.append(lv)
        for h, (idx, snr) in enumerate(lv):
            m = len(idx)
            segtab[k, h] = (off, m | (RAW if (k == raw_trial and h == 1) else 0))
            clust.append(np.stack([idx.view(np.uint32), snr.view(np.uint32)], axis=1))
            off += m
    clust = np.concatenate(clust) if off else np.zeros((1, 2), np.uint32)
    nt = len(sizes)
    d_clust = torch.from_numpy(clust.reshape(-1).view(np.int32).copy()).to(dev)
    d_seg = torch.from_numpy(segtab.reshape(-1).view(np.int32).copy()).to(dev)
    d_out = torch.zeros(2 * max(1, off), dtype=torch.int32, device=dev)
    d_ttab = torch.zeros(2 * nt, dtype=torch.int32, device=dev)
    d_tot = torch.zeros(1, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    K.harm_distill_batch(d_clust.data_ptr(), d_seg.data_ptr(), nt, nlev, factor, tol, max_harm, d_out.data_ptr(),
                         d_ttab.data_ptr(), d_tot.data_ptr(), s)
    torch.cuda.synchronize()
    ttab = d_ttab.cpu().numpy().view(np.uint32).reshape(nt, 2)
    out = d_out.cpu().numpy().view(np.uint32).reshape(-1, 2)
    hd = C.HarmonicDistiller(tol, max_harm, False, True)
    total = ndev = 0
    for k, n in enumerate(sizes):
        first, cnt = int(ttab[k, 0]), int(ttab[k, 1])
        allsnr = np.concatenate([snr for _, snr in trials[k]]) if n else np.zeros(0, np.float32)
        tie = len(np.unique(allsnr)) < len(allsnr)
        if k in (raw_trial, tie_trial) or n > cap or tie:
            assert cnt == HOST, (k, hex(cnt))
            continue
        assert not cnt & HOST, (k, n)
        ndev += 1
        cands = []
        for h, (idx, snr) in enumerate(trials[k]):
            for i, v in zip(idx, snr):
                cands.append(C.Candidate(10.0, 3, 0.0, h, float(v), float(np.float32(int(i) * factor[h]))))
        exp = [(c.nh, c.snr, c.freq) for c in hd.distill(cands)]
        got = []
        for x, y in out[first:first + cnt]:
            h = int(x >> 29)
            i = int(x & ((1 << 29) - 1))
            got.append((h, float(np.uint32(y).view(np.float32)), float(np.float32(i * factor[h]))))
        assert cnt == len(exp), (k, n, cnt, len(exp))
        assert got == exp, k
        if n >= 64:
            assert len(exp) < n  # the relation removed candidates
        total += cnt
    assert int(d_tot.item()) == total
    assert ndev >= 10, ndev  # most trials distilled on the device


def _search(C, trial, nsamps, accs, cluster, distill):
    os.environ["PSOUP_GPU_CLUSTER"] = "1" if cluster else "0"
    os.environ["PSOUP_GPU_DISTILL"] = "1" if distill else "0"
    try:
        p = C.SearchParams()
        p.fft_size, p.tsamp, p.nharmonics = 1 << 20, 64e-6, 4
        eng = C.SearchEngine(p, torch.cuda.current_stream().cuda_stream)
        c = eng.search_trial(trial.data_ptr(), nsamps, 10.0, 3, accs)
        ctr = eng.counters()
    finally:
        os.environ.pop("PSOUP_GPU_CLUSTER", None)
        os.environ.pop("PSOUP_GPU_DISTILL", None)
    return [(x.dm_idx, x.acc, x.nh, x.snr, x.freq, x.count_assoc()) for x in c], ctr


def test_engine_gpu_distill_equals_host(C):
    """Peak-heavy trial: device clustering + device harmonic distillation give
    the acceleration-distilled list of the all-host reference path."""
    rng = np.random.default_rng(7)
    n = (1 << 20) + 512
    t = np.arange(n) * 64e-6
    x = rng.normal(128, 6, n)
    for per, amp in ((0.00731, 30.0), (0.02, 60.0), (0.0613, 25.0)):
        ph = (t / per) % 1.0
        x += amp * (np.minimum(ph, 1 - ph) < 0.015)
    trial = torch.from_numpy(np.clip(np.rint(x), 0, 255).astype(np.uint8)).to(dev)
    accs = [float(a) for a in np.linspace(-60, 60, 41)]
    host, ch = _search(C, trial, n, accs, False, False)
    hdist, chd = _search(C, trial, n, accs, True, False)
    gpu, cg = _search(C, trial, n, accs, True, True)
    assert ch["peaks"] > 100000, ch
    assert cg["gpu_distilled"] > 0.9 * len(accs), cg
    assert chd["gpu_distilled"] == 0
    assert len(gpu) == len(host) and len(gpu) > 0
    assert hdist == host
    assert gpu == host
