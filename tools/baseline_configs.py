#!/usr/bin/env python3
"""Runs the five configurations named in BASELINE.json and prints one JSON
line per configuration (--out FILE also appends them there).

  1  tutorial.fil load + header parse -> empty overview.xml (CPU plumbing)
  2  zero-acceleration periodicity search: 1 DM, 2^22-sample series
  3  acceleration search: 1 DM, 2^23 samples, +-500 m/s^2, 8 harmonics
  4  1024-channel synthetic filterbank, 2000 DM trials dedispersed +
     acceleration-searched (one process per GPU; run under torchrun for 8 GPUs)
  5  full pipeline: config 4 + fold the top 128 candidates + multi-beam
     coincidence counts all-reduced over RCCL (one beam per rank)

Synthetic data only (no network): quantised Gaussian noise with an injected
dispersed pulsar, generated on the GPU.  Configs 4/5 default to a 2^20-sample
(67 s) observation so the file stays ~270 MB; --log2n 23 gives the headline
series length (2 GB filterbank).

    python tools/baseline_configs.py --configs 1,2,3,4,5 [--ndm 2000] [--log2n 20]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/baseline_configs.py --configs 4,5
    python tools/baseline_configs.py --configs 4 --as-rank 8:0,3,7   # ranks of an 8-GPU run, one at a time
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, REPO)

from peasoup_amd import _C  # noqa: E402
from peasoup_amd.parallel import dist as pdist  # noqa: E402
from peasoup_amd.utils.sigproc import header_bytes  # noqa: E402

TUTORIAL = os.path.join(REPO, "tests", "data", "tutorial.fil")
FCH1, FOFF, TSAMP = 1550.0, -400.0 / 1024, 64e-6


def gpu_filterbank(path: str, nsamps: int, nchans: int, tsamp: float, fch1: float, foff: float,
                   period: float, dm: float, duty: float, amp: float, seed: int, chunk: int = 1 << 15):
    """2-bit filterbank with a dispersed pulsar, generated chunk-wise on the GPU."""
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    freqs = fch1 + foff * torch.arange(nchans, device=dev, dtype=torch.float64)
    delay = 4.15e3 * dm * (1.0 / freqs ** 2 - 1.0 / fch1 ** 2)
    hdr = {"source_name": f"synthetic P={period} DM={dm}", "tsamp": tsamp, "fch1": fch1, "foff": foff,
           "nchans": nchans, "nbits": 2, "nifs": 1, "data_type": 1, "tstart": 60000.0, "nsamples": nsamps}
    w = duty / 2.3548
    with open(path, "wb") as f:
        f.write(header_bytes(hdr))
        for t0 in range(0, nsamps, chunk):
            n = min(chunk, nsamps - t0)
            t = (torch.arange(t0, t0 + n, device=dev, dtype=torch.float64) * tsamp)[:, None] - delay[None, :]
            ph = torch.remainder(t / period, 1.0)
            d = torch.minimum(ph, 1.0 - ph)
            x = torch.randn((n, nchans), device=dev, generator=g) + amp * torch.exp(-0.5 * (d / w) ** 2).float()
            q = torch.clamp(torch.round(1.5 + 0.75 * x), 0, 3).to(torch.uint8).view(n, nchans // 4, 4)
            packed = q[..., 0] | (q[..., 1] << 2) | (q[..., 2] << 4) | (q[..., 3] << 6)
            f.write(packed.cpu().numpy().tobytes())
    return hdr


def emit(rec, out):
    line = json.dumps(rec)
    print(line, flush=True)
    if out:
        with open(out, "a") as f:
            f.write(line + "\n")


def config1(a):
    t0 = time.perf_counter()
    fb = _C.Filterbank.from_file(TUTORIAL)
    hdr = fb.header
    ok, _, args = _C.parse_cmdline(["peasoup", "-i", TUTORIAL, "--dm_end", "250", "--acc_start", "-5",
                                    "--acc_end", "5", "-n", "4"])
    d = tempfile.mkdtemp()
    path = os.path.join(d, "overview.xml")
    _C.write_overview(path, args, TUTORIAL, [], [], [], [], {}, {"reading": time.perf_counter() - t0}, {})
    return {"config": 1, "desc": "tutorial.fil load + header parse -> empty overview.xml",
            "ok": bool(ok and os.path.getsize(path) > 0), "nchans": hdr["nchans"], "nsamples": hdr["nsamples"],
            "tsamp": hdr["tsamp"], "seconds": round(time.perf_counter() - t0, 4)}


def _series(n, tsamp, period, amp, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(n) * tsamp
    ph = (t / period) % 1.0
    x = rng.normal(128, 8, n) + amp * (np.minimum(ph, 1 - ph) < 0.02)
    return torch.from_numpy(np.clip(np.rint(x), 0, 255).astype(np.uint8)).cuda()


def _engine_run(log2n, accs, nharm, reps=3):
    n = 1 << log2n
    nsamps = n + 1000
    trial = _series(nsamps, TSAMP, 0.0123456, 3.0, 1)
    p = _C.SearchParams()
    p.fft_size, p.tsamp, p.nharmonics = n, TSAMP, nharm
    s = torch.cuda.current_stream().cuda_stream
    eng = _C.SearchEngine(p, s)
    eng.search_trial(trial.data_ptr(), nsamps, 0.0, 0, accs)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        c = eng.search_trial(trial.data_ptr(), nsamps, 0.0, 0, accs)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    best = max(c, key=lambda x: x.snr) if c else None
    return dt, best, eng


def config2(a):
    dt, best, eng = _engine_run(22, [0.0], 3)
    return {"config": 2, "desc": "zero-accel search, 1 DM, 2^22 samples (whiten + FFT + harmonic sum + peaks)",
            "ms_per_dm": round(1e3 * dt, 3), "fft_mode": eng.fft_mode,
            "best_period_s": (1.0 / best.freq) if best else None, "best_snr": best.snr if best else None}


def config3(a):
    n = 1 << 23
    plan = _C.AccelPlan(-500.0, 500.0, 1.1, 64.0, n, TSAMP, FCH1 + FOFF * 512, FOFF, _C.AccelConvention.Legacy)
    accs = list(plan.generate(0.0))
    dt, best, eng = _engine_run(23, accs, 3, reps=2)
    return {"config": 3, "desc": "accel search, 1 DM, 2^23 samples, +-500 m/s^2, 8 harmonics",
            "accel_trials": len(accs), "ms_per_dm": round(1e3 * dt, 3), "trials_per_s": round(len(accs) / dt, 1),
            "best_period_s": (1.0 / best.freq) if best else None, "best_snr": best.snr if best else None}


def config3_pipeline(a, as_rank=None):
    """Config 3 through the distributed driver (run_search): a 64-channel
    2-bit filterbank with one accelerated pulsar, searched at one DM, 2^23
    points, +-500 m/s^2, 8 harmonics.  Under torchrun (or --as-rank W:r) the
    DM's 685 acceleration trials are cut into slices the ranks share
    (search.accel_slices); one rank searches them all."""
    from peasoup_amd.models.search import run_search

    ctx = pdist.init()
    n = 1 << 23
    path = os.path.join(a.workdir, "cfg3_1dm.fil")
    if ctx.is_root and not os.path.exists(path):
        gpu_filterbank(path, n + 8192, 64, TSAMP, FCH1, -6.25, period=0.0123456, dm=50.0, duty=0.05, amp=0.3,
                       seed=3)
    pdist.barrier()
    out = os.path.join(a.workdir, "out_cfg3" + (f"_as{as_rank[0]}_{as_rank[1]}" if as_rank else ""))
    argv = ["peasoup", "-i", path, "-o", out, "--dm_start", "50", "--dm_end", "50", "--acc_start", "-500",
            "--acc_end", "500", "-n", "3", "--npdmp", "0", "--limit", "1000"]
    ok, _, args = _C.parse_cmdline(argv)
    assert ok
    t0 = time.perf_counter()
    res = run_search(args, as_rank=as_rank)
    wall = time.perf_counter() - t0
    if not ctx.is_root:
        return None
    st = res.rank_stats[0] if res.rank_stats else {}
    rec = {"config": 3, "driver": "run_search", "log2n": 23, "wall_s": round(wall, 3),
           "accel_trials": res.accel_trials, "accel_slices": st.get("accel_slices"),
           "search_s": round(st.get("search_s", 0.0), 4),
           "timers_s": {k: round(v, 4) for k, v in res.timers.items()}, "candidates": len(res.candidates)}
    if as_rank is not None:
        rec.update({"as_rank": as_rank[1], "world": as_rank[0],
                    "rank_stats": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in st.items()
                                   if isinstance(v, (int, float))},
                    "desc": f"rank {as_rank[1]} of a {as_rank[0]}-rank config-3 run (its acceleration slices)"})
    else:
        rec.update({"ranks": ctx.world_size, "desc": "1 DM, 2^23 samples, +-500 m/s^2, 8 harmonics, run_search",
                    "trials_per_s": round(res.accel_trials / st["search_s"], 1) if st.get("search_s") else None})
        if res.candidates:
            b = res.candidates[0]
            rec["best"] = {"period_s": 1.0 / b.freq, "acc": b.acc, "snr": b.snr}
    return rec


def config5_pulsars(n: int = 64, seed: int = 5):
    """The config-5 sky: n pulsars with incommensurate periods (2 ms - 1 s,
    log-uniform), DMs over the searched range, accelerations within +-100
    m/s^2 and 3-12% duty cycles, bright enough that each survives the
    harmonic / acceleration / DM distillation as its own candidate family:
    >= 128 candidates to fold (verdict r2: the single-pulsar file gave 22)."""
    from peasoup_amd.utils import synthetic

    rng = np.random.default_rng(seed)
    periods = np.exp(rng.uniform(np.log(0.002), np.log(1.0), n))
    return [synthetic.PulsarSpec(period=float(p), dm=float(rng.uniform(20.0, 1100.0)),
                                 duty=float(rng.uniform(0.03, 0.12)), amplitude=float(rng.uniform(0.06, 0.12)),
                                 accel=float(rng.uniform(-100.0, 100.0)), phase=float(rng.random()))
            for p in periods]


def _make_fb(a, ctx):
    path = os.path.join(a.workdir, f"cfg45_{a.log2n}_{a.sky}.fil")
    if ctx.is_root and not os.path.exists(path) and a.sky == "single":
        # round-2 config-4 data: one dispersed 37.1 ms pulsar at DM 110 in noise
        gpu_filterbank(path, (1 << a.log2n) + 65536, 1024, TSAMP, FCH1, FOFF, period=0.0371, dm=110.0, duty=0.05,
                       amp=0.25, seed=11)
    elif ctx.is_root and not os.path.exists(path):
        from peasoup_amd.utils import synthetic
        from peasoup_amd.utils.sigproc import header_bytes as _hb

        nsamps = (1 << a.log2n) + 65536
        hdr = {"source_name": "synthetic: 64 pulsars (tools/baseline_configs.config5_pulsars)", "tsamp": TSAMP,
               "fch1": FCH1, "foff": FOFF, "nchans": 1024, "nbits": 2, "nifs": 1, "data_type": 1,
               "tstart": 60000.0, "nsamples": nsamps}
        packed = synthetic.generate_packed_torch(nsamps, hdr, config5_pulsars(), seed=7)
        with open(path, "wb") as f:
            f.write(_hb(hdr))
            f.write(packed.cpu().numpy().tobytes())
        del packed
    pdist.barrier()
    return path


def _dm_end_for(ndm):
    dm_end = 10.0
    while len(_C.generate_dm_list(0.0, dm_end, TSAMP, 64.0, FCH1, FOFF, 1024, 1.1)) < ndm:
        dm_end *= 1.05
    return dm_end


def config45(a, npdmp, cfg, as_rank=None):
    from peasoup_amd.models.search import run_search

    ctx = pdist.init()
    path = _make_fb(a, ctx)
    out = os.path.join(a.workdir, f"out_cfg{cfg}" + (f"_as{as_rank[0]}_{as_rank[1]}" if as_rank else ""))
    argv = ["peasoup", "-i", path, "-o", out, "--dm_end", f"{_dm_end_for(a.ndm):.3f}", "--acc_start", "-500",
            "--acc_end", "500", "-n", "3", "--npdmp", str(npdmp), "--limit", "1000"]
    ok, _, args = _C.parse_cmdline(argv)
    assert ok
    if a.native:
        # the native C++ pipeline (bin/peasoup, one host thread per GPU + engines)
        import subprocess

        trace = os.path.join(a.workdir, f"trace_cfg{cfg}.json")
        t0 = time.perf_counter()
        r = subprocess.run([os.path.join(REPO, "bin", "peasoup")] + argv[1:] + ["--trace_json", trace],
                           capture_output=True, text=True)
        wall = time.perf_counter() - t0
        assert r.returncode == 0, r.stderr[-2000:]
        tr = json.load(open(trace))
        return {"config": cfg, "desc": "native bin/peasoup, same data and options", "log2n": a.log2n,
                "wall_s": round(wall, 3), "timers_s": {k: round(v, 3) for k, v in tr.get("timers_s", {}).items()},
                "performance": tr.get("performance", {}), "argv": argv[1:]}
    t0 = time.perf_counter()
    res = run_search(args, as_rank=as_rank)
    wall = time.perf_counter() - t0
    rec = None
    if as_rank is not None:
        st = res.rank_stats[0] if res.rank_stats else {}
        return {"config": cfg, "as_rank": as_rank[1], "world": as_rank[0], "log2n": a.log2n,
                "desc": f"rank {as_rank[1]} of a {as_rank[0]}-rank config-{cfg} run (static DM shard), on one GPU",
                "dm_trials": st.get("dm_trials"), "accel_trials": res.accel_trials, "wall_s": round(wall, 3),
                "timers_s": {k: round(v, 3) for k, v in res.timers.items()},
                "total_minus_search_s": round(res.timers["total"] - st.get("search_s", 0.0), 3),
                "search_s": round(st.get("search_s", 0.0), 3), "device_init_s": round(st.get("device_init_s", 0.0), 4),
                "candidates": len(res.candidates)}
    if ctx.is_root:
        best = res.candidates[0] if res.candidates else None
        rec = {"config": cfg,
               "desc": f"1024-ch synthetic, {len(res.dm_list)} DM trials dedispersed + accel-searched"
                       + (f", fold top-{npdmp}" if npdmp else ""),
               "log2n": a.log2n, "ranks": ctx.world_size, "dm_trials": len(res.dm_list),
               "accel_trials": res.accel_trials, "wall_s": round(wall, 3),
               "timers_s": {k: round(v, 3) for k, v in res.timers.items()},
               "dm_accel_trials_per_s": round(res.performance["dm_accel_trials_per_sec"], 1),
               "candidates": len(res.candidates),
               "folded": sum(1 for c in res.candidates if c.folded_snr != 0.0),
               "rank_stats": res.rank_stats,
               "fold_stats": res.fold_stats,
               "best": {"period_s": 1.0 / best.freq, "dm": best.dm, "acc": best.acc, "snr": best.snr,
                        "folded_snr": best.folded_snr} if best else None}
    if cfg == 5:
        from peasoup_amd.models.coincidencer import run_coincidencer

        t1 = time.perf_counter()
        mask_out = os.path.join(a.workdir, "cfg5_samp_mask.txt")
        bird_out = os.path.join(a.workdir, "cfg5_birdies.txt")
        info = run_coincidencer([path] * ctx.world_size, mask_out, bird_out, beam_thresh=max(1, ctx.world_size))
        if ctx.is_root:
            rec["coincidencer_s"] = round(time.perf_counter() - t1, 3)
            rec["coincidencer"] = info
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1,2,3,4,5")
    ap.add_argument("--ndm", type=int, default=2000)
    ap.add_argument("--log2n", type=int, default=20)
    ap.add_argument("--workdir", default=os.path.join(REPO, "gpurun_out", "configs"))
    ap.add_argument("--sky", default="multi", choices=["multi", "single"],
                    help="configs 4/5 data: the 64-pulsar sky (default) or one pulsar in noise (the round-2 data)")
    ap.add_argument("--out", default="")
    ap.add_argument("--native", action="store_true", help="configs 4/5 through bin/peasoup instead of Python")
    ap.add_argument("--as-rank", default="", metavar="W:r[,r...]",
                    help="configs 4/5: time ranks r of a W-rank run one after another on this GPU (setup included; "
                         "an untimed run of the first rank warms the process)")
    a = ap.parse_args()
    os.makedirs(a.workdir, exist_ok=True)
    ctx = pdist.init()
    for c in [int(x) for x in a.configs.split(",")]:
        if c == 3 and a.as_rank:
            w, _, rs_ = a.as_rank.partition(":")
            ranks = [int(x) for x in rs_.split(",") if x != ""]
            assert ctx.world_size == 1 and ranks, a.as_rank
            emit(dict(config3_pipeline(a), warmup=True), a.out)  # (and the one-rank reference)
            emit(config3_pipeline(a), a.out)
            for r in ranks:
                emit(config3_pipeline(a, (int(w), r)), a.out)
        elif c == 3:
            if ctx.is_root:
                emit(config3(a), a.out)  # the engine alone
            rec = config3_pipeline(a)  # the driver (all ranks under torchrun)
            if rec is not None:
                emit(rec, a.out)
        elif c in (1, 2):
            if ctx.is_root:
                emit({1: config1, 2: config2}[c](a), a.out)
        elif c in (4, 5) and a.as_rank:
            w, _, rs_ = a.as_rank.partition(":")
            ranks = [int(x) for x in rs_.split(",") if x != ""]
            assert ctx.world_size == 1 and ranks, a.as_rank
            first = config45(a, 0 if c == 4 else 128, c, (int(w), ranks[0]))
            emit(dict(first, warmup=True), a.out)
            for r in ranks:
                emit(config45(a, 0 if c == 4 else 128, c, (int(w), r)), a.out)
        elif c in (4, 5):
            rec = config45(a, 0 if c == 4 else 128, c)
            if rec is not None:
                emit(rec, a.out)
    pdist.shutdown()


if __name__ == "__main__":
    main()
