#!/usr/bin/env python3
"""Headline benchmark: DM x acceleration trials/s on 2^23-sample series with
an 8-harmonic sum (-n 3), one process per MI355X (torchrun for N > 1).

One step (per rank, weak scaling -- fixed work per GPU):
  * dedisperse this rank's DM shard (``--dms-per-gpu`` trials, default 8, one
    chunk -- the production pipeline dedisperses 32-DM chunks) from the
    resident 1024-channel 2-bit filterbank (Auto kernel choice: the LDS-staged
    byte-lane kernel with 8-DM workgroups -- the one-hot MFMA kernel computes
    whole 32-DM tiles, so an 8-DM chunk costs it twice as much; full tiles of
    low DMs go to MFMA),
  * whiten each trial and search +-500 m/s^2 (legacy acceleration-plan
    convention: ~684 trials per DM at 2^23 x 64 us) with an 8-harmonic sum,
    in 512-trial batches on one stream: fused resample + two-pass four-step
    FFT -> paired real-FFT post-processing + interbin/normalise -> LDS-staged
    harmonic sum + peak compaction -> peak clustering and per-trial
    harmonic distillation on the GPU -> per-DM acceleration distillation on
    host workers (overlapped with the next batches),
  * gather every rank's candidates to rank 0 over RCCL and run the global
    DM/harmonic distillation + scoring there -- on a worker thread, overlapped with
    the next step's dedispersion and search as the pipeline's DM blocks are
    (the timed region ends after the last step's merge; --serial-merge runs
    them back to back).
The synthetic filterbank (uniform 2-bit noise, random seed) is generated on
rank 0's GPU and RCCL-broadcast to the others outside the timed region.

Prints ONE JSON line on rank 0.  Reference number: BASELINE.md has no
published 2^23 figure; the N*log N extrapolation of the golden-run search
throughput (573 trials/s at 2^17 on 2x Tesla C2070) is ~6.6 trials/s, used
for vs_baseline.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

BASELINE_TRIALS_PER_S = 6.6  # 573 trials/s @2^17 scaled by N log N to 2^23 (2x C2070)


def parse():
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--log2n", type=int, default=23, help="FFT length = 2^log2n")
    p.add_argument("--nchans", type=int, default=1024)
    p.add_argument("--nbits", type=int, default=2)
    p.add_argument("--tsamp", type=float, default=64e-6)
    p.add_argument("--dms-per-gpu", type=int, default=8,
                   help="DM trials per GPU per step (dedispersed as one chunk, as the pipeline does)")
    p.add_argument("--acc", type=float, default=500.0, help="search +-acc m/s^2")
    p.add_argument("--nharmonics", type=int, default=3)
    p.add_argument("--accel-batch", type=int, default=0,
                   help="acceleration trials per batch (0 = auto: 512 at 2^23 within a 48 GiB budget, capped by free memory)")
    p.add_argument("--sub-batch", type=int, default=-1,
                   help="trials per sub-batch on two alternating streams (0 = off, -1 = auto: off from 2^22 samples, else half a batch, at most 2^28 samples)")
    p.add_argument("--fft-mode", type=int, default=2,
                   help="2: fused resample + four-step FFT; 1: rocFFT C2C(N/2) + fused r2c post; 0: rocFFT R2C")
    p.add_argument("--dedisp-kernel", default="auto", choices=["auto", "mfma", "valu", "direct", "packed2"])
    p.add_argument("--fft4-flags", type=int, default=-1, help="fused-FFT kernel variant flags (tuning; -1 = default)")
    p.add_argument("--harm-flags", type=int, default=-1,
                   help="harmonic-sum / tiled-r2c kernel variant flags (tuning; -1 = default)")
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--signal", "--peak-heavy", dest="signal", action="store_true",
                   help="peak-heavy data instead of pure noise: injected pulsars plus strong undispersed periodic "
                        "RFI (>= 1e4 threshold crossings per DM), to time the host clustering / distillation")
    p.add_argument("--serial-merge", action="store_true",
                   help="run each step's candidate gather + global distillation before the next step's "
                        "candidates are collected (default: on a worker thread, overlapped)")
    p.add_argument("--serial-steps", action="store_true",
                   help="each step a separate search() call (no overlap of a step's dedispersion and searches "
                        "with the previous step's collection; A/B of the step pipeline)")
    p.add_argument("--as-rank", default="",
                   help="N:r[,r...] -- on one GPU, time rank r's shard of a world-N run (the DM list of N ranks, "
                        "shard [r*dms, (r+1)*dms)), one JSON line per r: checks that every rank's step costs the same")
    p.add_argument("--rfi-amp", type=float, default=0.05,
                   help="--signal: amplitude of the two undispersed RFI pulse trains (the pulsars: 0.05-0.08)")
    return p.parse_args()


def main() -> int:
    a = parse()
    from peasoup_amd import _C
    from peasoup_amd.models.search import RankSearcher
    from peasoup_amd.parallel import dist as pdist

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus != world_env and world_env == 1 and a.gpus > 1:
        print("bench.py: for --gpus > 1 launch with torch.distributed.run (one rank per GPU)", file=sys.stderr)
        return 2
    ctx = pdist.init()
    dev = ctx.device
    as_world, as_ranks = 0, []
    if a.as_rank:
        w, _, rs_ = a.as_rank.partition(":")
        as_world, as_ranks = int(w), [int(x) for x in rs_.split(",") if x != ""]
        assert ctx.world_size == 1 and as_ranks and all(0 <= r < as_world for r in as_ranks), a.as_rank
    if a.fft4_flags >= 0:
        _C.kernels.fft4_set_flags(a.fft4_flags)
    if a.harm_flags >= 0:
        _C.kernels.harmonic_set_flags(a.harm_flags)
    assert dev.type == "cuda", "bench.py needs a GPU"

    n = 1 << a.log2n
    fch1, foff = 1550.0, -400.0 / a.nchans
    # DM list: enough trials for every rank's shard (Levin spacing, tol 1.1, 64 us)
    args = _C.CmdLineOptions()
    args.infilename = "synthetic"
    args.outdir = "/tmp/peasoup_bench"
    args.dm_start = 0.0
    need = a.dms_per_gpu * (as_world or ctx.world_size)
    dm_end = 5.0
    while True:
        dms = _C.generate_dm_list(0.0, dm_end, a.tsamp, 64.0, fch1, foff, a.nchans, 1.1)
        if len(dms) > need:
            break
        dm_end *= 1.5
    args.dm_end = dm_end
    args.acc_start, args.acc_end = -a.acc, a.acc
    args.nharmonics = a.nharmonics
    args.size = n
    args.accel_batch = a.accel_batch
    args.sub_batch = a.sub_batch
    args.fft_mode = a.fft_mode
    args.dedisp_kernel = a.dedisp_kernel
    delays = _C.generate_delay_table(a.nchans, a.tsamp, fch1, foff)
    max_delay = _C.compute_max_delay(dms, delays)
    nsamps = n + max_delay + 4096
    header = {"source_name": "synthetic noise", "tsamp": a.tsamp, "fch1": fch1, "foff": foff,
              "nchans": a.nchans, "nbits": a.nbits, "nifs": 1, "data_type": 1, "tstart": 60000.0,
              "nsamples": nsamps}
    nbytes = nsamps * a.nchans * a.nbits // 8

    # ---- synthetic filterbank on rank 0's GPU, RCCL broadcast to the others
    packed = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    if ctx.is_root and a.signal:
        from peasoup_amd.utils import synthetic

        # two binary pulsars in the searched DM range + periodic RFI at DM 0
        # (narrow 50 Hz and 16.7 Hz pulse trains: hundreds of harmonics above
        # threshold in every acceleration trial of every DM)
        sky = [synthetic.PulsarSpec(period=0.00731, dm=2.0, duty=0.05, amplitude=0.05, accel=120.0),
               synthetic.PulsarSpec(period=0.1532, dm=1.0, duty=0.04, amplitude=0.08, accel=-40.0),
               synthetic.PulsarSpec(period=0.02, dm=0.0, duty=0.02, amplitude=a.rfi_amp),
               synthetic.PulsarSpec(period=0.06, dm=0.0, duty=0.03, amplitude=0.67 * a.rfi_amp)]
        packed.copy_(synthetic.generate_packed_torch(nsamps, header, sky, seed=a.seed, device=dev))
    elif ctx.is_root:
        g = torch.Generator(device=dev)
        g.manual_seed(a.seed)
        packed.random_(0, 256, generator=g)  # every 2-bit field uniform on {0..3}
    pdist.broadcast_bytes(packed, nbytes)
    rs = RankSearcher(args, header, packed, nsamps)
    del packed
    torch.cuda.empty_cache()

    if as_world:
        return _as_rank(a, rs, args, as_world, as_ranks)
    shard = range(ctx.rank * a.dms_per_gpu, (ctx.rank + 1) * a.dms_per_gpu)
    trials_per_step_local = sum(len(rs.accel_list(rs.dm_list[d])) for d in shard)
    # exact job total: the plan's trial count shrinks slightly with DM (smearing term)
    tot = torch.tensor([trials_per_step_local], dtype=torch.int64, device=dev)
    trials_per_step = int(pdist.all_reduce_sum(tot).item())

    phase = {"search": 0.0, "merge": 0.0, "ser": 0.0, "wait": 0.0, "gather": 0.0, "gds": 0.0}
    # Steps are pipelined like the production run's DM blocks: step k's
    # candidate gather + global distillation (one worker thread, so the
    # gather collectives stay in order) overlaps step k+1's dedispersion and
    # search; the timed region ends after the last step's merge.
    from concurrent.futures import ThreadPoolExecutor

    # (the worker binds the rank's GPU first: its collectives and any torch
    # call must not create a context on device 0)
    merger = (ThreadPoolExecutor(max_workers=1, initializer=torch.cuda.set_device, initargs=(dev,))
              if not a.serial_merge else None)

    def merge(local):
        # as run_search: one rank's list merged in place; more: every rank's
        # serialised list gathered to rank 0 only (RCCL), merged there
        t1 = time.perf_counter()
        if not ctx.distributed:
            t2 = t3 = t1
            phase["blob_bytes"] = 0
            out = _C.merge_local(local, args, rs.header)
        else:
            blob = torch.from_numpy(_C.serialize_candidates_array(local))
            t2 = time.perf_counter()
            tm = {}
            bufs = pdist.gather_buffers(blob, dst=0, timing=tm)
            t3 = time.perf_counter()
            # the size exchange is where a rank waits for the slowest peer to
            # reach this step's merge (rank skew, not merge work)
            phase["wait"] += tm.get("sizes_done", t2) - t2
            phase["blob_bytes"] = blob.numel()
            out = (_C.merge_candidate_buffers([(b.data_ptr(), b.numel()) for b in bufs], args, rs.header)
                   if ctx.is_root else _C.CandidateBag())
        t4 = time.perf_counter()
        phase["merge"] += t4 - t1
        phase["ser"] += t2 - t1
        phase["gather"] += t3 - t2
        phase["gds"] += t4 - t3
        return out

    # a step: the shard's DM blocks dedispersed + searched, its candidates
    # merged.  Steps run back to back through the search pipeline, as a
    # rank's DM chunks do in a run: step k+1's dedispersion and searches are
    # in flight while step k's candidates are collected and handed to the
    # merge (no idle GPU between steps).  Every step of a run_steps() call is
    # issued and finished inside it.
    tile = int(_C.Dedisperser.tile_dms)
    step_blocks = rs.chunk_ranges(shard, max(tile, (a.dms_per_gpu + tile - 1) // tile * tile))

    def run_steps(nsteps):
        out, acc, got = [], _C.CandidateBag(), 0
        t = time.perf_counter()
        if a.serial_steps:
            for _ in range(nsteps):
                local = rs.search(blocks=step_blocks)
                phase["search"] += time.perf_counter() - t
                out.append(merger.submit(merge, local) if merger else merge(local))
                t = time.perf_counter()
            return out
        for _, bag in rs.search_iter(blocks=step_blocks * nsteps):
            acc.extend(bag)
            got += 1
            if got % len(step_blocks) == 0:
                phase["search"] += time.perf_counter() - t
                out.append(merger.submit(merge, acc) if merger else merge(acc))
                acc = _C.CandidateBag()
                t = time.perf_counter()
        return out

    def finish(r):
        return r.result() if merger else r

    for r in run_steps(a.warmup):
        finish(r)
    for e in rs.engines:
        e.reset_counters()
    phase.update(search=0.0, merge=0.0, ser=0.0, wait=0.0, gather=0.0, gds=0.0)
    pdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pending = run_steps(a.steps)
    ncands = len(finish(pending[-1]))
    for r in pending:
        finish(r)
    torch.cuda.synchronize()
    pdist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = pdist.all_reduce_max_float(elapsed)
    ms_per_step = 1e3 * elapsed / a.steps
    value = trials_per_step * a.steps / elapsed
    ctr = rs.counters()  # timed steps only: peaks compacted on the GPU, host clustering + distillation time
    if ctx.is_root:
        out = {
            "metric": "DM×accel trials/sec, 2^23-sample series, 8-harmonic sum",
            "value": round(value, 2),
            "unit": "trials/s",
            "n_gpus": ctx.world_size,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            # BASELINE.json publishes no number for this metric: no ratio is
            # claimed; the N log N extrapolation of the 2^17 golden run is
            # reported separately, labelled as such
            "vs_baseline": None,
            "vs_extrapolated_reference": round(value / BASELINE_TRIALS_PER_S, 2),
            "baseline_note": "no published reference number; 6.6 trials/s = the 2^17 golden run (2x C2070, "
                             "573 trials/s) scaled by N log N to 2^23 -- orientation only",
            "dtype": "fp32",
            "data": ("synthetic (2-bit Gaussian noise + 2 binary pulsars + periodic DM-0 RFI, random seed)" if a.signal
                     else "synthetic (uniform 2-bit noise filterbank, random seed)"),
            "config": {
                "model": f"peasoup accel search: 2^{a.log2n}-pt series, +-{a.acc:g} m/s^2 (legacy plan), "
                         f"{1 << a.nharmonics}-harmonic sum, {a.nchans}-ch {a.nbits}-bit filterbank, "
                         f"{a.dedisp_kernel} dedispersion kernel",
                "global_batch": trials_per_step,
                "seq_len": n,
                "parallelism": f"dm{ctx.world_size}",
                "dms_per_gpu": a.dms_per_gpu,
                "accel_trials_per_dm": trials_per_step_local // a.dms_per_gpu,
                "accel_batch": rs.engine.batch_size,
                # the batch the last launch used (short lists are cut into min_batches even batches)
                "accel_batch_used": rs.engine.last_batch,
                "sub_batch": rs.engine.sub_batch,
                "fft_mode": rs.engine.fft_mode,
                "candidates_after_distill": ncands,
                "signal": bool(a.signal),
                "peaks_per_dm": round(ctr.get("peaks", 0) / max(1, a.steps * a.dms_per_gpu), 1),
                "host_distill_s_per_step": round(ctr.get("host_s", 0) / a.steps, 4),
                # rank 0's wall split of a step: dedispersion + whitening + the
                # acceleration loop, then the candidate gather + global distillation
                "search_s_per_step": round(phase["search"] / a.steps, 4),
                "merge_s_per_step": round(phase["merge"] / a.steps, 4),
                # the merge without the wait for the slowest rank at its first collective
                "merge_work_s_per_step": round((phase["merge"] - phase["wait"]) / a.steps, 4),
                "merge_overlapped": not a.serial_merge,
                "steps_pipelined": not a.serial_steps,
                "merge_split_s": {k: round(phase[k] / a.steps, 4) for k in ("ser", "wait", "gather", "gds")},
                "candidate_blob_bytes": phase.get("blob_bytes", 0),
                "accel_s_per_step": round(ctr.get("accel_s", 0) / a.steps, 4),
                "accel_distill_s_per_step": round(ctr.get("accd_s", 0) / a.steps, 4),
                "tail_s_per_step": round(ctr.get("tail_s", 0) / a.steps, 4),
                "trials_distilled_on_gpu": int(ctr.get("gpu_distilled", 0)),
                "trials_distilled_on_host": int(ctr.get("host_distilled", 0)),
            },
        }
        print(json.dumps(out), flush=True)
    pdist.shutdown()
    return 0


def _as_rank(a, rs, args, world, ranks) -> int:
    """Time, on this one GPU, the step of each given rank of a world-N run:
    its shard's dedispersion + search + the candidate merge (a world of one)."""
    from peasoup_amd import _C
    from peasoup_amd.parallel import dist as pdist

    for r in ranks:
        shard = range(r * a.dms_per_gpu, (r + 1) * a.dms_per_gpu)
        trials = sum(len(rs.accel_list(rs.dm_list[d])) for d in shard)

        def step():
            local = rs.search(shard, chunk=a.dms_per_gpu)
            local.sort_by_dm()
            return _C.global_distill_and_score(local, args, rs.header)

        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(json.dumps({"as_rank": r, "world": world, "dms": [shard.start, shard.stop],
                          "dm_range": [round(rs.dm_list[shard.start], 3), round(rs.dm_list[shard.stop - 1], 3)],
                          "trials_per_step": trials, "ms_per_step": round(1e3 * el / a.steps, 3),
                          "trials_per_s": round(trials * a.steps / el, 2),
                          "dedisp_kernel": a.dedisp_kernel, "signal": bool(a.signal)}), flush=True)
    pdist.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
