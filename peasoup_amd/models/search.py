"""Distributed peasoup search: one process per GPU, RCCL collectives.

Flow per rank (SURVEY.md §7.1 distribution model):

1. rank 0 reads the ``.fil`` (mmap) and copies the packed bytes to its GPU;
   an RCCL broadcast over xGMI replicates them (``broadcast_bytes``), and
   every rank unpacks them into a channel-major int8 filterbank resident in
   HBM (``DeviceFilterbank``).
2. ranks take 32-DM chunks first-come from a queue they share
   (``--dm_schedule dynamic``, the default for several ranks and at least 4
   chunks per rank: the reference's
   DMDispenser, made cross-process with an atomic counter in the process
   group's key-value store, ``pdist.WorkQueue``), or each owns a contiguous
   DM shard balanced by acceleration-trial count (``static``,
   ``shard_range``); a rank dedisperses its chunks straight into HBM and runs
   the native ``SearchEngine`` (whitening + batched acceleration search) on
   each trial.  Any rank can take any chunk: every rank holds the whole
   filterbank.
3. per-rank candidate trees are serialised and gathered to rank 0 over RCCL
   (``gather_bytes``); rank 0 runs the global DM / harmonic distillation and
   scoring.
4. fold jobs are grouped by DM and spread round-robin over the ranks (each
   holds the whole filterbank, so any rank can re-dedisperse any DM); results
   are gathered to rank 0, which writes ``candidates.peasoup`` and
   ``overview.xml``.

Reference: src/pipeline_multi.cu:100-419 (Worker, DMDispenser, main) and
include/transforms/folder.hpp:337-442 (MultiFolder).
"""
from __future__ import annotations

import concurrent.futures
import json
import os
import struct
import threading
import time
import warnings
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import _C, dedisp_kernel
from ..parallel import dist as pdist
from ..utils.timing import Stopwatch, roctx_range


@dataclass
class SearchResult:
    candidates: list
    timers: Dict[str, float]
    performance: Dict[str, float]
    dm_list: List[float]
    acc_list0: List[float]
    devices: List[int]
    header: dict
    args: object = None
    accel_trials: int = 0
    rank_stats: list = field(default_factory=list)
    fold_stats: dict = field(default_factory=dict)


_BLOCK_TRACE = os.environ.get("PSOUP_BLOCK_TRACE", "")  # diagnostics: per-block host timeline (JSON lines)


_ENGINE_STREAMS: Dict[tuple, object] = {}  # (device index, slot) -> _C.GpuStream, alive for the process


def _engine_stream(device: torch.device, slot: int = 0) -> int:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if (idx, slot) not in _ENGINE_STREAMS:
        with torch.cuda.device(idx):
            _ENGINE_STREAMS[(idx, slot)] = _C.GpuStream()
    return _ENGINE_STREAMS[(idx, slot)].handle


def engines_per_gpu(args, max_trials_per_dm: int) -> int:
    """Search engines per GPU (each on its own stream, fed by its own host
    thread): DM trials of a chunk are dealt round-robin so one engine's small
    per-DM kernels and host work overlap the others'.  Auto: 1.  Three
    engines paid off (1.6x on config 4) while per-trial distillation ran on
    the host; with clustering and harmonic distillation on the device and the
    acceleration distillation overlapped, one engine is faster (round 4,
    `profiles/r4_configs/engines.md`: config 4 search 0.42 vs 0.47 s, config 5
    0.41 vs 0.45 s, single pulsar equal).  ``--engines_per_gpu`` /
    ``PSOUP_ENGINES`` still select more."""
    v = int(os.environ.get("PSOUP_ENGINES", "0") or 0) or int(getattr(args, "engines_per_gpu", 0) or 0)
    return max(1, v)


class RankSearcher:
    """Per-rank search state: resident filterbank, dedisperser, engine."""

    def __init__(self, args, header: dict, packed: Optional[torch.Tensor], nsamps: int,
                 killmask: Optional[Sequence[int]] = None, fft_mode: Optional[int] = None, resident: bool = True,
                 warm: bool = True):
        """``resident=False``: no device filterbank / dedisperser (the
        time-sharded path hands DM trials over already dedispersed:
        :meth:`search_rows`, ``fold(..., rows=...)``).  ``warm=False``: the
        dedispersion plan tables wait for :meth:`warm` (a static shard's own)."""
        self.ctx = pdist.context()
        self.args = args
        self.header = dict(header)
        self.header["nsamples"] = int(nsamps)
        params, dm_list, kill, fft_size, cfreq = _C.search_params_from_args(args, self.header)
        # constructor overrides of the options: the checkpoint identity is
        # built from args, so spills are refused under an override (search())
        self._overrides = [n for n, v in (("killmask", killmask), ("fft_mode", fft_mode)) if v is not None]
        if killmask is not None:
            kill = list(killmask)
        if fft_mode is not None:
            params.fft_mode = int(fft_mode)
        self.params = params
        self.dm_list = list(dm_list)
        self.fft_size = int(fft_size)
        self.cfreq = cfreq
        self.geom = _C.DedispGeometry.make(self.header, int(nsamps), self.dm_list, list(kill))
        # the engine, dedisperser and folder share one explicit non-blocking
        # stream; torch work that produced `packed` is drained first
        self.stream = _engine_stream(self.ctx.device)
        torch.cuda.synchronize(self.ctx.device)
        self.dfb = self.dedisperser = None
        if resident:
            self.dfb = _C.DeviceFilterbank(self.geom, self.stream)
            if packed is not None:
                self.load_packed(packed)
            self.dedisperser = _C.Dedisperser(self.dfb, self.stream)
            if warm:
                self.warm()
        self.kernel = dedisp_kernel(args.dedisp_kernel)
        self.row_stride = _C.Dedisperser.row_stride(self.geom.out_nsamps)
        self.accel_plan = _C.accel_plan_from_args(args, self.header)
        max_trials = max((len(self.accel_list(d)) for d in self.dm_list), default=0)
        self.max_trials = max_trials
        neng = engines_per_gpu(args, max_trials)
        self.params.engines_per_device = neng  # the auto batch budget is shared among them
        self.engine = _C.SearchEngine(self.params, self.stream)
        self.engines = [self.engine] + [_C.SearchEngine(self.params, _engine_stream(self.ctx.device, i))
                                        for i in range(1, neng)]
        self._pool = None
        self._trials: Optional[torch.Tensor] = None
        self._fold_engine = None
        # keep_trials: every searched block's dedispersed rows stay in HBM
        # ({d0: (d1, rows)}) so the fold stage reads them instead of running the
        # dedispersion again (the reference keeps its DispersionTrials in host
        # memory for the folder, pipeline_multi.cu:372-386); run_search turns
        # it on when the rank's DMs fit in a quarter of the free HBM
        self.keep_trials = False
        self.resident_rows: Dict[int, tuple] = {}

    def load_packed(self, packed: torch.Tensor) -> None:
        if packed.is_cuda:
            self.dfb.load_packed_device(packed.data_ptr())
        else:
            self.dfb.load_packed_host(packed.data_ptr())

    def warm(self, d0: int = 0, d1: int = -1) -> None:
        """Dedispersion plan tables for DMs [d0, d1) (default: the whole
        list) at setup, not at the first tile that needs them."""
        if self.dedisperser is not None:
            self.dedisperser.warm(d0, d1)

    def accel_list(self, dm: float) -> List[float]:
        return self.accel_plan.generate(float(dm))

    def dedisperse(self, d0: int, d1: int) -> torch.Tensor:
        n = d1 - d0
        need = n * self.row_stride
        if self._trials is None or self._trials.numel() < need:
            self._trials = torch.empty(need, dtype=torch.uint8, device=self.ctx.device)
        self.dedisperser.run(d0, d1, self._trials.data_ptr(), self.row_stride, self.kernel)
        return self._trials

    @staticmethod
    def chunk_ranges(idx: Sequence[int], chunk: int) -> List[tuple]:
        """Contiguous [d0, d1) blocks of ``idx`` cut at multiples of ``chunk``
        (itself a multiple of the MFMA tile), so every block but a shard's
        first starts on a tile of the resident dedispersion plan."""
        idx = list(idx)
        if not idx:
            return []
        lo, hi = idx[0], idx[-1] + 1
        assert hi - lo == len(idx), "DM shard must be contiguous"
        out = []
        d0 = lo
        while d0 < hi:
            d1 = min(hi, (d0 // chunk + 1) * chunk)
            out.append((d0, d1))
            d0 = d1
        return out

    def search(self, dm_indices: Optional[Sequence[int]] = None, chunk: int = 32,
               timers: Optional[Dict[str, Stopwatch]] = None, progress=None,
               blocks: Optional[List[tuple]] = None, claim: Optional[Callable[[], Optional[int]]] = None) -> list:
        """Dedisperse + search DM blocks (every block's candidates, in
        processing order, as one CandidateBag): :meth:`search_iter` drained."""
        cands = _C.CandidateBag()
        slices: List[int] = []
        split = blocks is not None and any(len(b) > 2 and b[3] > 1 for b in blocks)
        for j, got in self.search_iter(dm_indices, chunk, timers, progress, blocks, claim):
            if split:
                slices.extend([int(blocks[j][2]) if len(blocks[j]) > 2 else 0] * len(got))
            cands.extend(got)
        # acceleration-sliced units (blocks of (d0, d1, s, S)): their lists are
        # raw, and the merge joins a DM's slices (merge_split_*) by these indices
        self.raw_slices = slices if split else None
        return cands

    def search_iter(self, dm_indices: Optional[Sequence[int]] = None, chunk: int = 32,
                    timers: Optional[Dict[str, Stopwatch]] = None, progress=None,
                    blocks: Optional[List[tuple]] = None, claim: Optional[Callable[[], Optional[int]]] = None):
        """Dedisperse + search DM blocks, yielding ``(block index, candidates)``
        as each block is finalized -- while the next block's dedispersion and
        searches are already in flight, so a consumer that merges or writes a
        block's candidates keeps the GPU busy (bench.py's steps: one block
        each, back to back, as a rank's DM chunks in a run).  Chunk k+1 is dedispersed on a side
        stream into the other half of a double buffer while chunk k is
        searched (the reference dedisperses the whole DM list up front,
        pipeline.cu:325-359); the search stream waits on an event, never the
        host.  ``timers['dedispersion']`` accumulates the dedispersion
        kernels' GPU time (overlapped), ``timers['searching']`` the wall time
        of the search loop.

        The blocks are ``dm_indices`` cut into ``chunk``-aligned pieces, or
        ``blocks`` as given: ``(d0, d1)``, or ``(d0, d1, s, S)`` for slice s
        of S of every DM's acceleration trials (contiguous in plan order; the
        block's lists are then raw, :func:`accel_units`); with ``claim`` (a callable returning the next
        block index or None, e.g. ``pdist.WorkQueue.claim``) the blocks are
        taken first-come from a queue shared with the other ranks -- one block
        ahead, so the next block's dedispersion still overlaps this one's
        search -- instead of in order.  Candidates come back in processing
        order; every block's candidates are contiguous."""
        tile = int(_C.Dedisperser.tile_dms)
        chunk = max(tile, (int(chunk) + tile - 1) // tile * tile)
        if blocks is None:
            blocks = self.chunk_ranges(dm_indices, chunk)
        blocks = [tuple(b) for b in blocks]
        width = max((b[1] - b[0] for b in blocks), default=0)
        if claim is None:
            order = iter(range(len(blocks)))
            claim = lambda: next(order, None)  # noqa: E731
        # the candidates stay native (CandidateBag): no per-candidate Python
        # objects, no deep copies of association trees between the engine,
        # the spills and the merge
        t_dd = timers.get("dedispersion") if timers else None
        t_s = timers.get("searching") if timers else None
        ntrials = 0
        ckdir = getattr(self.args, "checkpoint_dir", "") or ""
        fault_after = int(getattr(self.args, "fault_after_dms", -1))
        fault_rank = int(os.environ.get("PSOUP_FAULT_RANK", "-1"))  # testing: inject on this rank only
        if fault_rank >= 0 and fault_rank != self.ctx.rank:
            fault_after = -1
        processed = 0
        ckey = 0
        if ckdir:
            if self._overrides:
                raise ValueError(f"checkpoint_dir with RankSearcher overrides {self._overrides}: the spill identity "
                                 "covers the command-line options only; pass them through args instead")
            # spills are bound to this run's identity (input, header, options):
            # a spill of another run, or a corrupt/truncated one, is recomputed
            ckey = _C.prepare_checkpoint_dir(ckdir, self.args, self.header)
        dev = self.ctx.device
        if self.keep_trials:
            self.resident_rows = {}  # rows of this call only (a searcher reused across calls must not grow)
        side = _C.GpuStream()
        bufs: List[torch.Tensor] = []  # double buffer, allocated on first use
        freed = [None, None]           # event: search stream finished with the buffer
        nissued = [0]
        self.blocks_done = []

        def pull():
            """Next block: (index, spill path, resumed candidates or None,
            (buffer, ready event, start event) or None); None when the queue is dry."""
            j = claim()
            if j is None:
                return None
            d0, d1 = blocks[j][:2]
            ck = _C.spill_path(ckdir, d0, d1) if ckdir else ""
            if ck and len(blocks[j]) > 2 and blocks[j][3] > 1:
                ck += ".slice%dof%d" % (blocks[j][2], blocks[j][3])  # (a slice's raw list)
            if ck:
                status, got = _C.load_spill_bag(ck, ckey)
                if status == "loaded":
                    return j, ck, got, None
                if status != "missing":
                    warnings.warn(f"checkpoint spill {ck} is {status}; recomputing DMs {(d0, d1)}")
            k = nissued[0] % 2
            nissued[0] += 1
            start, ready = _C.GpuEvent(True), _C.GpuEvent(True)
            buf = None
            if self.keep_trials:
                # a fresh buffer per block, kept for the fold stage (never reused
                # during the search, so no wait on the previous user).  The store
                # is sized by keep_trials_fits for this rank's even share; a
                # dynamic-schedule rank that claims far more and runs out of HBM
                # keeps the rows it has and searches on from the double buffer
                # (the fold stage re-dedisperses the rows nobody kept).
                try:
                    buf = torch.empty((d1 - d0) * self.row_stride, dtype=torch.uint8, device=dev)
                    self.resident_rows[d0] = (d1, buf)
                except torch.cuda.OutOfMemoryError:
                    warnings.warn(f"rank {self.ctx.rank}: no HBM left to keep DM rows {d0}..{d1 - 1}; keeping no "
                                  "further rows (the fold stage re-dedisperses them)")
                    self.keep_trials = False
            if buf is None:
                if k >= len(bufs):
                    bufs.append(torch.empty(width * self.row_stride, dtype=torch.uint8, device=dev))
                buf = bufs[k]
                for ev in freed[k] or ():
                    ev.wait(side.handle)
            start.record(side.handle)
            with roctx_range("Dedisperse"):
                self.dedisperser.run(d0, d1, buf.data_ptr(), self.row_stride, self.kernel, side.handle)
            ready.record(side.handle)
            return j, ck, None, (k, buf, ready, start)

        dd_events = []
        lock = threading.Lock()
        # Block pipeline (one engine, blocks of at most max_prepare DMs): block
        # k's searches are launched, block k+1 is whitened into the other half
        # of the prepared slots behind them on the engine's stream, and only
        # then does the host wait for block k's batches and process their
        # peaks -- the GPU runs k+1's whitening through that host time
        pipelined = (len(self.engines) == 1 and 0 < width <= self.engine.max_prepare
                     and os.environ.get("PSOUP_BLOCK_PIPELINE", "1") != "0")
        if self.engines and (width > getattr(self, "_reserved_width", 0)
                             or (pipelined and not getattr(self, "_reserved_two", False))):
            # whitening / batch buffers sized before the timer (growing one
            # mid-search frees the old buffer, which waits for the whole device)
            ne = len(self.engines)
            per_e = max(1, min(self.engine.max_prepare, -(-width // ne)))
            for e in self.engines:
                e.reserve(per_e, per_e * self.max_trials, pipelined)
            self._reserved_width = width
            self._reserved_two = getattr(self, "_reserved_two", False) or pipelined
        cur = pull()  # the first block's dedispersion is issued before the search timer starts
        if t_s:
            t_s.start()
        # A block's per-DM acceleration distillation may still be running on
        # the engines' host workers when its batches have retired: it is
        # collected after the next block's searches are issued, so that host
        # tail overlaps GPU work (SearchEngine.search_prepared_many_async).
        prev = None  # (j, ck, d0, d1, [(engine, jobs, handle)])

        def finalize(blk):
            _, ck_, b0, b1, pend = blk
            per_dm: Dict[int, object] = {}
            for e_, jobs_, h_ in pend:
                for job, c in zip(jobs_, _C.collect_bags(e_, h_)):
                    per_dm[job[2]] = c
            chunk_cands = _C.CandidateBag()
            for d in range(b0, b1):
                chunk_cands.extend(per_dm[d])
            if ck_:
                _C.save_spill(ck_, ckey, chunk_cands)  # atomic; raises on a failed write
            return chunk_cands

        def trials_of(d, blk):
            """DM d's acceleration trials in unit ``blk`` (all, or its slice)."""
            accs = self.accel_list(self.dm_list[d])
            if len(blk) > 2 and blk[3] > 1:
                s_, S_ = blk[2], blk[3]
                accs = accs[s_ * len(accs) // S_:(s_ + 1) * len(accs) // S_]
            return accs

        half = [0]

        def prep(blk):
            """Whiten a freshly dedispersed block into the next half of the
            prepared slots; returns its first slot (None: nothing to prepare)."""
            nonlocal processed
            if blk is None or blk[3] is None:
                return None
            j_, _, _, (k_, buf_, ready_, start_) = blk
            b0_, b1_ = blocks[j_][:2]
            e_ = self.engine
            first = half[0] * e_.max_prepare
            half[0] ^= 1
            ready_.wait(e_.stream)
            dd_events.append((start_, ready_))
            with lock:
                if 0 <= fault_after < processed + (b1_ - b0_):
                    raise RuntimeError(f"fault injection: rank {self.ctx.rank} aborting after {processed} DM trials")
                processed += b1_ - b0_
            e_.prepare(buf_.data_ptr(), self.row_stride, self.geom.out_nsamps, b1_ - b0_, first)
            ev = _C.GpuEvent()
            ev.record(e_.stream)
            freed[k_] = [ev]  # the dedispersion buffer is read by the whitening alone
            return first

        cur_first = prep(cur) if pipelined else None
        while pipelined and cur is not None:
            j, ck, resumed, inflight = cur
            d0, d1 = blocks[j][:2]
            raw = len(blocks[j]) > 2 and blocks[j][3] > 1
            self.blocks_done.append(j)
            if resumed is not None:
                if prev is not None:
                    done = finalize(prev)
                    pj = prev[0]
                    prev = None
                    yield pj, done
                yield j, resumed
                ntrials += sum(len(trials_of(d, blocks[j])) for d in range(d0, d1))
                if progress is not None:
                    progress(d1 - d0)
                cur = pull()
                cur_first = prep(cur)
                continue
            e = self.engine
            nxt = pull()  # its dedispersion overlaps this block's search
            jobs = [(cur_first + i, self.dm_list[d], d, trials_of(d, blocks[j]), raw)
                    for i, d in enumerate(range(d0, d1))]
            def fail_closing(extra=None):
                # the blocks searched whole are collected and spilled before a
                # failure propagates, so a resume does not redo them
                for blk in (prev, extra):
                    if blk is not None:
                        try:
                            finalize(blk)
                        except Exception:  # the original failure is the one to report
                            pass

            try:
                h = e.search_launch(jobs)
            except BaseException:
                fail_closing()
                raise
            perr = None
            try:
                nxt_first = prep(nxt)  # behind this block's first batches on the engine's stream
            except BaseException as x:  # (this block is still finished and spilled first)
                perr = x
            try:
                e.search_finish(h)
            except BaseException:
                fail_closing()
                raise
            if perr is not None:
                fail_closing((j, ck, d0, d1, [(e, jobs, h)]))
                raise perr
            for (_, _, _, accs, _) in jobs:
                ntrials += len(accs)
                if progress is not None:
                    progress(1)
            done = finalize(prev) if prev is not None else None
            pj = prev[0] if prev is not None else -1
            prev = (j, ck, d0, d1, [(e, jobs, h)])
            cur, cur_first = nxt, nxt_first
            if done is not None:
                yield pj, done
        while cur is not None:
            j, ck, resumed, inflight = cur
            d0, d1 = blocks[j][:2]
            raw = len(blocks[j]) > 2 and blocks[j][3] > 1
            self.blocks_done.append(j)
            if resumed is not None:
                if prev is not None:  # keep the block order of the candidate list
                    done = finalize(prev)
                    pj = prev[0]
                    prev = None
                    yield pj, done
                # resume: same spill format as the native pipeline (keyed CandidatePOD trees)
                yield j, resumed
                ntrials += sum(len(trials_of(d, blocks[j])) for d in range(d0, d1))
                if progress is not None:
                    progress(d1 - d0)
                cur = pull()
                continue
            k, buf, ready, start = inflight
            ne = len(self.engines)
            tb0 = tb1 = time.perf_counter()
            if ne == 1:
                nxt = pull()  # its dedispersion overlaps the search below
                tb1 = time.perf_counter()
            for e in self.engines:
                ready.wait(e.stream)
            dd_events.append((start, ready))
            pend: list = []
            eng_t: Dict[int, list] = {}

            def run_dms(e, dms):
                # this engine's DMs are every ne-th row of the chunk: whitened
                # as batches of up to max_prepare, then searched one by one
                nonlocal processed, ntrials
                dms = list(dms)
                step = (dms[1] - dms[0]) if len(dms) > 1 else 1
                for p0 in range(0, len(dms), e.max_prepare):
                    part = dms[p0:p0 + e.max_prepare]
                    with lock:
                        if 0 <= fault_after < processed + len(part):
                            raise RuntimeError(f"fault injection: rank {self.ctx.rank} aborting after "
                                               f"{processed} DM trials")
                        processed += len(part)
                    te0 = time.perf_counter()
                    e.prepare(buf.data_ptr() + (part[0] - d0) * self.row_stride, step * self.row_stride,
                              self.geom.out_nsamps, len(part))
                    te1 = time.perf_counter()
                    jobs = [(b, self.dm_list[d], d, trials_of(d, blocks[j]), raw) for b, d in enumerate(part)]
                    # one flat trial list over the part's DMs (batches span DM boundaries)
                    h = e.search_prepared_many_async(jobs)
                    if _BLOCK_TRACE:
                        eng_t.setdefault(dms[0] - d0, []).append((te0 - tb1, te1 - te0, time.perf_counter() - te1))
                    with lock:
                        pend.append((e, jobs, h))
                        for (b, dm, d, accs, _) in jobs:
                            ntrials += len(accs)
                            if progress is not None:
                                progress(1)

            try:
                if ne == 1:
                    run_dms(self.engine, range(d0, d1))
                else:
                    futs = [self._executor().submit(run_dms, e, range(d0 + i, d1, ne))
                            for i, e in enumerate(self.engines)]
                    # the next block is issued while the engines run: whatever it
                    # costs on the host (a plan table, a spill read) no longer
                    # leaves the GPU idle
                    nxt = pull()
                    tb1 = time.perf_counter()
                    for f in futs:
                        f.result()
            except BaseException:
                # the previous block completed: collect and spill it before the
                # failure propagates, so a resume does not redo it
                if prev is not None:
                    try:
                        finalize(prev)
                    except Exception:  # the original failure is the one to report
                        pass
                    prev = None
                raise
            tb2 = time.perf_counter()
            evs = []
            for e in self.engines:
                ev = _C.GpuEvent()
                ev.record(e.stream)
                evs.append(ev)
            freed[k] = evs  # the double buffer's slot k is free once these retire
            done = finalize(prev) if prev is not None else None
            pj = prev[0] if prev is not None else -1
            prev = (j, ck, d0, d1, pend)
            if _BLOCK_TRACE:
                with open(_BLOCK_TRACE, "a") as f:
                    f.write(json.dumps({"block": j, "t0": tb0, "pull_s": tb1 - tb0, "search_s": tb2 - tb1,
                                        "engines": eng_t, "tail_s": time.perf_counter() - tb2}) + "\n")
            cur = nxt
            if done is not None:
                yield pj, done  # (this block's searches and the next block's dedispersion are in flight)
        if prev is not None:
            yield prev[0], finalize(prev)
        side.synchronize()
        for e in self.engines:
            _C.stream_synchronize(e.stream)
        if t_s:
            t_s.stop()
        if t_dd and dd_events:
            t_dd.add(sum(a.elapsed_ms(b) for a, b in dd_events) * 1e-3)
        self.accel_trials = ntrials

    def search_rows(self, rows: torch.Tensor, dm_first: int, timers: Optional[Dict[str, Stopwatch]] = None) -> list:
        """Search DM trials already resident on the GPU: ``rows`` is uint8
        ``[n, row_stride]``, row i = DM trial ``dm_first + i`` (the time-sharded
        path's DM shard after the corner turn).  Whitened in batches of
        ``max_prepare`` and searched as flat trial lists, like :meth:`search`."""
        assert rows.dtype == torch.uint8 and rows.is_cuda and rows.shape[1] == self.row_stride
        rows = rows.contiguous()
        t_s = timers.get("searching") if timers else None
        if t_s:
            t_s.start()
        torch.cuda.current_stream(self.ctx.device).synchronize()  # rows were produced on torch's stream
        e = self.engine
        cands = _C.CandidateBag()
        ntrials = 0
        base = rows.data_ptr()
        for p0 in range(0, rows.shape[0], e.max_prepare):
            cnt = min(e.max_prepare, rows.shape[0] - p0)
            e.prepare(base + p0 * self.row_stride, self.row_stride, self.geom.out_nsamps, cnt)
            jobs = [(b, self.dm_list[d], d, self.accel_list(self.dm_list[d]))
                    for b, d in enumerate(range(dm_first + p0, dm_first + p0 + cnt))]
            for (_, _, _, accs), c in zip(jobs, _C.collect_bags(e, e.search_prepared_many_async(jobs))):
                cands.extend(c)
                ntrials += len(accs)
        _C.stream_synchronize(e.stream)
        if t_s:
            t_s.stop()
        self.accel_trials = ntrials
        self.blocks_done = []
        return cands

    def fold_engine(self, njobs_hint: int = 0):
        """The searcher's FoldEngine (whitener, shift table, buffers), built on
        first use; ``njobs_hint`` > 0 also allocates a full batch's buffers
        (run_search does this before the search, outside the fold stage)."""
        if self._fold_engine is None:
            n = _C.prev_power_of_two(self.geom.out_nsamps)
            self._fold_engine = _C.FoldEngine(n, float(self.header["tsamp"]), self.stream)
        if njobs_hint > 0:
            self._fold_engine.reserve(njobs_hint)
        return self._fold_engine

    def resident_row(self, d: int) -> Optional[torch.Tensor]:
        """DM ``d``'s dedispersed row kept from the search (keep_trials), or None."""
        for d0, (d1, buf) in self.resident_rows.items():
            if d0 <= d < d1:
                return buf[(d - d0) * self.row_stride:(d - d0 + 1) * self.row_stride]
        return None

    def resident_dms(self) -> List[int]:
        return sorted(d for d0, (d1, _) in self.resident_rows.items() for d in range(d0, d1))

    def _executor(self):
        if self._pool is None:
            # engine threads bind the rank's GPU before any HIP/torch call
            # (else a multi-GPU rank's worker could create a context on GPU 0)
            kw = {}
            if self.ctx.device.type == "cuda":
                kw = dict(initializer=torch.cuda.set_device, initargs=(self.ctx.device,))
            self._pool = concurrent.futures.ThreadPoolExecutor(len(self.engines), thread_name_prefix="psoup-eng", **kw)
        return self._pool

    def counters(self) -> Dict[str, float]:
        """Engine counters summed over this rank's engines."""
        out: Dict[str, float] = {}
        for e in self.engines:
            for key, v in dict(e.counters()).items():
                out[key] = out.get(key, 0) + v
        return out

    def fold(self, groups: Dict[int, List[int]], cands: list, rows: Optional[torch.Tensor] = None,
             dm_first: int = 0) -> Dict[int, tuple]:
        """Fold candidates (index -> (folded_snr, opt_period, fold)) for the DM
        groups given; the DM trials are dedispersed again, or taken from
        resident ``rows`` (row i = DM ``dm_first + i``, see :meth:`search_rows`)."""
        out: Dict[int, tuple] = {}
        if not groups:
            return out
        fe = self.fold_engine()
        items = sorted(groups.items())
        B = int(fe.max_batch)
        t_dd = t_fe = 0.0
        n_kept = 0
        for b0 in range(0, len(items), B):
            batch = items[b0:b0 + B]
            periods = [[float(struct.unpack("f", struct.pack("f", 1.0 / cands[i].freq))[0]) for i in members]
                       for _, members in batch]
            accs = [[cands[i].acc for i in members] for _, members in batch]
            kept = [self.resident_row(d) for d, _ in batch] if rows is None and self.resident_rows else []
            if kept and all(r is not None for r in kept):
                # rows kept from the search: gathered on the device by one
                # kernel, whitened and folded (no dedispersion, no host wait)
                t0 = time.perf_counter()
                res = fe.fold_rows([r.data_ptr() for r in kept], self.geom.out_nsamps, periods, accs)
                t_fe += time.perf_counter() - t0
                n_kept += len(batch)
                for (_, members), rr in zip(batch, res):
                    for i, r in zip(members, rr):
                        out[i] = (r.folded_snr, r.opt_period, r.fold_array)
                continue
            # every DM of the batch dedispersed into one buffer, then whitened
            # and folded together (one accumulate / optimise launch)
            buf = torch.empty(len(batch) * self.row_stride, dtype=torch.uint8, device=self.ctx.device)
            torch.cuda.current_stream(self.ctx.device).synchronize()  # the allocation is ours on self.stream
            if rows is not None:
                idx = torch.tensor([d - dm_first for d, _ in batch], dtype=torch.int64, device=rows.device)
                buf.view(len(batch), self.row_stride).copy_(rows.index_select(0, idx))
                torch.cuda.current_stream(self.ctx.device).synchronize()
            else:  # one launch for the batch's (scattered) DMs
                t0 = time.perf_counter()
                self.dedisperser.run_list([d for d, _ in batch], buf.data_ptr(), self.row_stride, self.stream)
                _C.stream_synchronize(self.stream)  # (GPU time of the dedispersion included)
                t_dd += time.perf_counter() - t0
            t0 = time.perf_counter()
            res = fe.fold_trials(buf.data_ptr(), self.row_stride, self.geom.out_nsamps, periods, accs)
            t_fe += time.perf_counter() - t0
            for (_, members), rr in zip(batch, res):
                for i, r in zip(members, rr):
                    out[i] = (r.folded_snr, r.opt_period, r.fold_array)
        self.fold_stats = {"fold_dedisp_s": t_dd, "fold_engine_s": t_fe, "fold_dms": len(items),
                           "fold_batches": (len(items) + B - 1) // B, "fold_rows_kept": n_kept}
        return out


def _encode_fold_results(res: Dict[int, tuple]) -> bytes:
    parts = [struct.pack("<i", len(res))]
    for i, (snr, per, fold) in res.items():
        fold = np.ascontiguousarray(fold, dtype="<f4")
        parts.append(struct.pack("<ifdi", i, snr, per, fold.size))
        parts.append(fold.tobytes())
    return b"".join(parts)


def _decode_fold_results(b: bytes) -> Dict[int, tuple]:
    out: Dict[int, tuple] = {}
    (n,) = struct.unpack_from("<i", b, 0)
    off = 4
    for _ in range(n):
        i, snr, per, nf = struct.unpack_from("<ifdi", b, off)
        off += struct.calcsize("<ifdi")
        fold = np.frombuffer(b, dtype="<f4", count=nf, offset=off)
        off += 4 * nf
        out[i] = (snr, per, fold)
    return out


def broadcast_header(infilename: str, ctx: pdist.DistContext) -> dict:
    """Rank 0 reads the SIGPROC header; every rank gets it (RCCL broadcast)."""
    hdr_bytes = None
    if ctx.is_root:
        hdr_bytes = repr(_C.read_header(infilename)).encode()
    hdr_bytes = pdist.broadcast_object_bytes(hdr_bytes)
    import ast

    return ast.literal_eval(hdr_bytes.decode())


def load_packed_for_rank(infilename: str, ctx: pdist.DistContext, timers=None):
    """Rank 0 reads the filterbank; the packed bytes are RCCL-broadcast to
    every rank's GPU.  Returns (header, packed_tensor_on_device, nsamps).
    With ``timers``, "reading" (running on entry) stops after the file read and
    the device upload is charged to "dedispersion" (the reference's timers:
    pipeline_multi.cu:287-289 read the file, its dedispersion copies it to
    the GPU)."""
    header = None
    packed = None
    if ctx.is_root:
        fb = _C.Filterbank.from_file(infilename)
        header = fb.header
        nbytes = int(fb.data_bytes)
        hdr_bytes = repr(header).encode()
    else:
        hdr_bytes = None
    hdr_bytes = pdist.broadcast_object_bytes(hdr_bytes)
    if header is None:
        import ast

        header = ast.literal_eval(hdr_bytes.decode())
    nsamps = int(header["nsamples"])
    nbytes = nsamps * int(header["nchans"]) * int(header["nbits"]) // 8
    if timers is not None:
        timers["reading"].stop()
        timers["dedispersion"].start()
    if ctx.device.type == "cuda":
        packed = torch.empty(nbytes, dtype=torch.uint8, device=ctx.device)
        if ctx.is_root:
            # threaded pread into pinned stages, copies overlapping the reads
            # (a copy out of the fresh mapping faults every page in: ~0.15 s
            # for config 4's 268 MB, ~10 ms this way)
            torch.cuda.synchronize(ctx.device)
            if nbytes > fb.data_bytes:
                raise ValueError(f"{infilename}: header promises {nbytes} data bytes, the file holds {fb.data_bytes}")
            fb.upload(packed.data_ptr(), nbytes, packed.numel(), torch.cuda.current_stream(ctx.device).cuda_stream)
        if ctx.distributed:
            pdist.broadcast_bytes(packed, nbytes)
    else:
        packed = torch.from_numpy(fb.data()[:nbytes].copy()) if ctx.is_root else None
    if timers is not None:
        if ctx.device.type == "cuda":
            torch.cuda.synchronize()
        timers["dedispersion"].stop()
    return header, packed, nsamps


DYNAMIC_CHUNK = 32  # DMs per claimed block (the dedispersion tile multiple the static path also uses)


def static_chunk(nshard: int) -> int:
    """DMs per block of a static shard: the engine call of a block waits for
    its last batch and processes its peaks before the next block is issued,
    so larger blocks of a long shard leave the GPU idle less often (that
    host gap is ~0.7 ms per block on config 4: 64-DM blocks 0.254-0.266 s
    of search against 0.272-0.274 at 32 and 0.259-0.274 at 128, same box).
    PSOUP_STATIC_CHUNK overrides (a multiple of the 32-DM dedispersion tile)."""
    env = os.environ.get("PSOUP_STATIC_CHUNK")
    if env:
        return max(DYNAMIC_CHUNK, int(env) // DYNAMIC_CHUNK * DYNAMIC_CHUNK)
    return 2 * DYNAMIC_CHUNK if nshard >= 8 * DYNAMIC_CHUNK else DYNAMIC_CHUNK


def dm_schedule(args, world_size: int, ndm: Optional[int] = None) -> str:
    """``--dm_schedule``: "dynamic" (first-come DM chunks from a queue shared
    by the ranks), "static" (contiguous trial-weighted shards); auto = dynamic
    for more than one rank when the list has at least 4 chunks per rank (with
    fewer, 32-DM chunks leave ranks idle: 113 DMs on 8 ranks ran 4 ranks,
    tools/expt/dyn8_rehearsal.sh), else static.  An explicit "dynamic" is
    honoured on one rank too (the rank claims every chunk from the queue)."""
    s = (getattr(args, "dm_schedule", "auto") or "auto").lower()
    if s not in ("auto", "dynamic", "static"):
        raise ValueError(f"--dm_schedule must be dynamic, static or auto, not {s!r}")
    if world_size <= 1:
        return "dynamic" if s == "dynamic" else "static"
    if s == "auto":
        enough = ndm is None or (ndm + DYNAMIC_CHUNK - 1) // DYNAMIC_CHUNK >= 4 * world_size
        return "dynamic" if enough else "static"
    return s


MIN_SLICE_TRIALS = 64  # auto slicing keeps at least this many acceleration trials per DM and unit


def accel_slices(args, world: int, nblocks: int, max_trials: int) -> int:
    """Slices per DM of the acceleration trials (``--accel_slices``; 0 =
    auto).  A job with fewer DM chunks than 4 per rank (a single DM at 2^23,
    a short DM list on 8 GPUs) would leave ranks idle or finish on a few:
    auto cuts every DM's trial list into S contiguous slices so that the
    (chunk, slice) units number at least 4 per rank, with at least
    MIN_SLICE_TRIALS trials per slice.  One rank: no slicing."""
    v = int(getattr(args, "accel_slices", 0) or 0)
    if v > 0:
        return v
    if world <= 1 or nblocks <= 0 or nblocks >= 4 * world:
        return 1
    want = -(-4 * world // nblocks)
    cap = max(1, min(want, max_trials // MIN_SLICE_TRIALS))
    # prefer a unit count the ranks divide evenly (1 DM on 8 ranks: 8 slices,
    # not 10) unless that gives up more than half the slices
    for s_ in range(cap, 0, -1):
        if (nblocks * s_) % world == 0:
            return s_ if 2 * s_ >= cap else cap
    return cap


def accel_units(blocks: List[tuple], S: int) -> List[tuple]:
    """Work units: every DM block, or (d0, d1, s, S) for each of its S
    acceleration slices (block-major, so ranks claiming in turn take the
    slices of one block)."""
    if S <= 1:
        return [tuple(b[:2]) for b in blocks]
    return [(b[0], b[1], s_, S) for b in blocks for s_ in range(S)]


def unit_weight(rs: "RankSearcher", unit: tuple) -> int:
    """Acceleration trials a work unit searches."""
    tot = 0
    for d in range(unit[0], unit[1]):
        n = len(rs.accel_list(rs.dm_list[d]))
        if len(unit) > 2 and unit[3] > 1:
            n = (unit[2] + 1) * n // unit[3] - unit[2] * n // unit[3]
        tot += n
    return tot


def keep_trials_fits(rs: RankSearcher, ndm: int, world: int) -> bool:
    """Keep every searched DM row in HBM for the fold stage when this rank's
    share (with 2x slack for dynamic-schedule imbalance) fits in a quarter of
    the free device memory.  PSOUP_KEEP_TRIALS=0/1 forces it."""
    env = os.environ.get("PSOUP_KEEP_TRIALS")
    if env is not None:
        return env not in ("0", "")
    if rs.ctx.device.type != "cuda":
        return False
    free, _ = torch.cuda.mem_get_info(rs.ctx.device)
    share = (ndm + world - 1) // world * (2 if world > 1 else 1)
    return share * rs.row_stride <= free // 4


def fold_owners(rs: RankSearcher, ctx) -> Dict[int, int]:
    """DM index -> the rank that kept its dedispersed row (all ranks agree:
    every rank's kept ranges are all-gathered)."""
    mine = [(d0, d1) for d0, (d1, _) in sorted(rs.resident_rows.items())]
    if ctx.world_size == 1:
        return {d: 0 for d0, d1 in mine for d in range(d0, d1)}
    blobs = pdist.gather_bytes(json.dumps(mine).encode(), dst=None)
    owner: Dict[int, int] = {}
    for r, b in enumerate(blobs):
        for d0, d1 in json.loads(b.decode()):
            for d in range(d0, d1):
                owner.setdefault(d, r)
    return owner


def run_search(args, write: bool = True, as_rank: Optional[tuple] = None) -> Optional[SearchResult]:
    """Full distributed search (torchrun: one rank per GPU).  Returns the
    result on rank 0 (None elsewhere).

    ``as_rank=(W, r)`` (one process): rank r's whole share of a W-rank run --
    setup for its static DM shard, its search, a merge of its own list -- so
    one GPU can time every rank of a larger job (tools/baseline_configs.py
    --as-rank)."""
    ctx = pdist.init()
    if as_rank is not None:
        assert ctx.world_size == 1 and 0 <= as_rank[1] < as_rank[0], as_rank
    timers = {k: Stopwatch() for k in ("reading", "dedispersion", "searching", "folding", "total")}
    timers["total"].start()
    # device start-up (context, allocator, kernel code objects) in "total"
    # only, as the reference's context creation: stage timers hold stage work
    device_init_s = 0.0
    if ctx.device.type == "cuda":
        t_init = time.perf_counter()
        torch.empty(1, device=ctx.device)
        _C.warm_device()
        device_init_s = time.perf_counter() - t_init
    timers["reading"].start()
    sharded = bool(getattr(args, "time_shards", False))
    if sharded:
        header, packed, nsamps = broadcast_header(args.infilename, ctx), None, 0
        nsamps = int(header["nsamples"])
        timers["reading"].stop()
    else:
        header, packed, nsamps = load_packed_for_rank(args.infilename, ctx, timers)

    rs = RankSearcher(args, header, packed, nsamps, resident=not sharded, warm=False)
    del packed
    ndm = len(rs.dm_list)
    weights = [len(rs.accel_list(d)) for d in rs.dm_list]
    world = ctx.world_size if as_rank is None else as_rank[0]
    # work units: 32-DM chunks, each cut into S acceleration slices when the
    # job has too few chunks for the ranks (accel_slices)
    nslices = 1 if sharded else accel_slices(args, world, -(-ndm // DYNAMIC_CHUNK), max(weights, default=0))
    units = accel_units(rs.chunk_ranges(range(ndm), DYNAMIC_CHUNK), nslices) if nslices > 1 else None
    if units is not None:
        schedule = "static" if as_rank else dm_schedule(args, world, len(units) * DYNAMIC_CHUNK)
    else:
        schedule = "time_sharded" if sharded else "static" if as_rank else dm_schedule(args, world, ndm)
    my_units = None
    if schedule == "static" and units is not None:
        uw = [unit_weight(rs, u) for u in units]
        us = pdist.shard_range(len(units), world, ctx.rank if as_rank is None else as_rank[1], uw)
        my_units = [units[i] for i in us]
        if my_units:
            rs.warm(my_units[0][0], my_units[-1][1])
    elif schedule == "static":
        # a static shard's plan tables only (dynamic ranks may claim any chunk)
        shard = pdist.shard_range(ndm, world, ctx.rank if as_rank is None else as_rank[1], weights)
        if len(shard):
            rs.warm(shard.start, shard.stop)
    elif not sharded:
        rs.warm()
    rows = None
    row_first = 0
    if not sharded and args.npdmp > 0:
        rs.keep_trials = keep_trials_fits(rs, ndm, world)
    if args.npdmp > 0 and _C.prev_power_of_two(rs.geom.out_nsamps) >= 1024:
        rs.fold_engine(njobs_hint=args.npdmp)  # folder buffers allocated with the rest of the setup
    pdist.barrier()
    t0 = time.perf_counter()
    if sharded:
        # every rank holds only its time slice of the filterbank;
        # ring halo exchange + all-to-all corner turn hand each rank whole DM
        # series for its trial-weighted DM shard, searched in place
        from ..parallel import timeshard

        plan = timeshard.make_plan(rs.header, nsamps, rs.dm_list, ctx.world_size, weights)
        timers["reading"].start()
        fb = _C.Filterbank.from_file(args.infilename)
        rr = plan.input_range(ctx.rank)
        with warnings.catch_warnings():  # read-only mmap view, only copied to the device
            warnings.simplefilter("ignore", UserWarning)
            own = torch.from_numpy(fb.data()[rr.start * plan.bytes_per_sample:rr.stop * plan.bytes_per_sample])
            own = own.to(ctx.device)
        del fb
        timers["reading"].stop()
        timers["dedispersion"].start()
        dd = timeshard.native_dedisperser(rs.header, rs.dm_list, list(rs.geom.killmask), kernel=args.dedisp_kernel)
        trials = timeshard.time_sharded_dedisperse(own, plan, dd)
        del own
        shard = plan.dm_shards[ctx.rank]
        rows = torch.zeros((len(shard), rs.row_stride), dtype=torch.uint8, device=ctx.device)
        rows[:, :rs.geom.out_nsamps] = trials
        del trials
        torch.cuda.synchronize()
        timers["dedispersion"].stop()
        row_first = shard.start
        local = rs.search_rows(rows, shard.start, timers)
        local_trials = sum(weights[i] for i in shard)
    elif schedule == "dynamic":
        # DMDispenser across processes: every rank claims 32-DM chunks (or
        # their acceleration slices) of the whole list from one shared
        # first-come queue (pipeline_multi.cu:33-81)
        blocks = units if units is not None else rs.chunk_ranges(range(ndm), DYNAMIC_CHUNK)
        queue = pdist.WorkQueue("dm_chunks", len(blocks))
        local = rs.search(blocks=blocks, claim=queue.claim, timers=timers)
        local_trials = sum(unit_weight(rs, blocks[j]) for j in rs.blocks_done)
    elif my_units is not None:
        local = rs.search(blocks=my_units, timers=timers)
        local_trials = sum(unit_weight(rs, u) for u in my_units)
    else:
        local = rs.search(shard, timers=timers, chunk=static_chunk(len(shard)))
        local_trials = sum(weights[i] for i in shard)
    torch.cuda.synchronize()
    search_wall = time.perf_counter() - t0
    rank_stats = rs.counters()
    rank_stats.update({"rank": ctx.rank, "search_s": search_wall, "accel_trials_planned": local_trials,
                       "device_init_s": device_init_s, "accel_slices": nslices,
                       "dm_schedule": schedule, "dm_blocks": len(rs.blocks_done),
                       "fft_mode": rs.engine.fft_mode, "accel_batch": rs.engine.batch_size,
                       "sub_batch": rs.engine.sub_batch,
                       "dedispersion_s": timers["dedispersion"].get_time(), "searching_s": timers["searching"].get_time()})
    all_stats = pdist.gather_bytes(json.dumps(rank_stats).encode(), dst=0)

    # ---- candidate gather (RCCL) + global distillation on rank 0
    total_trials = sum(weights) if as_rank is None else local_trials
    raw_slices = getattr(rs, "raw_slices", None) if nslices > 1 else None
    if nslices > 1 and raw_slices is None:
        raw_slices = []  # (a rank that searched no unit)
    if not ctx.distributed:
        # a world of one: the merge takes the rank's own list (no serialisation)
        if raw_slices is not None:
            cands = _C.merge_split_local(local, raw_slices, args, rs.header)
        else:
            cands = _C.merge_local(local, args, rs.header)
    else:
        # every rank's list to rank 0 only (RCCL gather of raw buffers), merged
        # there: rank order, stable by DM index, global distillation, scoring.
        # Acceleration-sliced units: their raw lists and slice indices, each
        # DM's slices joined in plan order and acceleration-distilled on rank 0
        # first (the list an unsplit DM's engine distils: identical output)
        bufs = pdist.gather_buffers(torch.from_numpy(_C.serialize_candidates_array(local)), dst=0)
        sbufs = None
        if raw_slices is not None:
            sl = np.asarray(raw_slices, dtype=np.int32)
            sbufs = pdist.gather_buffers(torch.from_numpy(sl.view(np.uint8)), dst=0)
        del local
        if not ctx.is_root:
            cands = None
        elif sbufs is not None:
            cands = _C.merge_split_buffers([(b.data_ptr(), b.numel()) for b in bufs],
                                           [(b.data_ptr(), b.numel() // 4) for b in sbufs], args, rs.header)
        else:
            cands = _C.merge_candidate_buffers([(b.data_ptr(), b.numel()) for b in bufs], args, rs.header)
        del bufs, sbufs
        if args.npdmp > 0:
            # the fold stage needs the top candidates' frequency, acceleration
            # and DM row on every rank (not their association trees)
            cands = _FoldView.share(cands, min(args.npdmp, len(cands)) if cands is not None else 0)
    search_wall = pdist.all_reduce_max_float(search_wall)

    # ---- distributed folding (all ranks hold identical `cands`)
    timers["folding"].start()
    fold_stats: Dict[str, float] = {}
    if args.npdmp > 0 and cands:
        groups = {}
        count = min(args.npdmp, len(cands))
        for i in range(count):
            p = float(struct.unpack("f", struct.pack("f", 1.0 / cands[i].freq))[0])
            if 0.001 < p < 10.0:
                groups.setdefault(cands[i].dm_idx, []).append(i)
        keys = sorted(groups)
        if rows is not None:  # time-sharded: the owner of the DM row folds it
            mine = {k: groups[k] for k in keys if row_first <= k < row_first + rows.shape[0]}
        else:
            # the rank holding a DM's dedispersed row (keep_trials) folds it;
            # DMs nobody kept (resumed blocks) go round-robin
            owner = fold_owners(rs, ctx)
            rest = [k for k in keys if k not in owner]
            mine = {k: groups[k] for k in keys if owner.get(k) == ctx.rank}
            mine.update({k: groups[k] for j, k in enumerate(rest) if j % ctx.world_size == ctx.rank})
        t_f0 = time.perf_counter()
        res = rs.fold(mine, cands, rows=rows, dm_first=row_first)
        t_f1 = time.perf_counter()
        # one rank: the results as they are; more: encoded and gathered to rank 0
        parts = [res] if ctx.world_size == 1 else [
            _decode_fold_results(p) for p in pdist.gather_bytes(_encode_fold_results(res), dst=0) or []]
        if ctx.is_root:
            for part in parts:
                for i, (snr, per, fold) in part.items():
                    c = cands[i]
                    c.folded_snr = snr
                    c.opt_period = per
                    c.set_fold_array(fold, 64, 16)
            # sort_by_folded_snr's permutation, applied to the Python list
            order = _C.sort_order_by_folded_snr([c.snr for c in cands], [c.folded_snr for c in cands])
            cands.permute(order)
        fold_stats = dict(getattr(rs, "fold_stats", {}))
        fold_stats.update({"fold_call_s": t_f1 - t_f0, "fold_merge_s": time.perf_counter() - t_f1})
    timers["folding"].stop()
    if not ctx.is_root:
        timers["total"].stop()
        return None
    cands.truncate(max(0, args.limit))
    timers["total"].stop()
    perf = {
        "dm_accel_trials": float(total_trials),
        "dm_accel_trials_per_sec": total_trials / search_wall if search_wall > 0 else 0.0,
        "ranks": float(ctx.world_size),
    }
    tdict = {k: v.get_time() for k, v in timers.items()}
    acc0 = rs.accel_list(0.0)
    res = SearchResult(cands, tdict, perf, rs.dm_list, acc0, list(range(ctx.world_size)) if ctx.device.type == "cuda" else [],
                       rs.header, args, total_trials)
    res.rank_stats = [json.loads(b.decode()) for b in all_stats] if all_stats else []
    res.fold_stats = fold_stats  # rank 0's fold-stage breakdown (seconds)
    if write:
        write_outputs(args, res)
    return res


class _FoldView:
    """Rank r != 0's view of the merged list for the fold stage: the first
    ``n`` candidates' (freq, acc, dm_idx), broadcast from rank 0 (20 bytes per
    candidate) -- indexable like the list, for :meth:`RankSearcher.fold`."""

    class _C:
        __slots__ = ("freq", "acc", "dm_idx")

        def __init__(self, freq, acc, dm_idx):
            self.freq, self.acc, self.dm_idx = freq, acc, dm_idx

    def __init__(self, rows):
        self._rows = rows

    def __len__(self):
        return len(self._rows)

    def __getitem__(self, i):
        return self._rows[i]

    def __bool__(self):
        return bool(self._rows)

    @staticmethod
    def share(cands, n):
        """On rank 0 return ``cands`` (after broadcasting its head); elsewhere a _FoldView."""
        import numpy as np

        ctx = pdist.context()
        if ctx.is_root:
            head = np.zeros(n, dtype=[("freq", "<f4"), ("acc", "<f4"), ("dm_idx", "<i4")])
            for i in range(n):
                head[i] = (cands[i].freq, cands[i].acc, cands[i].dm_idx)
            pdist.broadcast_object_bytes(head.tobytes())
            return cands
        raw = pdist.broadcast_object_bytes(None)
        head = np.frombuffer(raw, dtype=[("freq", "<f4"), ("acc", "<f4"), ("dm_idx", "<i4")])
        return _FoldView([_FoldView._C(float(r["freq"]), float(r["acc"]), int(r["dm_idx"])) for r in head])


def trace_dict(args, res: SearchResult) -> dict:
    """The --trace_json document (same layout as the native CLI's)."""
    return {
        "input": args.infilename,
        "config": {"fft_size": int(args.size) or None, "nharmonics": args.nharmonics, "ndm": len(res.dm_list),
                   "acc_start": args.acc_start, "acc_end": args.acc_end,
                   "accel_convention": args.accel_convention, "dedisp_kernel": args.dedisp_kernel,
                   "fft_mode": args.fft_mode},
        "timers_s": res.timers,
        "performance": res.performance,
        "devices": res.rank_stats,
        "candidates": len(res.candidates),
    }


def write_outputs(args, res: SearchResult) -> None:
    os.makedirs(args.outdir, exist_ok=True)
    if getattr(args, "trace_json", ""):
        with open(args.trace_json, "w") as f:
            json.dump(trace_dict(args, res), f, indent=2)
    bm = _C.write_candidates_binary(args.outdir, res.candidates, "candidates.peasoup")
    devices = [torch.cuda.current_device()] if res.devices else []
    if len(res.devices) > 1:
        devices = list(range(min(len(res.devices), torch.cuda.device_count())))
    _C.write_overview(os.path.join(args.outdir, "overview.xml"), args, args.infilename, res.dm_list, res.acc_list0,
                      devices, res.candidates, bm, res.timers, res.performance)
