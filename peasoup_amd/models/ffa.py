"""Distributed FFA periodicity search: one process per GPU (torchrun), the
same distribution model as the acceleration search (models/search.py):

1. rank 0 reads the ``.fil``; the packed bytes are RCCL-broadcast and every
   rank keeps a channel-major filterbank resident in HBM;
2. each rank dedisperses (MFMA kernel) a contiguous DM shard and runs the
   native ``FfaEngine`` on every trial (detrend, octave downsampling,
   batched FFA, boxcar S/N, per-DM clustering);
3. candidates are gathered to rank 0 over RCCL and clustered across DMs;
   rank 0 writes the text output.

Reference: the FFA options of include/utils/cmdline.hpp:35-67, 211-292 and
the ``ffaster`` target (Makefile:41-42; its source is not in the reference).
"""
from __future__ import annotations

import struct
import time
from typing import List, Optional

import torch

from .. import _C, dedisp_kernel
from ..parallel import dist as pdist
from ..utils.timing import Stopwatch
from .search import load_packed_for_rank

_REC = struct.Struct("<dfiifii")  # period, snr, width, nbins, dm, dm_idx, octave


def encode_candidates(cands) -> bytes:
    return struct.pack("<i", len(cands)) + b"".join(
        _REC.pack(c.period, c.snr, c.width, c.nbins, c.dm, c.dm_idx, c.octave) for c in cands)


def decode_candidates(b: bytes) -> list:
    (n,) = struct.unpack_from("<i", b, 0)
    out = []
    for i in range(n):
        period, snr, width, nbins, dm, dm_idx, octave = _REC.unpack_from(b, 4 + i * _REC.size)
        c = _C.FfaCandidate()
        c.period, c.snr, c.width, c.nbins, c.dm, c.dm_idx, c.octave = period, snr, width, nbins, dm, dm_idx, octave
        out.append(c)
    return out


class RankFfa:
    """Per-rank FFA state: resident filterbank, dedisperser, FFA engine."""

    def __init__(self, args, header: dict, packed: Optional[torch.Tensor], nsamps: int):
        self.ctx = pdist.context()
        self.args = args
        self.header = dict(header)
        self.dm_list = list(_C.generate_dm_list(args.dm_start, args.dm_end, header["tsamp"], args.dm_pulse_width,
                                                header["fch1"], header["foff"], header["nchans"], args.dm_tol))
        kill = [1] * int(header["nchans"])
        if args.killfilename:
            kill = list(_C.read_killfile(args.killfilename, int(header["nchans"]))[0])
        self.geom = _C.DedispGeometry.make(self.header, int(nsamps), self.dm_list, kill)
        self.stream = torch.cuda.current_stream().cuda_stream
        self.dfb = _C.DeviceFilterbank(self.geom, self.stream)
        if packed is not None:
            if packed.is_cuda:
                self.dfb.load_packed_device(packed.data_ptr())
            else:
                self.dfb.load_packed_host(packed.data_ptr())
        self.dedisperser = _C.Dedisperser(self.dfb, self.stream)
        self.kernel = dedisp_kernel(args.dedisp_kernel)
        self.params = _C.ffa_params_from(args, float(header["tsamp"]))
        self.engine = _C.FfaEngine(self.params, int(self.geom.out_nsamps), self.stream)
        self.row_stride = _C.Dedisperser.row_stride(self.geom.out_nsamps)
        self._trials: Optional[torch.Tensor] = None

    def search(self, dm_indices, chunk: int = 32) -> list:
        from .search import RankSearcher

        out: list = []
        # chunks cut at multiples of the dedispersion tile (resident plans)
        for d0, d1 in RankSearcher.chunk_ranges(dm_indices, chunk):
            block = range(d0, d1)
            need = (d1 - d0) * self.row_stride
            if self._trials is None or self._trials.numel() < need:
                self._trials = torch.empty(need, dtype=torch.uint8, device=self.ctx.device)
            self.dedisperser.run(d0, d1, self._trials.data_ptr(), self.row_stride, self.kernel)
            for k, d in enumerate(block):
                out.extend(self.engine.search(self._trials.data_ptr() + k * self.row_stride, self.dm_list[d], d))
        return out


def run_ffa_search(args, write: bool = True):
    """Distributed FFA search; returns the FfaResult on rank 0 (None elsewhere)."""
    ctx = pdist.init()
    timers = {k: Stopwatch() for k in ("reading", "searching", "total")}
    timers["total"].start()
    timers["reading"].start()
    header, packed, nsamps = load_packed_for_rank(args.infilename, ctx)
    timers["reading"].stop()
    rf = RankFfa(args, header, packed, nsamps)
    del packed
    shard = pdist.shard_range(len(rf.dm_list), ctx.world_size, ctx.rank)
    pdist.barrier()
    timers["searching"].start()
    t0 = time.perf_counter()
    local = rf.search(shard)
    torch.cuda.synchronize()
    wall = pdist.all_reduce_max_float(time.perf_counter() - t0)
    timers["searching"].stop()
    blobs = pdist.gather_bytes(encode_candidates(local), dst=0)
    if not ctx.is_root:
        return None
    cands: List = []
    for b in blobs:
        cands.extend(decode_candidates(b))
    cands.sort(key=lambda c: (c.dm_idx, c.period))
    tobs = float(rf.engine.tobs)
    cands = _C.ffa_cluster(cands, rf.params.cluster_tol / tobs)[: max(0, args.limit)]
    timers["total"].stop()
    res = _C.FfaResult()
    res.candidates = cands
    res.dm_list = rf.dm_list
    res.devices = list(range(ctx.world_size))
    res.timers = {k: v.get_time() for k, v in timers.items()} | {"searching_wall": wall}
    res.nsamps = int(rf.geom.out_nsamps)
    res.tobs = tobs
    res.nb0 = int(_C.ffa_base_bins(rf.params))
    if write:
        _C.write_ffa_output(args.outfilename, args, res)
    return res
