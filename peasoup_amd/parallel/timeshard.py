"""Time-sharded dedispersion for series longer than one GPU holds
(the "Ulysses analog" of the inventory's §2.7 row).

The reference keeps the whole series on one GPU.  With 288 GB of HBM per
MI355X that remains the default here; this module is the scale-out path when
a filterbank does not fit (or should not be replicated) on every rank:

1. each rank holds only its own slice of the packed filterbank: the input
   samples of its output time window ``[o0, o1)``;
2. a ring **halo exchange** (point-to-point send/recv over xGMI) appends the
   next rank's first ``max_delay`` samples, so the rank can dedisperse every
   DM trial for its window;
3. an **all-to-all corner turn** (``all_to_all_single``) re-distributes the
   ``[ndm][window]`` blocks from time shards to DM shards, so each rank again
   owns whole time series for its DM range and the normal per-DM search runs
   unchanged.

The dedispersion itself is pluggable: :func:`native_dedisperser` runs the
MFMA kernel on the rank's GPU, :func:`reference_dedisperser` the NumPy oracle
(CPU tests on gloo).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from . import dist as pdist

DedispFn = Callable[[torch.Tensor, int, int], torch.Tensor]


@dataclass
class TimeShardPlan:
    nsamps: int          # input samples of the whole observation
    max_delay: int
    out_nsamps: int      # dedispersed samples of the whole observation
    bytes_per_sample: int
    windows: List[range]  # output-sample window of each rank
    dm_shards: List[range]

    def input_range(self, rank: int) -> range:
        """Input samples rank ``rank`` holds before the halo exchange."""
        w = self.windows[rank]
        end = self.nsamps if rank == len(self.windows) - 1 else w.stop
        return range(w.start, end)


def make_plan(header: dict, nsamps: int, dm_list: Sequence[float], world: int,
              dm_weights: Optional[Sequence[float]] = None) -> TimeShardPlan:
    from .. import _C

    delays = _C.generate_delay_table(int(header["nchans"]), float(header["tsamp"]), float(header["fch1"]),
                                     float(header["foff"]))
    max_delay = int(_C.compute_max_delay(list(dm_list), delays))
    out = nsamps - max_delay
    if out <= 0:
        raise ValueError("observation shorter than the maximum dispersion delay")
    windows = [pdist.shard_range(out, world, r) for r in range(world)]
    if world > 1 and min(len(w) for w in windows[:-1]) < max_delay:
        raise ValueError("time shards must be at least max_delay samples long (use fewer ranks)")
    bps = int(header["nchans"]) * int(header["nbits"]) // 8
    if int(header["nchans"]) * int(header["nbits"]) % 8:
        raise ValueError("nchans * nbits must be a whole number of bytes")
    shards = [pdist.shard_range(len(dm_list), world, r, dm_weights) for r in range(world)]
    return TimeShardPlan(nsamps, max_delay, out, bps, windows, shards)


def _p2p(t: torch.Tensor, ctx) -> torch.Tensor:
    return t.cpu() if ctx.backend == "gloo" and t.is_cuda else t


def exchange_halo(own: torch.Tensor, plan: TimeShardPlan) -> torch.Tensor:
    """Ring halo exchange: returns ``own`` (this rank's packed input bytes)
    extended by the first ``max_delay`` samples of the next rank's slice."""
    ctx = pdist.context()
    halo = plan.max_delay * plan.bytes_per_sample
    if not ctx.distributed or halo == 0:
        return own
    r, w = ctx.rank, ctx.world_size
    reqs = []
    send_buf = None
    if r > 0:  # my head is the previous rank's halo
        send_buf = _p2p(own[:halo].contiguous(), ctx)
        reqs.append(dist.isend(send_buf, r - 1))
    recv = None
    if r < w - 1:
        recv = torch.empty(halo, dtype=torch.uint8, device=send_buf.device if send_buf is not None
                           else _p2p(own[:1], ctx).device)
        reqs.append(dist.irecv(recv, r + 1))
    for q in reqs:
        q.wait()
    if recv is None:
        return own
    return torch.cat([own, recv.to(own.device)])


def corner_turn(local: torch.Tensor, plan: TimeShardPlan) -> torch.Tensor:
    """All-to-all from time shards ``[ndm][len(window_r)]`` to DM shards:
    returns ``[len(dm_shard_r)][out_nsamps]`` for this rank."""
    ctx = pdist.context()
    if not ctx.distributed:
        return local
    r, w = ctx.rank, ctx.world_size
    win = len(plan.windows[r])
    assert local.shape[1] == win
    send = torch.cat([local[s.start:s.stop].reshape(-1) for s in plan.dm_shards])
    in_splits = [len(s) * win for s in plan.dm_shards]
    out_splits = [len(plan.dm_shards[r]) * len(wq) for wq in plan.windows]
    send_c = _p2p(send, ctx)
    recv = torch.empty(sum(out_splits), dtype=torch.uint8, device=send_c.device)
    dist.all_to_all_single(recv, send_c, out_splits, in_splits)
    recv = recv.to(local.device)
    nd = len(plan.dm_shards[r])
    parts, off = [], 0
    for wq, n in zip(plan.windows, out_splits):
        parts.append(recv[off:off + n].view(nd, len(wq)))
        off += n
    return torch.cat(parts, dim=1)


def time_sharded_dedisperse(own_packed: torch.Tensor, plan: TimeShardPlan, dedisp: DedispFn) -> torch.Tensor:
    """Full time-sharded dedispersion on this rank: halo exchange, local
    dedispersion of every DM for the rank's window, corner turn.  Returns the
    rank's DM shard as ``uint8 [ndm_local][out_nsamps]``."""
    ctx = pdist.context()
    window = plan.windows[ctx.rank]
    ext = exchange_halo(own_packed, plan)
    nin = ext.numel() // plan.bytes_per_sample
    local = dedisp(ext, nin, len(window))
    return corner_turn(local, plan)


# ------------------------------------------------------------ dedispersers --
def reference_dedisperser(header: dict, dm_list: Sequence[float], killmask=None) -> DedispFn:
    """NumPy oracle (CPU)."""
    from ..utils import reference as ref
    from ..utils import sigproc

    nchans, nbits = int(header["nchans"]), int(header["nbits"])
    offs = ref.dm_offsets(dm_list, ref.delay_table(nchans, float(header["tsamp"]), float(header["fch1"]),
                                                   float(header["foff"])))

    def fn(packed: torch.Tensor, nin: int, nout: int) -> torch.Tensor:
        vals = sigproc.unpack_samples(packed.cpu().numpy(), nin, nchans, nbits)
        return torch.from_numpy(ref.dedisperse(vals, offs, nbits, killmask, nout))

    return fn


def native_dedisperser(header: dict, dm_list: Sequence[float], killmask=None, kernel: str = "auto") -> DedispFn:
    """Dedispersion of the rank's (haloed) window on its GPU (kernel: auto |
    mfma | valu | direct | packed2; bit-identical outputs)."""
    from .. import _C, dedisp_kernel

    def fn(packed: torch.Tensor, nin: int, nout: int) -> torch.Tensor:
        hdr = dict(header)
        hdr["nsamples"] = nin
        g = _C.DedispGeometry.make(hdr, nin, list(dm_list), list(killmask or []))
        assert g.out_nsamps == nout, (g.out_nsamps, nout)
        stream = torch.cuda.current_stream().cuda_stream
        dfb = _C.DeviceFilterbank(g, stream)
        dfb.load_packed_device(packed.data_ptr())
        dd = _C.Dedisperser(dfb, stream)
        stride = _C.Dedisperser.row_stride(nout)
        out = torch.empty((len(dm_list), stride), dtype=torch.uint8, device=packed.device)
        dd.run(0, len(dm_list), out.data_ptr(), stride, dedisp_kernel(kernel))
        torch.cuda.current_stream().synchronize()
        return out[:, :nout]

    return fn


def slice_packed(packed: np.ndarray, plan: TimeShardPlan, rank: int) -> np.ndarray:
    """This rank's own input bytes from a whole packed filterbank (how a
    rank would read only its part of the file)."""
    rr = plan.input_range(rank)
    return packed[rr.start * plan.bytes_per_sample: rr.stop * plan.bytes_per_sample]
