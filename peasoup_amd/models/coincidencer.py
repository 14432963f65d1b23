"""Multi-beam RFI coincidencer (src/coincidencer.cpp:46-215,
include/transforms/coincidencer.hpp:17-85).

Each beam (filterbank) is dedispersed at DM 0, whitened (running median),
and both its normalised time series and its normalised interbinned spectrum
are thresholded.  A time sample / Fourier bin is flagged as RFI when it
exceeds ``thresh`` in at least ``beam_thresh`` beams.

Distributed form: beams are spread over the ranks (one beam per GPU in the
8-beam case); every rank accumulates uint8 indicator counts for its beams
and an RCCL all-reduce(sum) over xGMI adds them (messages of N and N/2+1
bytes); rank 0 thresholds and writes the sample mask ("#0 1" + one int per
line) and the birdie list ("%.9f\\t%.6f" centre/width of each masked run).
"""
from __future__ import annotations

from typing import List, Sequence

import torch

from .. import _C
from .. import ops
from ..parallel import dist as pdist


def _beam_trial(path: str, device: torch.device):
    fb = _C.Filterbank.from_file(path)
    hdr = fb.header
    dms = _C.generate_dm_list(0.0, 0.0, fb.tsamp, 0.4, fb.fch1, fb.foff, fb.nchans, 1.1)
    g = _C.DedispGeometry.make(hdr, fb.nsamps, dms, [])
    s = torch.cuda.current_stream().cuda_stream
    dfb = _C.DeviceFilterbank(g, s)
    packed = torch.from_numpy(fb.data().copy()).to(device)
    dfb.load_packed_device(packed.data_ptr())
    dd = _C.Dedisperser(dfb, s)
    stride = _C.Dedisperser.row_stride(g.out_nsamps)
    trial = torch.empty(stride, dtype=torch.uint8, device=device)
    dd.run(0, 1, trial.data_ptr(), stride, _C.DedispKernel.Direct)
    return trial, int(g.out_nsamps), float(fb.tsamp)


def run_coincidencer(filterbanks: Sequence[str], samp_out: str = "rfi.eb_mask", spec_out: str = "birdies.txt",
                     thresh: float = 4.0, beam_thresh: int = 4) -> dict:
    if len(filterbanks) > 255:
        # the per-sample beam counts are uint8 (count_above / the RCCL sum)
        raise ValueError(f"{len(filterbanks)} beams: the coincidencer counts beams in uint8, at most 255")
    ctx = pdist.init()
    dev = ctx.device
    mine = [f for i, f in enumerate(filterbanks) if i % ctx.world_size == ctx.rank]
    size = None
    tsamp = None
    tcount = scount = None
    for path in mine:
        trial, n, ts = _beam_trial(path, dev)
        if size is None:
            size, tsamp = n, ts
            tcount = torch.zeros(n, dtype=torch.uint8, device=dev)
            scount = torch.zeros(n // 2 + 1, dtype=torch.uint8, device=dev)
        if n != size:
            raise ValueError("Not all filterbanks the same length")
        series = torch.empty(n, dtype=torch.float32, device=dev)
        spec = torch.empty(n // 2 + 1, dtype=torch.float32, device=dev)
        _C.coincidencer_beam(trial.data_ptr(), n, ts, series.data_ptr(), spec.data_ptr(),
                             torch.cuda.current_stream().cuda_stream)
        ops.coincidence_counts(series, thresh, tcount)
        ops.coincidence_counts(spec, thresh, scount)
    # every rank needs the common length even if it holds no beam
    n_all = torch.tensor([size or 0], dtype=torch.float64, device=dev)
    size = int(pdist.all_reduce_max_float(float(n_all.item())))
    if tcount is None:
        tcount = torch.zeros(size, dtype=torch.uint8, device=dev)
        scount = torch.zeros(size // 2 + 1, dtype=torch.uint8, device=dev)
    if tsamp is None:
        tsamp = 0.0
    tsamp = pdist.all_reduce_max_float(tsamp)
    pdist.all_reduce_sum(tcount)
    pdist.all_reduce_sum(scount)
    smask = ops.coincidence_mask(tcount, beam_thresh)
    fmask = ops.coincidence_mask(scount, beam_thresh)
    out = {"nsamps": size, "masked_samples": int((smask == 0).sum()), "masked_bins": int((fmask == 0).sum())}
    if ctx.is_root:
        bin_width = 1.0 / float(torch.tensor(size * tsamp, dtype=torch.float32))
        hs = smask.to(torch.float32).cpu().contiguous()
        hf = fmask.to(torch.float32).cpu().contiguous()
        _C.write_samp_mask_ptr(hs.data_ptr(), hs.numel(), samp_out)
        _C.write_birdie_list_ptr(hf.data_ptr(), hf.numel(), bin_width, spec_out)
    return out


def main(argv: List[str] = None) -> int:
    import sys

    argv = list(sys.argv if argv is None else argv)
    ok, exit_now, a = _C.parse_coincidencer_cmdline(argv)
    if not ok:
        return 1
    if exit_now:
        return 0
    run_coincidencer(a.filterbanks, a.samp_outfilename, a.spec_outfilename, a.threshold, a.beam_threshold)
    pdist.shutdown()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
