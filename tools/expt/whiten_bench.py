#!/usr/bin/env python3
"""Isolated cost of the per-DM work around the acceleration trials at the
config-4 size (2^20-point series, 1024-channel 2-bit filterbank): batched
whitening (``SearchEngine.prepare``: u8 load/pad, forward real FFT, running
medians, dereddening, inverse FFT, statistics) and one full DM chunk search,
each timed alone on one engine with HIP events.

    python tools/expt/whiten_bench.py [--log2n 20] [--dms 32] [--reps 5]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=20)
    ap.add_argument("--dms", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--acc", type=float, default=500.0)
    a = ap.parse_args()
    from peasoup_amd import _C
    from peasoup_amd.models.search import RankSearcher
    from peasoup_amd.parallel import dist as pdist

    ctx = pdist.init()
    dev = ctx.device
    n = 1 << a.log2n
    nchans, tsamp, fch1, foff = 1024, 64e-6, 1550.0, -400.0 / 1024
    args = _C.CmdLineOptions()
    args.infilename = "synthetic"
    args.outdir = "/tmp/whiten_bench"
    args.dm_end = 150.0
    args.acc_start, args.acc_end = -a.acc, a.acc
    args.nharmonics = 3
    args.size = n
    args.engines_per_gpu = 1
    dms = _C.generate_dm_list(0.0, args.dm_end, tsamp, 64.0, fch1, foff, nchans, 1.1)
    delays = _C.generate_delay_table(nchans, tsamp, fch1, foff)
    nsamps = n + _C.compute_max_delay(dms, delays) + 4096
    header = {"source_name": "synthetic", "tsamp": tsamp, "fch1": fch1, "foff": foff, "nchans": nchans,
              "nbits": 2, "nifs": 1, "data_type": 1, "tstart": 60000.0, "nsamples": nsamps}
    packed = torch.empty(nsamps * nchans * 2 // 8, dtype=torch.uint8, device=dev)
    packed.random_(0, 256, generator=torch.Generator(device=dev).manual_seed(7))
    rs = RankSearcher(args, header, packed, nsamps)
    del packed
    ndm = min(a.dms, len(rs.dm_list))
    trials = rs.dedisperse(0, ndm)
    torch.cuda.synchronize()
    e = rs.engine
    cnt = min(ndm, e.max_prepare)

    def whiten():
        e.prepare(trials.data_ptr(), rs.row_stride, rs.geom.out_nsamps, cnt)

    whiten()
    _C.stream_synchronize(e.stream)
    t0 = time.perf_counter()
    for _ in range(a.reps):
        whiten()
    _C.stream_synchronize(e.stream)
    tw = (time.perf_counter() - t0) / a.reps
    print(f"whitening batch of {cnt} DMs at 2^{a.log2n}: {tw * 1e3:.3f} ms ({tw * 1e6 / cnt:.1f} us per DM)", flush=True)
    ntr = sum(len(rs.accel_list(rs.dm_list[d])) for d in range(ndm))
    rs.search(range(ndm), chunk=ndm)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        rs.search(range(ndm), chunk=ndm)
    torch.cuda.synchronize()
    ts = (time.perf_counter() - t0) / a.reps
    print(f"search of {ndm} DMs ({ntr} trials): {ts * 1e3:.3f} ms ({ts * 1e6 / ndm:.1f} us per DM, "
          f"{ntr / ts:.0f} trials/s)", flush=True)


if __name__ == "__main__":
    main()
