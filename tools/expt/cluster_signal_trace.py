#!/usr/bin/env python3
"""Per-phase wall time of the large peak-clustering kernel on the peak-heavy
bench data (bench.py --signal's sky): one DM chunk searched with the
kernel's trace buffer set; the last batch's large-kernel segments are
reported (crossings, chunks, phase times)."""
import argparse
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, REPO)
from peasoup_amd import _C  # noqa: E402
from peasoup_amd.models.search import RankSearcher  # noqa: E402
from peasoup_amd.utils import synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=23)
    ap.add_argument("--dms", type=int, default=8)
    ap.add_argument("--rfi-amp", type=float, default=0.05)
    a = ap.parse_args()
    n = 1 << a.log2n
    nchans, tsamp, fch1 = 1024, 64e-6, 1550.0
    foff = -400.0 / nchans
    args = _C.CmdLineOptions()
    args.infilename, args.outdir = "synthetic", "/tmp/peasoup_cltrace"
    args.dm_start, args.dm_end = 0.0, 5.0
    args.acc_start, args.acc_end = -500.0, 500.0
    args.nharmonics, args.size = 3, n
    dms = _C.generate_dm_list(0.0, 5.0, tsamp, 64.0, fch1, foff, nchans, 1.1)
    nsamps = n + _C.compute_max_delay(dms, _C.generate_delay_table(nchans, tsamp, fch1, foff)) + 4096
    header = {"source_name": "synthetic", "tsamp": tsamp, "fch1": fch1, "foff": foff, "nchans": nchans, "nbits": 2,
              "nifs": 1, "data_type": 1, "tstart": 60000.0, "nsamples": nsamps}
    sky = [synthetic.PulsarSpec(period=0.00731, dm=2.0, duty=0.05, amplitude=0.05, accel=120.0),
           synthetic.PulsarSpec(period=0.1532, dm=1.0, duty=0.04, amplitude=0.08, accel=-40.0),
           synthetic.PulsarSpec(period=0.02, dm=0.0, duty=0.02, amplitude=a.rfi_amp),
           synthetic.PulsarSpec(period=0.06, dm=0.0, duty=0.03, amplitude=0.67 * a.rfi_amp)]
    packed = synthetic.generate_packed_torch(nsamps, header, sky, seed=1234, device="cuda")
    os.environ.setdefault("PSOUP_ENGINES", "1")
    rs = RankSearcher(args, header, packed, nsamps)
    del packed
    rs.search(range(0, a.dms), chunk=a.dms)  # warm
    torch.cuda.synchronize()
    maxseg = 65536
    tr = torch.zeros(maxseg * 8, dtype=torch.int64, device="cuda")
    _C.kernels.peak_cluster_set_trace(tr.data_ptr())
    rs.search(range(0, a.dms), chunk=a.dms)
    torch.cuda.synchronize()
    _C.kernels.peak_cluster_set_trace(0)
    t = tr.view(maxseg, 8).cpu().numpy()
    ok = np.nonzero(t[:, 7] > 0)[0]
    d = np.diff(t[ok], axis=1) * 10.0  # 100 MHz ticks -> ns
    names = ["sort", "gather", "window", "nextsurv", "next+runs", "chains", "compact"]
    print(f"large-kernel segments in the last batch: {len(ok)} (ids {ok[:8].tolist()} ...)")
    if len(ok):
        print("per-segment wall (us): " + ", ".join(f"{nm} {v / 1e3:.1f}" for nm, v in zip(names, d.mean(axis=0))) +
              f"; total {d.sum(axis=1).mean() / 1e3:.1f}; max total {d.sum(axis=1).max() / 1e3:.1f}")
        span = (t[ok, 7].max() - t[ok, 0].min()) * 10.0 / 1e3
        print(f"kernel span over those segments: {span:.1f} us")
    c = rs.engine.counters() if hasattr(rs.engine, "counters") else {}
    print({k: v for k, v in c.items() if "peak" in k or "clust" in k or "harm" in k})


if __name__ == "__main__":
    main()
