#!/usr/bin/env python3
"""Replays the peak clustering kernels on one real batch of peak records
(dumped by the engine with PSOUP_DUMP_PEAKS=file, e.g. from bench.py
--peak-heavy): time per batch, segment-size histogram, and with --trace the
large kernel's per-phase wall time."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from peasoup_amd import _C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--trace", action="store_true")
    a = ap.parse_args()
    K = _C.kernels
    raw = np.fromfile(a.dump, dtype=np.uint32)
    nseg, gap, n = (int(x) for x in raw[:3])
    recs = raw[3:3 + 3 * n].reshape(n, 3)
    chunk = (recs[:, 0] & 0x80000000) != 0  # kPeakChunk descriptors
    seg = recs[chunk, 0] & 0xFFFF
    cnt = (recs[chunk, 0] >> 16) & 0x7F
    per = np.bincount(seg, weights=cnt, minlength=nseg)
    print(f"nseg {nseg} gap {gap} records {n} chunks {int(chunk.sum())} crossings {int(cnt.sum())} "
          f"({cnt.mean() if cnt.size else 0:.1f} per chunk); segments > 4096: {(per > 4096).sum()}, "
          f"> 14000: {(per > 14000).sum()}, max {int(per.max())}, mean of >4096: {per[per > 4096].mean() if (per > 4096).any() else 0:.0f}")
    dev = "cuda"
    cap = n + 100
    peaks = torch.from_numpy(recs.reshape(-1).view(np.int32).copy()).to(dev)
    count = torch.tensor([n], dtype=torch.int32, device=dev)
    work = torch.empty(5 * nseg, dtype=torch.int32, device=dev)
    srt = torch.empty(4 * cap, dtype=torch.int32, device=dev)
    out = torch.empty(2 * cap, dtype=torch.int32, device=dev)
    tab = torch.empty(2 * nseg, dtype=torch.int32, device=dev)
    tot = torch.zeros(1, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    run = lambda: K.peak_cluster_batch(peaks.data_ptr(), count.data_ptr(), cap, nseg, gap, work.data_ptr(),
                                       srt.data_ptr(), out.data_ptr(), tab.data_ptr(), tot.data_ptr(), s)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    print(f"peak_cluster_batch: {e0.elapsed_time(e1) / a.reps:.3f} ms per batch; cluster peaks {int(tot.item())}")
    if a.trace:
        tr = torch.zeros(nseg * 8, dtype=torch.int64, device=dev)
        K.peak_cluster_set_trace(tr.data_ptr())
        run()
        torch.cuda.synchronize()
        K.peak_cluster_set_trace(0)
        t = tr.view(nseg, 8).cpu().numpy()
        ok = t[:, 7] > 0
        d = np.diff(t[ok], axis=1) * 10.0
        names = ["sort", "gather", "window", "nextsurv", "next+runs", "chains", "compact"]
        print(f"large-kernel segments {ok.sum()}: per-segment wall (us) " +
              ", ".join(f"{nm} {v / 1e3:.1f}" for nm, v in zip(names, d.mean(axis=0))) +
              f"; total {d.sum(axis=1).mean() / 1e3:.1f} (max {d.sum(axis=1).max() / 1e3:.1f}); "
              f"launch span {(t[ok, 7].max() - t[ok, 0].min()) * 10.0 / 1e3:.1f} us")


if __name__ == "__main__":
    main()
