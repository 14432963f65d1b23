#!/usr/bin/env python3
"""Peak-clustering kernels on RFI-like segments: nseg segments of ~n
threshold crossings each (dense runs around periodic spikes plus scattered
noise crossings), records shuffled like the harmonic kernel's atomics emit
them.  Prints the time of kern::peak_cluster_batch and, with --trace, the
large kernel's per-phase shader-clock times."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from peasoup_amd import _C  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
from test_peakcluster_gpu import chunked_records  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nseg", type=int, default=2048)
    ap.add_argument("--n", type=int, default=4200)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--trace", action="store_true", help="per-phase wall time of the large cluster kernel")
    ap.add_argument("--dense", action="store_true",
                    help="RFI-like segments: runs of 100-500 consecutive bins (acceleration-smeared harmonics), "
                         "S/N a smooth bump plus noise")
    a = ap.parse_args()
    K = _C.kernels
    rng = np.random.default_rng(1)
    segs = {}
    for sgi in range(a.nseg):
        n = int(rng.integers(a.n // 2, a.n * 3 // 2))
        if a.dense:
            parts, snrs, tot_ = [], [], 0
            while tot_ < n:
                L = int(rng.integers(100, 500))
                c = int(rng.integers(0, (1 << 22) - L))
                parts.append(np.arange(c, c + L))
                x = np.linspace(-1, 1, L)
                snrs.append(9.5 + 30.0 * np.exp(-3 * x * x) * rng.uniform(0.5, 1.5) + rng.normal(0, 1.5, L))
                tot_ += L
            idx, first = np.unique(np.concatenate(parts), return_index=True)
            snr = np.maximum(np.concatenate(snrs)[first], 9.01)
            idx, snr = idx[:n].astype(np.int32), snr[:n].astype(np.float32)
        else:
            spikes = rng.choice(1 << 22, max(1, n // 40), replace=False)
            idx = np.unique((spikes[:, None] + np.arange(-20, 20)[None, :]).reshape(-1))
            idx = idx[idx >= 0][:n].astype(np.int32)
            snr = (9.0 + 30.0 * rng.random(idx.size)).astype(np.float32)
        segs[sgi] = (idx, snr)
    allr = chunked_records(segs, rng)  # chunk descriptors + crossings, as the harmonic kernel emits them
    n = len(allr)
    dev = "cuda"
    cap = n + 100
    peaks = torch.from_numpy(allr.reshape(-1).view(np.int32).copy()).to(dev)
    count = torch.tensor([n], dtype=torch.int32, device=dev)
    work = torch.empty(5 * a.nseg, dtype=torch.int32, device=dev)
    srt = torch.empty(4 * cap, dtype=torch.int32, device=dev)
    out = torch.empty(2 * cap, dtype=torch.int32, device=dev)
    tab = torch.empty(2 * a.nseg, dtype=torch.int32, device=dev)
    tot = torch.zeros(1, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    run = lambda: K.peak_cluster_batch(peaks.data_ptr(), count.data_ptr(), cap, a.nseg, 30, work.data_ptr(),
                                       srt.data_ptr(), out.data_ptr(), tab.data_ptr(), tot.data_ptr(), s)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    print(f"{'dense' if a.dense else 'spiky'} records={n} segments={a.nseg}: "
          f"{e0.elapsed_time(e1) / a.reps:.3f} ms per batch", flush=True)
    if a.trace:
        tr = torch.zeros(a.nseg * 8, dtype=torch.int64, device=dev)
        K.peak_cluster_set_trace(tr.data_ptr())
        run()
        torch.cuda.synchronize()
        K.peak_cluster_set_trace(0)
        t = tr.view(a.nseg, 8).cpu().numpy()
        ok = t[:, 7] > 0  # segments the large kernel clustered
        d = np.diff(t[ok], axis=1) * 10.0  # 100 MHz ticks -> ns
        names = ["sort", "gather", "window", "nextsurv", "next+runs", "chains", "compact"]
        print(f"large-kernel segments: {ok.sum()}, per-segment wall (us): " +
              ", ".join(f"{nm} {v / 1e3:.1f}" for nm, v in zip(names, d.mean(axis=0))) +
              f"; total {d.sum(axis=1).mean() / 1e3:.1f}", flush=True)


if __name__ == "__main__":
    main()
