#!/usr/bin/env python3
"""Where the multi-beam coincidencer's time goes on one beam of the config-5
filterbank (2^20 + 64k samples x 1024 channels, 2-bit): file read, upload,
DM-0 dedispersion, whitening + spectrum (first and second call), counts, mask
writers.  python tools/expt/coinc_timing.py FIL"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main():
    from peasoup_amd import _C, ops
    from peasoup_amd.models import coincidencer as co

    path = sys.argv[1]
    dev = torch.device("cuda")
    torch.zeros(1, device=dev)
    torch.cuda.synchronize()
    T = {}
    t = time.perf_counter()
    trial, n, ts = co._beam_trial(path, dev)
    torch.cuda.synchronize()
    T["read+upload+dedisperse"] = time.perf_counter() - t
    for rep in range(2):
        series = torch.empty(n, dtype=torch.float32, device=dev)
        spec = torch.empty(n // 2 + 1, dtype=torch.float32, device=dev)
        t = time.perf_counter()
        _C.coincidencer_beam(trial.data_ptr(), n, ts, series.data_ptr(), spec.data_ptr(),
                             torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        T[f"coincidencer_beam #{rep + 1} (n={n})"] = time.perf_counter() - t
    tc = torch.zeros(n, dtype=torch.uint8, device=dev)
    sc = torch.zeros(n // 2 + 1, dtype=torch.uint8, device=dev)
    t = time.perf_counter()
    ops.coincidence_counts(series, 4.0, tc)
    ops.coincidence_counts(spec, 4.0, sc)
    sm = ops.coincidence_mask(tc, 1)
    fm = ops.coincidence_mask(sc, 1)
    torch.cuda.synchronize()
    T["counts+masks"] = time.perf_counter() - t
    t = time.perf_counter()
    hs, hf = sm.to(torch.float32).cpu().contiguous(), fm.to(torch.float32).cpu().contiguous()
    _C.write_samp_mask_ptr(hs.data_ptr(), hs.numel(), "/tmp/ct_mask.txt")
    _C.write_birdie_list_ptr(hf.data_ptr(), hf.numel(), 1.0 / (n * ts), "/tmp/ct_birdies.txt")
    T["write mask + birdies"] = time.perf_counter() - t
    for k, v in T.items():
        print(f"{k:40s} {v * 1e3:9.1f} ms", flush=True)


if __name__ == "__main__":
    main()
