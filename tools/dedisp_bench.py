#!/usr/bin/env python3
"""Dedispersion kernel bench: MFMA one-hot vs packed-byte VALU (and Auto) per
32-DM chunk across a DM list, bit-exactness checked against each other.

    python tools/dedisp_bench.py [--nchans 1024] [--nbits 2] [--log2n 20] [--ndm 2000]
Prints one JSON line per chunk sampled plus a whole-list summary line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, REPO)
from peasoup_amd import _C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nchans", type=int, default=1024)
    ap.add_argument("--nbits", type=int, default=2)
    ap.add_argument("--log2n", type=int, default=20)
    ap.add_argument("--ndm", type=int, default=2000)
    ap.add_argument("--tsamp", type=float, default=64e-6)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--samples", type=int, default=8, help="chunks timed individually")
    a = ap.parse_args()
    fch1, foff = 1550.0, -400.0 / a.nchans
    dm_end = 10.0
    while len(_C.generate_dm_list(0.0, dm_end, a.tsamp, 64.0, fch1, foff, a.nchans, 1.1)) < a.ndm:
        dm_end *= 1.05
    dms = list(_C.generate_dm_list(0.0, dm_end, a.tsamp, 64.0, fch1, foff, a.nchans, 1.1))
    delays = _C.generate_delay_table(a.nchans, a.tsamp, fch1, foff)
    max_delay = _C.compute_max_delay(dms, delays)
    nsamps = (1 << a.log2n) + max_delay + 1024
    hdr = {"source_name": "bench", "tsamp": a.tsamp, "fch1": fch1, "foff": foff, "nchans": a.nchans,
           "nbits": a.nbits, "nifs": 1, "data_type": 1, "tstart": 60000.0, "nsamples": nsamps}
    g = _C.DedispGeometry.make(hdr, nsamps, dms, [])
    s = _C.GpuStream()
    dfb = _C.DeviceFilterbank(g, s.handle)
    packed = torch.randint(0, 256, (nsamps * a.nchans * a.nbits // 8,), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    dfb.load_packed_device(packed.data_ptr())
    s.synchronize()
    del packed
    dd = _C.Dedisperser(dfb, s.handle)
    ndm = len(dms)
    rs = _C.Dedisperser.row_stride(g.out_nsamps)
    T = _C.Dedisperser.tile_dms
    bufs = {k: torch.empty(T * rs, dtype=torch.uint8, device="cuda") for k in ("m", "v", "p")}
    kinds = {"m": _C.DedispKernel.Mfma, "v": _C.DedispKernel.Valu}
    if a.nbits <= 2:
        kinds["p"] = _C.DedispKernel.Packed2  # the 2-bit kernel

    def timed(k, d0, d1, reps):
        e0, e1 = _C.GpuEvent(True), _C.GpuEvent(True)
        dd.run(d0, d1, bufs[k].data_ptr(), rs, kinds[k], s.handle)  # warm (plans)
        e0.record(s.handle)
        for _ in range(reps):
            dd.run(d0, d1, bufs[k].data_ptr(), rs, kinds[k], s.handle)
        e1.record(s.handle)
        e1.synchronize()
        return e0.elapsed_ms(e1) / reps

    starts = sorted({min(ndm - 1, i * ndm // a.samples) // T * T for i in range(a.samples)} |
                    {T * k for k in (1, 4, 8, 12, 16) if T * k < ndm})
    for d0 in starts:
        d1 = min(ndm, d0 + T)
        tm = timed("m", d0, d1, a.reps)
        tv = timed("v", d0, d1, a.reps)
        tp = timed("p", d0, d1, a.reps) if "p" in kinds else None
        s.synchronize()
        n = g.out_nsamps
        view = lambda k: bufs[k][: (d1 - d0) * rs].view(d1 - d0, rs)[:, :n]  # noqa: E731
        same = bool(torch.equal(view("m"), view("v"))) and (tp is None or bool(torch.equal(view("m"), view("p"))))
        print(json.dumps({"d0": d0, "dm": round(dms[d0], 2), "mfma_ms": round(tm, 4), "valu_ms": round(tv, 4),
                          "packed2_ms": round(tp, 4) if tp is not None else None,
                          "auto": "MfmaLds" if dd.mfma_lds_split(d0, d1) > d0 else str(dd.choose(d0, d1)).split(".")[-1],
                          "bit_exact": same,
                          "mfma_steps_per_chan": round(dd.mfma_steps_per_channel(d0, d1), 3)}), flush=True)
    tot = {}
    for k in [x for x in ("m", "v", "p") if x in kinds] + ["auto"]:
        e0, e1 = _C.GpuEvent(True), _C.GpuEvent(True)
        e0.record(s.handle)
        for d0 in range(0, ndm, T):
            kind = _C.DedispKernel.Auto if k == "auto" else kinds[k]
            dd.run(d0, min(ndm, d0 + T), bufs["m"].data_ptr(), rs, kind, s.handle)
        e1.record(s.handle)
        e1.synchronize()
        tot[k] = round(e0.elapsed_ms(e1), 2)
    # the whole list in one Auto call (the hybrid split: MFMA tiles, then VALU)
    whole = torch.empty(ndm * rs, dtype=torch.uint8, device="cuda")
    dd.run(0, ndm, whole.data_ptr(), rs, _C.DedispKernel.Auto, s.handle)
    e0, e1 = _C.GpuEvent(True), _C.GpuEvent(True)
    e0.record(s.handle)
    dd.run(0, ndm, whole.data_ptr(), rs, _C.DedispKernel.Auto, s.handle)
    e1.record(s.handle)
    e1.synchronize()
    tot["auto_whole"] = round(e0.elapsed_ms(e1), 2)
    e0.record(s.handle)
    dd.run(0, ndm, whole.data_ptr(), rs, _C.DedispKernel.Valu, s.handle)
    e1.record(s.handle)
    e1.synchronize()
    tot["valu_whole"] = round(e0.elapsed_ms(e1), 2)
    if "p" in kinds:
        e0.record(s.handle)
        dd.run(0, ndm, whole.data_ptr(), rs, kinds["p"], s.handle)
        e1.record(s.handle)
        e1.synchronize()
        tot["packed2_whole"] = round(e0.elapsed_ms(e1), 2)
    tot["split_dm"] = dd.mfma_lds_split(0, ndm)
    gsamp = ndm * g.out_nsamps * g.nactive / 1e9
    print(json.dumps({"ndm": ndm, "nchans": a.nchans, "nbits": a.nbits, "out_nsamps": g.out_nsamps,
                      "total_ms": {"mfma": tot["m"], "valu": tot["v"], "packed2": tot.get("p"), "auto": tot["auto"],
                                   "auto_whole_list": tot["auto_whole"], "valu_whole_list": tot["valu_whole"],
                                   "packed2_whole_list": tot.get("packed2_whole")},
                      "mfma_lds_split_dm_index": tot["split_dm"],
                      "G_chan_samples_per_s": {k: round(gsamp / (v * 1e-3), 1) for k, v in
                                               (("mfma", tot["m"]), ("valu", tot["v"]), ("packed2", tot.get("p")),
                                                ("auto", tot["auto"])) if v}}))


if __name__ == "__main__":
    main()
