#!/usr/bin/env python3
"""Antenna delay map from a PSRDADA voltage file (the reference's `accmap`,
src/accmap.cpp:12-32, which hard-codes a /lustre path and does not build):
extract one channel of every antenna and find the pairwise delays by FFT
cross-correlation on the GPU (models/correlator.py, DelayFinder).

    python tools/peasoup_accmap.py obs.dada --channel 0 --size 65536 --max-delay 2048
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("dada")
    ap.add_argument("--channel", type=int, default=0)
    ap.add_argument("--size", type=int, default=65536)
    ap.add_argument("--offset", type=int, default=0)
    ap.add_argument("--max-delay", type=int, default=2048)
    a = ap.parse_args(argv)
    from peasoup_amd.models.correlator import find_delays
    from peasoup_amd.utils import dada

    hdr = dada.read_header(a.dada)
    arrays = dada.extract_channel(a.dada, a.channel, a.size, a.offset, hdr=hdr)
    delays = find_delays(arrays, a.max_delay)
    print(json.dumps({"source": hdr.get("source_name", ""), "nant": int(hdr["nant"]), "channel": a.channel,
                      "delays": {f"{i}-{j}": d for (i, j), d in sorted(delays.items())}}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
