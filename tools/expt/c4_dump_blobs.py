#!/usr/bin/env python3
"""Config 4 (Python driver) with the candidate blobs that go into the global
distillation saved to --out (one file per rank blob), so the host-side
merge / distillation / scoring can be timed and profiled on any machine:
    python tools/expt/c4_dump_blobs.py --out gpurun_out/c4blobs
    python tools/expt/gds_bench.py gpurun_out/c4blobs"""
import argparse
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

import baseline_configs as bc  # noqa: E402
from peasoup_amd.models import search  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--out", required=True)
ap.add_argument("--ndm", type=int, default=2000)
ap.add_argument("--log2n", type=int, default=20)
ap.add_argument("--workdir", default="/tmp/cfg")
ap.add_argument("--sky", default="multi")
a = ap.parse_args()
a.native = False
os.makedirs(a.workdir, exist_ok=True)
os.makedirs(a.out, exist_ok=True)
orig = search._C.merge_candidate_blobs


def keep(blobs, args, header):
    import json

    for i, b in enumerate(blobs):
        with open(os.path.join(a.out, f"blob_{i}.bin"), "wb") as f:
            f.write(bytes(b))
    with open(os.path.join(a.out, "header.json"), "w") as f:
        json.dump({k: v for k, v in dict(header).items()}, f)
    with open(os.path.join(a.out, "args.json"), "w") as f:
        json.dump({"dm_end": args.dm_end, "acc_start": args.acc_start, "acc_end": args.acc_end,
                   "nharmonics": args.nharmonics, "limit": args.limit}, f)
    return orig(blobs, args, header)


search._C.merge_candidate_blobs = keep
rec = bc.config45(a, 0, 4)
print(rec["timers_s"], rec["candidates"])
