#!/usr/bin/env python3
"""Host cost of the global candidate merge (deserialise, DM sort, DM +
harmonic distillation, scoring) on blobs saved by c4_dump_blobs.py."""
import glob
import json
import os
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, REPO)
from peasoup_amd import _C  # noqa: E402

d = sys.argv[1]
blobs = [open(f, "rb").read() for f in sorted(glob.glob(os.path.join(d, "blob_*.bin")))]
hdr = json.load(open(os.path.join(d, "header.json")))
a = json.load(open(os.path.join(d, "args.json")))
argv = ["peasoup", "-i", "x.fil", "--dm_end", f"{a['dm_end']:.3f}", "--acc_start", str(a["acc_start"]),
        "--acc_end", str(a["acc_end"]), "-n", str(a["nharmonics"]), "--limit", str(a["limit"])]
ok, _, args = _C.parse_cmdline(argv)
n_in = sum(len(_C.deserialize_candidates(b)) for b in blobs)
for rep in range(3):
    t = time.perf_counter()
    out = _C.merge_candidate_blobs(blobs, args, hdr)
    print(json.dumps({"candidates_in": n_in, "out": len(out), "blob_mb": round(sum(map(len, blobs)) / 1e6, 2),
                      "merge_s": round(time.perf_counter() - t, 4)}))

# the writers on the merged list (candidates.peasoup; overview.xml's candidate section)
import tempfile  # noqa: E402

out.truncate(max(0, args.limit))
with tempfile.TemporaryDirectory() as td:
    for rep in range(2):
        t = time.perf_counter()
        bm = _C.write_candidates_binary(td, out, "candidates.peasoup")
        t1 = time.perf_counter()
        _C.write_overview(os.path.join(td, "overview.xml"), args, hdr, [0.0], [0.0], [], out, bm, {}, {})
        t2 = time.perf_counter()
        print(json.dumps({"write_binary_s": round(t1 - t, 4), "overview_s": round(t2 - t1, 4),
                          "bytes": os.path.getsize(os.path.join(td, "candidates.peasoup"))}))
