"""Diagnostic: resident-plan chunked dedispersion vs per-DM on-the-fly plan on
the config-4 filterbank; byte-compares dedispersed trials and candidates."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
import baseline_configs as bc  # noqa: E402
from peasoup_amd import _C  # noqa: E402
from peasoup_amd.models.search import RankSearcher, load_packed_for_rank  # noqa: E402
from peasoup_amd.parallel import dist as pdist  # noqa: E402


class A:
    workdir = "/tmp/cfgs"
    log2n = 20
    ndm = 2000


def main():
    os.makedirs(A.workdir, exist_ok=True)
    ctx = pdist.init()
    path = bc._make_fb(A, ctx)
    argv = ["peasoup", "-i", path, "-o", "/tmp/cfgs/diag", "--dm_end", f"{bc._dm_end_for(A.ndm):.3f}",
            "--acc_start", "-500", "--acc_end", "500", "-n", "3", "--limit", "1000"]
    ok, _, args = _C.parse_cmdline(argv)
    header, packed, nsamps = load_packed_for_rank(args.infilename, ctx)
    rs = RankSearcher(args, header, packed, nsamps)
    ndm = len(rs.dm_list)
    rsz = rs.row_stride
    T = 32
    bad = 0
    a = torch.empty(T * rsz, dtype=torch.uint8, device="cuda")
    b = torch.empty(T * rsz, dtype=torch.uint8, device="cuda")
    t0 = time.perf_counter()
    for d0 in range(0, ndm, T):
        d1 = min(ndm, d0 + T)
        rs.dedisperser.run(d0, d1, a.data_ptr(), rsz, _C.DedispKernel.Mfma)
        for d in range(d0, d1):
            rs.dedisperser.run(d, d + 1, b.data_ptr() + (d - d0) * rsz, rsz, _C.DedispKernel.Mfma)
        torch.cuda.synchronize()
        n = rs.geom.out_nsamps
        A_ = a[: (d1 - d0) * rsz].view(d1 - d0, rsz)[:, :n]
        B_ = b[: (d1 - d0) * rsz].view(d1 - d0, rsz)[:, :n]
        neq = (A_ != B_).any(dim=1)
        if bool(neq.any()):
            bad += int(neq.sum())
            if bad < 10:
                print("mismatch rows", d0 + torch.nonzero(neq).flatten().cpu().numpy()[:8], flush=True)
    print("dedisp compare", time.perf_counter() - t0, "bad rows", bad, flush=True)

    def key(c):
        return (c.dm_idx, round(c.freq, 6), round(c.acc, 3), round(c.snr, 3), c.nh)

    import peasoup_amd.models.search as S

    def dm0(v):
        return sorted(key(c) for c in v if c.dm_idx == 0)

    res = {}
    S._SYNC_DEDISP = True
    r = RankSearcher(args, header, packed, nsamps)
    res["fresh_sync"] = r.search(range(64))
    print("fresh_sync counters", dict(r.engine.counters()), flush=True)
    S._SYNC_DEDISP = False
    r = RankSearcher(args, header, packed, nsamps)
    tr = r.dedisperse(0, 1)
    torch.cuda.synchronize()
    res["fresh_oldpath"] = r.engine.search_trial(tr.data_ptr(), r.geom.out_nsamps, r.dm_list[0], 0, r.accel_list(r.dm_list[0]))
    print("fresh_oldpath counters", dict(r.engine.counters()), flush=True)
    for i in range(3):
        r = RankSearcher(args, header, packed, nsamps)
        res[f"fresh_overlap{i}"] = r.search(range(64))
        print("fresh_overlap counters", dict(r.engine.counters()), flush=True)
    t_new = 0.0
    new = rs.search(range(ndm))
    new = rs.search(range(ndm))
    old = []
    t0 = time.perf_counter()
    for d in range(ndm):
        tr = rs.dedisperse(d, d + 1)
        old.extend(rs.engine.search_trial(tr.data_ptr(), rs.geom.out_nsamps, rs.dm_list[d], d, rs.accel_list(rs.dm_list[d])))
    t_old = time.perf_counter() - t0
    kn, ko = sorted(map(key, new)), sorted(map(key, old))
    for nm, v in res.items():
        print(nm, "dm0 equal old", dm0(v) == dm0(old), len(dm0(v)), len(dm0(old)), flush=True)
    print("cands new", len(kn), t_new, "old", len(ko), t_old, "equal", kn == ko, flush=True)
    if kn != ko:
        sn, so = set(kn), set(ko)
        print("only new", sorted(sn - so)[:10])
        print("only old", sorted(so - sn)[:10])
        dn = {}
        for k in sn - so:
            dn[k[0]] = dn.get(k[0], 0) + 1
        print("dm_idx of extra new", sorted(dn.items())[:40])


if __name__ == "__main__":
    main()
