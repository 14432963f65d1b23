"""Diagnose the config-3 host crash: the 2^23 accel search of a bright
pulsar (peak-heavy) with host_threads 1 and 4, and the peak counters."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from peasoup_amd import _C  # noqa: E402

ht = int(sys.argv[1])
n = 1 << 23
nsamps = n + 1000
rng = np.random.default_rng(1)
t = np.arange(nsamps) * 64e-6
x = rng.normal(128, 8, nsamps) + 3.0 * (np.minimum((t / 0.0123456) % 1.0, 1 - (t / 0.0123456) % 1.0) < 0.02)
trial = torch.from_numpy(np.clip(np.rint(x), 0, 255).astype(np.uint8)).cuda()
plan = _C.AccelPlan(-500.0, 500.0, 1.1, 64.0, n, 64e-6, 1350.0, -0.39, _C.AccelConvention.Legacy)
accs = list(plan.generate(0.0))
print("accs", len(accs), flush=True)
p = _C.SearchParams()
p.fft_size, p.tsamp, p.nharmonics, p.host_threads = n, 64e-6, 3, ht
eng = _C.SearchEngine(p, torch.cuda.current_stream().cuda_stream)
for r in range(2):
    c = eng.search_trial(trial.data_ptr(), nsamps, 0.0, 0, accs)
    torch.cuda.synchronize()
    print("rep", r, "cands", len(c), dict(eng.counters()), flush=True)
