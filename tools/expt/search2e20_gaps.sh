#!/bin/bash
# Kernel trace of repeated 32-DM chunk searches at 2^20 (config-4 shape): GPU
# busy fraction and idle gaps over the search-only tail of the run.
set -o pipefail
mkdir -p gpurun_out/s20
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s20 -o s --output-format csv -- python3 tools/expt/whiten_bench.py --dms 32 --reps 20 "$@" > gpurun_out/s20/run.txt 2>&1 || { echo FAIL; tail -20 gpurun_out/s20/run.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/s20/run.txt | grep -v rocprofv3
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/s20/s_kernel_trace.csv")))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# the last 40% of the timeline: searches only
t0, t1 = iv[0][0], iv[-1][1]
cut = t0 + 0.6 * (t1 - t0)
print(f"total trace span {(t1 - t0) * 1e-6:.1f} ms; analysing after {(cut - t0) * 1e-6:.1f} ms")
open("gpurun_out/s20/tail.csv", "w").write("Start_Timestamp,End_Timestamp,Kernel_Name\n" + "".join(
    f'{s},{e},"{n}"\n' for s, e, n in iv if s >= cut))
PY
python3 tools/trace_gaps.py gpurun_out/s20/tail.csv
rm -f gpurun_out/s20/s_kernel_trace.csv gpurun_out/s20/tail.csv
