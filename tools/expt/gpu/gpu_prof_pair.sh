#!/bin/bash
# Kernel-trace profiles of the noise and --peak-heavy benches on one box:
# per-step kernel tables (tools/step_kernels.py) and idle gaps
# (tools/trace_gaps.py) under gpurun_out/$1.
set -o pipefail
O=gpurun_out/${1:-profpair}
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for tag in noise sig; do
  extra=""; [ $tag = sig ] && extra="--peak-heavy"
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p_$tag -o run -- python3 $R/bench.py --steps 4 --warmup 1 $extra > $R/$O/p_$tag.log 2>&1) || { echo PROF_FAIL; tail -5 $O/p_$tag.log; exit 1; }
  python3 tools/step_kernels.py $O/p_$tag/run_kernel_trace.csv --skip 1 --steps 3 > $O/k_$tag.md 2>&1
  python3 tools/trace_gaps.py $O/p_$tag/run_kernel_trace.csv > $O/gaps_$tag.txt 2>&1
  head -16 $O/k_$tag.md
  gzip $O/p_$tag/run_kernel_trace.csv
done
