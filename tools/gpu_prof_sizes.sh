#!/bin/bash
# Kernel-stat profiles of the bench at 2^20 (32 DMs per step), of the
# peak-heavy --signal step at 2^23, and sub-batch A/B at 2^23, under gpurun_out/$1.
set -o pipefail
O=gpurun_out/${1:-profsizes}
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
prof() {  # tag, bench args...
  local tag=$1; shift
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/$tag -o run -- python3 $R/bench.py "$@" > $R/$O/$tag.log 2>&1) || { echo PROF_FAIL_$tag; tail -20 $O/$tag.log; return 1; }
  python3 tools/step_kernels.py $O/$tag/run_kernel_trace.csv --skip 1 --steps 3 > $O/$tag.md 2>&1
  head -16 $O/$tag.md
}
prof k20 --log2n 20 --dms-per-gpu 32 --steps 4 --warmup 1 && \
prof sig23 --peak-heavy --steps 4 --warmup 1 && \
for sb in 0 256 128; do
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --sub-batch $sb > $O/sb$sb.log 2>&1 || { echo SB_FAIL; exit 1; }
  echo "sub-batch $sb: $(grep '^{"metric"' $O/sb$sb.log | cut -c80-140)"
done
