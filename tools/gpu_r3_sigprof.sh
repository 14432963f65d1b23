#!/bin/bash
# kernel stats of the peak-heavy bench (GPU clustering cost)
set -o pipefail
O=${O:-gpurun_out/r3f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sig -o sig -- python3 bench.py --steps 3 --warmup 1 --signal --rfi-amp ${AMP:-0} > $O/prof_sig.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof_sig.log; exit 1; }
grep '^{"metric"' $O/prof_sig.log | cut -c1-200
head -25 $(find $O/prof_sig -name "*kernel_stats.csv") | cut -d, -f1-8
