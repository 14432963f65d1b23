#!/bin/bash
# Kernel trace of the peak-heavy bench (GPU distillation on): per-kernel time
# and the GPU busy fraction of the timed steps.
set -o pipefail
O=gpurun_out/r4sig
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o sig -- python3 bench.py --signal --steps 4 --warmup 2 > $O/sig.log 2>&1 || { echo SIG_FAIL; tail -20 $O/sig.log; exit 1; }
grep '^{"metric"' $O/sig.log | cut -c1-200
K=$(find $O/prof -name "*kernel_stats.csv" | head -1)
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/prof_summary.py $K 22 > $O/kernel_stats.md
cat $O/kernel_stats.md
python3 tools/trace_gaps.py $T --after-ms ${AFTER:-0} > $O/gaps.txt
cat $O/gaps.txt
cp $T $O/kernel_trace.csv
echo DONE
