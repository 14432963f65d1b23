#!/bin/bash
# Kernel trace of a bench run (args after the script name go to bench.py);
# per-step kernel table via tools/step_kernels.py.
set -o pipefail
O=${O:-gpurun_out/r4trace}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o tr -- python3 bench.py --steps 4 --warmup 2 "$@" > $O/bench.log 2>&1 || { echo PROF_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-150
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
cp $T $O/kernel_trace.csv
python3 tools/step_kernels.py $O/kernel_trace.csv --skip 2 --steps 4 --top 16 | tee $O/step_kernels.md
echo DONE
