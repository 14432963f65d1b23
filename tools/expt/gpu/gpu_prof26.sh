#!/bin/bash
# rocprofv3 kernel table of one 2^26 bench step (external-row FFT path).
set -o pipefail
O=gpurun_out/${1:-prof26}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O -o b --output-format csv -- python3 bench.py --log2n 26 --dms-per-gpu 1 --steps 1 --warmup 1 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
rm -f $O/b_kernel_trace.csv
python3 tools/prof_summary.py $O/b_kernel_stats.csv 16
