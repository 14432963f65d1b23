#!/bin/bash
set -o pipefail
O=gpurun_out/r3sig
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o sig -- python3 bench.py --signal --steps 3 --warmup 1 > $O/sig.log 2>&1 || { echo SIG_FAIL; tail -20 $O/sig.log; exit 1; }
grep '^{"metric"' $O/sig.log | cut -c1-200
echo DONE
