#!/bin/bash
# Dedisperser plan-table host cost; peak-heavy bench kernel trace.
set -o pipefail
O=gpurun_out/r3sig
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/expt/dedisp_setup_timing.py > $O/dd_setup.log 2>&1 || { echo DD_FAIL; tail -20 $O/dd_setup.log; exit 1; }
tail -1 $O/dd_setup.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o sig -- python3 bench.py --signal --steps 3 --warmup 1 > $O/sig.log 2>&1 || { echo PROF_FAIL; tail -20 $O/sig.log; exit 1; }
grep '^{"metric"' $O/sig.log | cut -c1-200
echo DONE
