#!/bin/bash
# Last check of the final tree: smoke() and the default bench.
set -o pipefail
O=gpurun_out/r4last
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-200
echo DONE
