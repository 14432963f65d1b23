#!/bin/bash
# Session-2 re-entry check: GPU suite, noise bench, pass-A phase split.
set -o pipefail
O=gpurun_out/r3s2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 280 --timeout-method thread tests/ > $O/pytest_gpu.log 2>&1 \
  || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-400
timeout -k 10 200 python -u tools/expt/passa_phases.py --extra 0 > $O/passa_phases.txt 2>&1 || { echo PHASES_FAIL; tail -20 $O/passa_phases.txt; exit 1; }
cat $O/passa_phases.txt
echo DONE
