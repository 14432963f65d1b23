#!/bin/bash
# End-of-session check of the tree: GPU suite, smoke, bench, config 4.
set -o pipefail
O=gpurun_out/r3final3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 280 --timeout-method thread tests/ > $O/pytest_gpu.log 2>&1 \
  || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_default.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench_default.log; exit 1; }
grep '^{"metric"' $O/bench_default.log | cut -c1-200
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-200
timeout -k 10 400 python3 tools/baseline_configs.py --configs 4 --sky single --workdir /tmp/cfg --out $O/c4.jsonl > $O/c4.log 2>&1 || { echo C4_FAIL; tail -20 $O/c4.log; exit 1; }
cut -c1-330 $O/c4.jsonl
echo DONE
