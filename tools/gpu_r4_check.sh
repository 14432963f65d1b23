#!/bin/bash
# Screen tests + bench (noise, --signal) after a harmonic-kernel change.
set -o pipefail
O=gpurun_out/r4check
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_screen_gpu.py tests/test_harmdistill_gpu.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-200
timeout -k 10 300 python -u bench.py --signal --steps 4 --warmup 2 > $O/bench_sig.log 2>&1 || { echo BENCH_SIG_FAIL; tail -20 $O/bench_sig.log; exit 1; }
grep '^{"metric"' $O/bench_sig.log | cut -c1-200
timeout -k 10 300 python -u bench.py --log2n 20 --dms-per-gpu 32 --steps 20 --warmup 3 > $O/bench20.log 2>&1 || { echo BENCH20_FAIL; tail -20 $O/bench20.log; exit 1; }
grep '^{"metric"' $O/bench20.log | cut -c1-200
echo DONE
