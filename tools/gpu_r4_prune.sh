#!/bin/bash
# After the FFT4 flag prune: kernel tests (all flag sets, no skips), pipeline/model tests,
# short bench; then the async/golden/config script.
set -o pipefail
O=gpurun_out/r4prune
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_kernels_gpu.py > $O/pytest_kernels.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest_kernels.log | head; tail -30 $O/pytest_kernels.log; exit 1; }
tail -1 $O/pytest_kernels.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-200
bash tools/gpu_r4_async.sh
