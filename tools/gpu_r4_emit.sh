#!/bin/bash
# One atomic per wave for all harmonic levels; native merge; cluster PMC.
set -o pipefail
O=gpurun_out/r4emit
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_peakcluster_gpu.py tests/test_harmdistill_gpu.py tests/test_kernels_gpu.py -k "harmonic or cluster or distill" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --signal > $O/bench_signal.log 2>&1 || { echo SIG_FAIL; tail -20 $O/bench_signal.log; exit 1; }
grep '^{"metric"' $O/bench_signal.log | cut -c1-120; grep '^{"metric"' $O/bench_signal.log | grep -o '"peaks_per_dm.*'
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-120
bash tools/gpu_r4_clpmc.sh
