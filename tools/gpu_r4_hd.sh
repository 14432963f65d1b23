#!/bin/bash
# GPU harmonic distillation: exactness tests, then noise / signal bench.
set -o pipefail
O=gpurun_out/r4hd
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_harmdistill_gpu.py tests/test_peakcluster_gpu.py tests/test_models_gpu.py::test_rank_fault_aborts_group_then_resume > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --signal > $O/bench_signal.log 2>&1 || { echo SIG_FAIL; tail -20 $O/bench_signal.log; exit 1; }
grep '^{"metric"' $O/bench_signal.log | cut -c1-120; grep '^{"metric"' $O/bench_signal.log | grep -o '"config".*'
PSOUP_GPU_DISTILL=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --signal > $O/bench_signal_hostd.log 2>&1 || { echo SIG0_FAIL; tail -20 $O/bench_signal_hostd.log; exit 1; }
grep '^{"metric"' $O/bench_signal_hostd.log | cut -c1-120; grep '^{"metric"' $O/bench_signal_hostd.log | grep -o '"config".*'
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-120
echo DONE
