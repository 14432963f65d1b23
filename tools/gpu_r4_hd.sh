#!/bin/bash
# GPU harmonic distillation + unaligned dedispersion: exactness tests, then
# noise / signal bench, and every rank's step of a world-8 run on this GPU.
set -o pipefail
O=gpurun_out/r4hd
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_harmdistill_gpu.py tests/test_peakcluster_gpu.py "tests/test_kernels_gpu.py::test_dedisperse_1024ch_hybrid_mfma_bit_exact" "tests/test_kernels_gpu.py::test_mfma_resident_plan_ranges_and_side_stream" "tests/test_kernels_gpu.py::test_dedisperse_direct_mfma_valu_bit_exact" tests/test_models_gpu.py::test_rank_fault_aborts_group_then_resume tests/test_pipeline_gpu.py::test_native_oversubscribed_device_workers_match_one > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "PASS|FAIL|Error" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --signal > $O/bench_signal.log 2>&1 || { echo SIG_FAIL; tail -20 $O/bench_signal.log; exit 1; }
grep '^{"metric"' $O/bench_signal.log | cut -c1-120; grep '^{"metric"' $O/bench_signal.log | grep -o '"config".*'
PSOUP_GPU_DISTILL=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --signal > $O/bench_signal_hostd.log 2>&1 || { echo SIG0_FAIL; tail -20 $O/bench_signal_hostd.log; exit 1; }
grep '^{"metric"' $O/bench_signal_hostd.log | cut -c1-120; grep '^{"metric"' $O/bench_signal_hostd.log | grep -o '"config".*'
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-120
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --as-rank 8:0,1,2,3,4,5,6,7,0 > $O/as_rank.log 2>&1 || { echo ASRANK_FAIL; tail -20 $O/as_rank.log; exit 1; }
grep '^{"as_rank"' $O/as_rank.log
echo DONE
