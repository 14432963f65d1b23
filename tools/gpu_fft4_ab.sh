#!/bin/bash
# fft4 numerics tests + per-kernel microbenchmark + phase trace + 3-step bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "fft4 or resample or batching or short_list or whiten" > gpurun_out/fft4_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/fft4_tests.log; exit 1; }
tail -1 gpurun_out/fft4_tests.log
timeout -k 10 200 python tools/kbench.py --K 32 --reps 20 --flags 81155 > gpurun_out/kbench_ab.log 2>&1 || { echo KBENCH_FAIL; tail -5 gpurun_out/kbench_ab.log; exit 1; }
grep -E "colpass|rowpass" gpurun_out/kbench_ab.log
timeout -k 10 200 python tools/expt/fft4_trace.py > gpurun_out/trace.log 2>&1 || { echo TRACE_FAIL; tail -5 gpurun_out/trace.log; exit 1; }
sed -n 2,12p gpurun_out/trace.log
timeout -k 10 300 python bench.py --steps 3 > gpurun_out/bench_ab.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/bench_ab.log; exit 1; }
tail -1 gpurun_out/bench_ab.log | cut -c1-200
