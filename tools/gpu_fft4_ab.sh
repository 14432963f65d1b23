#!/bin/bash
# fft4 numerics tests + per-kernel microbenchmark (colpass breakdown flags) + 2-step bench.
set -o pipefail
mkdir -p gpurun_out
F=78083
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "fft4 or resample or batching or short_list" > gpurun_out/fft4_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/fft4_tests.log; exit 1; }
tail -1 gpurun_out/fft4_tests.log
timeout -k 10 200 python tools/kbench.py --K 32 --flags 81155,$F,$((F|64)),$((F|128|8)) > gpurun_out/kbench_ab.log 2>&1 || { echo KBENCH_FAIL; tail -5 gpurun_out/kbench_ab.log; exit 1; }
grep -E "colpass|rowpass" gpurun_out/kbench_ab.log
timeout -k 10 300 python bench.py --steps 3 > gpurun_out/bench_ab.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/bench_ab.log; exit 1; }
tail -1 gpurun_out/bench_ab.log | cut -c1-200
