#!/bin/bash
# Quick GPU iteration: fft4/r2c numerics, then one 2^23 bench (args passed through).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "fft4 or r2c" > gpurun_out/pytest_fft4.log 2>&1 || { echo FFT4_FAIL; tail -40 gpurun_out/pytest_fft4.log; exit 1; }
tail -1 gpurun_out/pytest_fft4.log
timeout -k 10 400 python bench.py --steps 2 "$@" > gpurun_out/bench_quick.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_quick.log; exit 1; }
tail -1 gpurun_out/bench_quick.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["accel_batch"], d["config"]["fft_mode"])'
