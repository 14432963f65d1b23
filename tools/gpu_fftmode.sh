#!/bin/bash
# GPU check of the accel-trial FFT paths: fft4 numerics first, then the GPU
# suite, then the 2^23 bench with rocFFT C2C (mode 1) and the fused four-step (2).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "fft4 or r2c" > gpurun_out/pytest_fft4.log 2>&1 || { echo FFT4_FAIL; tail -40 gpurun_out/pytest_fft4.log; exit 1; }
tail -1 gpurun_out/pytest_fft4.log
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for m in 1 2; do
  timeout -k 10 400 python bench.py --fft-mode $m > gpurun_out/bench23_m$m.log 2>&1 || { echo B${m}_FAIL; tail -30 gpurun_out/bench23_m$m.log; exit 1; }
  tail -1 gpurun_out/bench23_m$m.log
done
