#!/bin/bash
# GPU check of the fused real-FFT path: kernel tests, then the 2^23 bench with
# both FFT modes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --fft-mode 0 > gpurun_out/bench23_m0.log 2>&1 || { echo B0_FAIL; tail -30 gpurun_out/bench23_m0.log; exit 1; }
tail -1 gpurun_out/bench23_m0.log
timeout -k 10 400 python bench.py --fft-mode 1 > gpurun_out/bench23_m1.log 2>&1 || { echo B1_FAIL; tail -30 gpurun_out/bench23_m1.log; exit 1; }
tail -1 gpurun_out/bench23_m1.log
