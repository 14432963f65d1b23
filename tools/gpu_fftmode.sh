#!/bin/bash
# GPU check of the accel-trial FFT paths: fft4 numerics first, then the GPU
# suite, then the 2^23 bench: rocFFT C2C (mode 1) and the fused four-step
# (mode 2) over a few batch sizes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "fft4 or r2c" > gpurun_out/pytest_fft4.log 2>&1 || { echo FFT4_FAIL; tail -40 gpurun_out/pytest_fft4.log; exit 1; }
tail -1 gpurun_out/pytest_fft4.log
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for cfg in "1 0" "2 0" "2 8" "2 4" "2 2"; do
  set -- $cfg
  timeout -k 10 400 python bench.py --steps 2 --fft-mode $1 --accel-batch $2 > gpurun_out/bench23_m$1_k$2.log 2>&1 || { echo B$1_$2_FAIL; tail -30 gpurun_out/bench23_m$1_k$2.log; exit 1; }
  echo "mode=$1 K=$2 $(tail -1 gpurun_out/bench23_m$1_k$2.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["accel_batch"])')"
done
