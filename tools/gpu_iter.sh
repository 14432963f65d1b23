#!/bin/bash
# Iteration loop on the GPU box: selected GPU tests (-k filter), the default
# bench, then rocprofv3 kernel stats of a single-stream bench (per-kernel times).
# usage: tools/gpu_iter.sh "<pytest -k expr>" [extra bench args...]
set -o pipefail
mkdir -p gpurun_out
kexpr=${1:-fft4}; shift || true
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread -k "$kexpr" > gpurun_out/pytest_iter.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/pytest_iter.log; exit 1; }
tail -1 gpurun_out/pytest_iter.log
timeout -k 10 400 python bench.py "$@" > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
bash tools/gpu_prof.sh prof1 --sub-batch 0 "$@" && python3 tools/prof_summary.py gpurun_out/prof1/bench_kernel_stats.csv 8
