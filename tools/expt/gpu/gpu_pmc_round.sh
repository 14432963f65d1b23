#!/bin/bash
# kernel numerics tests + kbench + PMC passes over the production bench kernels
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "${1:-harm or peak or r2c or fft4 or interbin}" > gpurun_out/pytest_k.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/pytest_k.log; exit 1; }
tail -1 gpurun_out/pytest_k.log
timeout -k 10 300 python tools/kbench.py --K 32 --flags 0 > gpurun_out/kbench.log 2>&1 || { echo KBENCH_FAIL; tail -30 gpurun_out/kbench.log; exit 1; }
grep -E "harmonic|tiled|torch" gpurun_out/kbench.log
bash tools/expt/gpu/gpu_pmc.sh pmc --sub-batch 0 --dms-per-gpu 2 && python3 tools/pmc_summary.py gpurun_out/pmc/*/p_counter_collection.csv --match fft4,r2c_inter,harmonic_peaks
