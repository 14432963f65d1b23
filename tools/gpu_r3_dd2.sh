#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "dedisperse or mfma_resident" > gpurun_out/r3/pytest_dedisp2.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/r3/pytest_dedisp2.log; exit 1; }
tail -1 gpurun_out/r3/pytest_dedisp2.log
timeout -k 10 300 python -u tools/dedisp_bench.py --ndm 2000 --log2n 20 --reps 3 > gpurun_out/r3/dedisp_bench2.jsonl 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/r3/dedisp_bench2.jsonl; exit 1; }
cat gpurun_out/r3/dedisp_bench2.jsonl
