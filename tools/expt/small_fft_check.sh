#!/bin/bash
# fft4/whitening numerics at every size, then the 2^20 search microbenchmark and configs 2-4.
set -o pipefail
mkdir -p gpurun_out/sf
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_pipeline_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "fft4 or whiten or golden or mixed" > gpurun_out/sf/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/sf/pytest.log; exit 1; }
tail -1 gpurun_out/sf/pytest.log
timeout -k 10 200 python -u tools/expt/whiten_bench.py --dms 32 --reps 10 2>&1 | grep -v amdgpu.ids
timeout -k 10 400 python tools/baseline_configs.py --configs 2,3,4 --workdir /tmp/cfgsf --out gpurun_out/sf/cfg.jsonl > gpurun_out/sf/cfg.log 2>&1 || { echo CFG_FAIL; tail -20 gpurun_out/sf/cfg.log; exit 1; }
cat gpurun_out/sf/cfg.jsonl
