#!/bin/bash
# Auto batch of 512 trials at 2^23: GPU suite, same-box bench A/B against the
# old 256-trial batch, configs 3 and 4.
set -o pipefail
mkdir -p gpurun_out/b512
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/b512/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/b512/pytest.log; exit 1; }
tail -1 gpurun_out/b512/pytest.log
bash tools/expt/gpu/gpu_ab_args.sh 2 "" "--accel-batch 256" || exit 1
timeout -k 10 400 python tools/baseline_configs.py --configs 3,4 --workdir /tmp/cfgb --out gpurun_out/b512/cfg.jsonl > gpurun_out/b512/cfg.log 2>&1 || { echo CFG_FAIL; tail -20 gpurun_out/b512/cfg.log; exit 1; }
cat gpurun_out/b512/cfg.jsonl
