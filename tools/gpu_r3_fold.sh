#!/bin/bash
# Fold stage: register-FFT optimiser + kept dedispersed rows. GPU suite,
# config 5 with a kernel trace.
set -o pipefail
O=gpurun_out/r3fold
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 280 --timeout-method thread tests/ > $O/pytest_gpu.log 2>&1 \
  || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 tools/baseline_configs.py --configs 4,5 --workdir /tmp/cfg --out $O/c45.jsonl > $O/c5.log 2>&1 || { echo C5_FAIL; tail -20 $O/c5.log; exit 1; }
cut -c1-1500 $O/c45.jsonl
echo DONE
