#!/bin/bash
# Fold stage v2: gathered kept rows, pre-built fold engines. Fold/pipeline
# GPU tests, config 5 kernel trace, native config-5-like CLI run timing.
set -o pipefail
O=gpurun_out/r3fold2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_pipeline_gpu.py tests/test_models_gpu.py tests/test_kernels_gpu.py -k "fold or golden or multi_rank or oversub or time_shard or checkpoint" > $O/pytest.log 2>&1 \
  || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest.log | head; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 tools/baseline_configs.py --configs 5 --workdir /tmp/cfg --out $O/c5.jsonl > $O/c5.log 2>&1 || { echo C5_FAIL; tail -20 $O/c5.log; exit 1; }
cut -c1-1500 $O/c5.jsonl
timeout -k 10 400 python3 tools/baseline_configs.py --configs 5 --native --workdir /tmp/cfg --out $O/c5n.jsonl > $O/c5n.log 2>&1 || { echo C5N_FAIL; tail -20 $O/c5n.log; exit 1; }
cut -c1-1500 $O/c5n.jsonl
echo DONE
