#!/bin/bash
# Native block pipeline: the pipeline GPU tests, then config 4 with
# PSOUP_BLOCK_PIPELINE=0 / 1, alternating on one box.
set -o pipefail
O=gpurun_out/${1:-npipe}
mkdir -p $O /tmp/cfgw
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_pipeline_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --native --workdir /tmp/cfgw > $O/warm.log 2>&1 || { tail -10 $O/warm.log; exit 1; }
for rep in 1 2 3; do
  for p in 0 1; do
    PSOUP_BLOCK_PIPELINE=$p timeout -k 10 300 python3 tools/baseline_configs.py --configs 4,5 --native --workdir /tmp/cfgw --out $O/native_pipe$p.jsonl > $O/n.log 2>&1 || { tail -10 $O/n.log; exit 1; }
  done
done
for p in 0 1; do echo "pipeline $p"; python3 tools/summarize_jsonl.py $O/native_pipe$p.jsonl timers_s.searching timers_s.total performance.phase_search_s; done
echo DONE
