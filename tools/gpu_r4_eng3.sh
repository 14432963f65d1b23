#!/bin/bash
# After the engine default change: pipeline/model tests, 2^20 bench with 1 vs 3 engines.
set -o pipefail
O=gpurun_out/r4eng3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_pipeline_gpu.py tests/test_models_gpu.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for e in 1 3 1 3; do
  PSOUP_ENGINES=$e timeout -k 10 300 python -u bench.py --log2n 20 --dms-per-gpu 32 --steps 20 --warmup 3 > $O/bench20_e$e.log 2>&1 || { echo BENCH20_FAIL; tail -20 $O/bench20_e$e.log; exit 1; }
  echo -n "engines $e: "; grep '^{"metric"' $O/bench20_e$e.log | cut -c1-140
done
echo DONE
