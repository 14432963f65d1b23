#!/bin/bash
# Full GPU suite on the new defaults; config-5 kernel trace (fold stage);
# signal bench under marker + kernel trace (host/GPU timeline).
set -o pipefail
O=gpurun_out/r3p2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 280 --timeout-method thread tests/ > $O/pytest_gpu.log 2>&1 \
  || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 tools/baseline_configs.py --configs 5 --workdir /tmp/cfg --out $O/c5.jsonl > $O/c5.log 2>&1 || { echo C5_FAIL; tail -20 $O/c5.log; exit 1; }
cut -c1-1200 $O/c5.jsonl
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $O/prof_sig -o sig -- python3 bench.py --signal --steps 3 --warmup 1 > $O/sig.log 2>&1 || { echo SIG_FAIL; tail -20 $O/sig.log; exit 1; }
grep '^{"metric"' $O/sig.log | cut -c1-300
echo DONE
