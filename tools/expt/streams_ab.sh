#!/bin/bash
# Same-box A/B of the number of sub-batch compute streams (and sub-batch sizes).
set -o pipefail
mkdir -p gpurun_out
for cfg in "2 32" "3 32" "4 32" "3 16" "4 16" "2 32"; do
  set -- $cfg
  PSOUP_SUB_STREAMS=$1 timeout -k 10 200 python bench.py --steps 4 --sub-batch $2 > gpurun_out/sab.log 2>&1 || { echo FAIL $cfg; tail -5 gpurun_out/sab.log; exit 1; }
  echo "streams=$1 sub=$2 $(tail -1 gpurun_out/sab.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
