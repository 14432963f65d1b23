#!/bin/bash
# Sweep the acceleration batch size K at 2^23 (MALL residency vs launch count).
set -o pipefail
mkdir -p gpurun_out
for k in 2 4 8 16 64; do
  timeout -k 10 300 python bench.py --steps 2 --accel-batch $k > gpurun_out/sweep_k$k.log 2>&1 || { echo FAIL_$k; tail -30 gpurun_out/sweep_k$k.log; exit 1; }
  echo "K=$k $(tail -1 gpurun_out/sweep_k$k.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
