#!/bin/bash
# Same-box sweep of the acceleration batch (K) and FFT sub-batch for bench.py.
set -o pipefail
mkdir -p gpurun_out/sweep
CFGS=("64 32" "128 32" "128 64" "256 32" "64 64" "64 32")
[ -n "$SWEEP" ] && IFS=, read -ra CFGS <<< "$SWEEP"
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --accel-batch $1 --sub-batch $2 > gpurun_out/sweep/b_$1_$2.log 2>&1 || { echo "FAIL $cfg"; tail -20 gpurun_out/sweep/b_$1_$2.log; exit 1; }
  echo "ab=$1 sb=$2 $(tail -1 gpurun_out/sweep/b_$1_$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
