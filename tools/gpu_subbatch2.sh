#!/bin/bash
# (accel_batch, sub_batch) sweep of the headline bench: args are K:SB pairs.
set -o pipefail
mkdir -p gpurun_out
for kv in "$@"; do
  k=${kv%%:*}; sb=${kv##*:}
  PSOUP_SUB_BATCH=$sb timeout -k 10 300 python bench.py --steps 2 --warmup 1 --accel-batch $k > gpurun_out/bench_k${k}_sb$sb.log 2>&1 || { echo BENCH_FAIL $kv; tail -30 gpurun_out/bench_k${k}_sb$sb.log; exit 1; }
  echo -n "K=$k sub=$sb "; tail -1 gpurun_out/bench_k${k}_sb$sb.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
done
