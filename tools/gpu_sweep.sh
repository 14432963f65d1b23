#!/bin/bash
# Headline bench over (accel_batch:sub_batch) pairs, after the kernel microbenchmark.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/kbench.py --K 32 > gpurun_out/kbench.log 2>&1 || { echo KBENCH_FAIL; tail -30 gpurun_out/kbench.log; exit 1; }
cat gpurun_out/kbench.log
for kv in "$@"; do
  k=${kv%%:*}; sb=${kv##*:}
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --accel-batch $k --sub-batch $sb > gpurun_out/bench_k${k}_sb$sb.log 2>&1 || { echo BENCH_FAIL $kv; tail -30 gpurun_out/bench_k${k}_sb$sb.log; exit 1; }
  echo -n "K=$k sub=$sb "; tail -1 gpurun_out/bench_k${k}_sb$sb.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
done
