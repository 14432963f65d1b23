#!/bin/bash
# Same-box A/B of the short-list batch balancing (PSOUP_MIN_BATCHES) on BASELINE config 3, then bench.
set -o pipefail
mkdir -p gpurun_out/cfg3
for mb in 8 1 8 1; do
  PSOUP_MIN_BATCHES=$mb timeout -k 10 200 python tools/baseline_configs.py --configs 3 > gpurun_out/cfg3/mb$mb.log 2>&1 || { tail -20 gpurun_out/cfg3/mb$mb.log; exit 1; }
  echo "min_batches=$mb $(grep '^{' gpurun_out/cfg3/mb$mb.log | cut -c90-200)"
done
timeout -k 10 300 python bench.py --steps 8 --warmup 2 > gpurun_out/cfg3/bench.log 2>&1 || { tail -20 gpurun_out/cfg3/bench.log; exit 1; }
tail -1 gpurun_out/cfg3/bench.log | cut -c1-200
