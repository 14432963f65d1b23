#!/bin/bash
# Sub-batch sweep at 2^23 (same box, interleaved): sub-batch 0/16/32/64/128
# at K = 256, and K = 128/512 without sub-batches.
set -o pipefail
O=gpurun_out/r3sub
mkdir -p $O
for r in 1 2; do
  for cfg in "256 0" "256 32" "256 64" "256 128" "256 16" "512 0" "128 0"; do
    set -- $cfg
    tag="K${1}_sb${2}_$r"
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --accel-batch $1 --sub-batch $2 > $O/$tag.log 2>&1 || { echo BENCH_FAIL $tag; tail -20 $O/$tag.log; exit 1; }
    echo -n "$tag: "; grep '^{"metric"' $O/$tag.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["accel_batch"], d["config"]["sub_batch"])'
  done
done
echo DONE
