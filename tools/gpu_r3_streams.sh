#!/bin/bash
# Strip input vs row-pitch input, single stream (--sub-batch 0) and the default
# two sub-batch streams; whole-CU one-exchange pass A with strips.
set -o pipefail
O=gpurun_out/r3streams
mkdir -p $O
for r in 1 2; do
  for cfg in "0 1073954051" "0 212227" "-1 1073954051" "-1 212227" "-1 1074216195"; do
    set -- $cfg
    tag="sb${1}_f${2}_$r"
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --sub-batch $1 --fft4-flags $2 > $O/$tag.log 2>&1 || { echo BENCH_FAIL $tag; tail -20 $O/$tag.log; exit 1; }
    echo -n "$tag: "; grep '^{"metric"' $O/$tag.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["sub_batch"])'
  done
done
echo DONE
for r in 1; do
  for ht in -1 8 12; do
    tag="sig_ht${ht}_$r"
    PSOUP_HOST_THREADS=$ht timeout -k 10 300 python -u bench.py --signal --steps 5 --warmup 2 > $O/$tag.log 2>&1 || { echo BENCH_FAIL $tag; tail -20 $O/$tag.log; exit 1; }
    echo -n "$tag: "; grep '^{"metric"' $O/$tag.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["host_distill_s_per_step"])'
  done
done
echo DONE2
