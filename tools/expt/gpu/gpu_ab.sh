#!/bin/bash
# A/B of bench.py over fft4 flag sets, interleaved repeats: tools/expt/gpu/gpu_ab.sh REPS flagsA flagsB ...
set -o pipefail
mkdir -p gpurun_out
reps=$1; shift
for r in $(seq 1 $reps); do
  for f in "$@"; do
    log=gpurun_out/ab_${f}_${r}.log
    timeout -k 10 300 python bench.py --steps 3 --fft4-flags $f > $log 2>&1 || { echo FAIL $f; tail -5 $log; exit 1; }
    echo -n "flags=$f rep=$r "; tail -1 $log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"])'
  done
done
