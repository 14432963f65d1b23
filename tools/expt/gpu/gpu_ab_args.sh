#!/bin/bash
# Same-box A/B of bench.py over option sets, interleaved repeats:
#   tools/expt/gpu/gpu_ab_args.sh REPS "--dedisp-kernel auto" "--dedisp-kernel mfma" ...
set -o pipefail
mkdir -p gpurun_out
reps=$1; shift
for r in $(seq 1 $reps); do
  i=0
  for opts in "$@"; do
    i=$((i + 1))
    log=gpurun_out/abargs_${i}_${r}.log
    timeout -k 10 300 python bench.py --steps 3 $opts > $log 2>&1 || { echo "FAIL $opts"; tail -5 $log; exit 1; }
    echo -n "[$opts] rep=$r "; tail -1 $log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
  done
done
