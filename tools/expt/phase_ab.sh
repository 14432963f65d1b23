#!/bin/bash
# Same-box bench A/B of the sub-batch stage gating (PSOUP_SUB_PHASE), interleaved.
set -o pipefail
mkdir -p gpurun_out/phase
for r in 1 2; do
  for ph in "$@"; do
    PSOUP_SUB_PHASE=$ph timeout -k 10 300 python bench.py --steps 3 > gpurun_out/phase/ph${ph}_$r.log 2>&1 || { echo FAIL $ph; tail -5 gpurun_out/phase/ph${ph}_$r.log; exit 1; }
    echo -n "phase=$ph rep=$r "; tail -1 gpurun_out/phase/ph${ph}_$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
  done
done
