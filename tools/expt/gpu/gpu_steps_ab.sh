#!/bin/bash
# Same-box A/B of the bench's step pipeline (default) against --serial-steps
# at 2^23 (noise, --peak-heavy) and 2^20 (32 DMs per step), one JSON line per
# run in gpurun_out/$1/bench.jsonl (profiles/r5_pipe).
set -o pipefail
O=gpurun_out/${1:-steps_ab}
mkdir -p $O
export TMPDIR=/tmp
for c in "--steps 10 --warmup 2" "--steps 10 --warmup 2 --serial-steps" \
         "--steps 10 --warmup 2 --peak-heavy" "--steps 10 --warmup 2 --peak-heavy --serial-steps" \
         "--log2n 20 --dms-per-gpu 32 --steps 20 --warmup 3" "--log2n 20 --dms-per-gpu 32 --steps 20 --warmup 3 --serial-steps"; do
  timeout -k 10 300 python bench.py $c > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  grep "^{" $O/b.log >> $O/bench.jsonl
  echo "$c: $(grep "^{" $O/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
