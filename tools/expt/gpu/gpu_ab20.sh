#!/bin/bash
# Same-box A/B of two fft4 flag sets on the 2^20 bench (ABAB) and at 2^23.
set -o pipefail
O=gpurun_out/${1:-ab20}; A=$2; B=$3
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for f in $A $B; do
    timeout -k 10 300 python bench.py --log2n 20 --dms-per-gpu 32 --steps 10 --warmup 2 --fft4-flags $f > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    grep "^{" $O/b.log >> $O/b20_$f.jsonl
    echo "2^20 flags $f: $(grep -o '"value": [0-9.]*' $O/b.log)"
  done
done
for f in $A $B; do
  timeout -k 10 300 python bench.py --log2n 22 --dms-per-gpu 16 --steps 6 --warmup 2 --fft4-flags $f > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  grep "^{" $O/b.log >> $O/b22_$f.jsonl
  echo "2^22 flags $f: $(grep -o '"value": [0-9.]*' $O/b.log)"
done
echo DONE
