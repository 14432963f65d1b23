#!/bin/bash
# kFft4WideStockham A/B: bit-identity, then the 2^20 / 2^22 / 2^25 benches ABAB.
set -o pipefail
O=gpurun_out/${1:-widest}
A=1135033603; B=1269251331
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/expt/wide_stockham_check.py $A $B > $O/check.log 2>&1 || { tail -20 $O/check.log; exit 1; }
grep 2^ $O/check.log
for rep in 1 2; do
  for f in $A $B; do
    timeout -k 10 300 python bench.py --log2n 20 --dms-per-gpu 32 --steps 10 --warmup 2 --fft4-flags $f > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "2^20 $f: $(grep -o '"value": [0-9.]*' $O/b.log)"
    timeout -k 10 300 python bench.py --log2n 22 --dms-per-gpu 16 --steps 6 --warmup 2 --fft4-flags $f > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "2^22 $f: $(grep -o '"value": [0-9.]*' $O/b.log)"
    timeout -k 10 300 python bench.py --log2n 25 --dms-per-gpu 1 --steps 2 --warmup 1 --fft4-flags $f > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "2^25 $f: $(grep -o '"value": [0-9.]*' $O/b.log)"
  done
done
echo DONE
