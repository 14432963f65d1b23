#!/bin/bash
# Final-default whitening check: equality tests, then the 2^23 headline
# bench A/B (old whitening flags vs the default) and the 2^22 bench.
set -o pipefail
O=gpurun_out/${1:-wq}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "whiten or batched or flat" > $O/t0.log 2>&1 || { tail -40 $O/t0.log; exit 1; }
tail -1 $O/t0.log
for f in 1084701955 1135033603 1084701955 1135033603; do
  timeout -k 10 300 python bench.py --fft4-flags $f > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  grep "^{" $O/b.log >> $O/b23_$f.jsonl
  echo "2^23 flags $f: $(grep -o '"value": [0-9.]*' $O/b.log)"
done
for f in 1084701955 1135033603; do
  timeout -k 10 300 python bench.py --log2n 22 --dms-per-gpu 16 --steps 6 --warmup 2 --fft4-flags $f > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  grep "^{" $O/b.log >> $O/b22_$f.jsonl
  echo "2^22 flags $f: $(grep -o '"value": [0-9.]*' $O/b.log)"
done
echo DONE
