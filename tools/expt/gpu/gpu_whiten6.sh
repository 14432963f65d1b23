#!/bin/bash
# Whitening strip path: numerics tests, the isolated whitening cost, a
# same-box A/B of the whitener's strip path (kFft4WhitenStrips) on the 2^20
# bench, and a kernel profile of the new default.   tools/expt/gpu/gpu_whiten6.sh OUT
set -o pipefail
O=gpurun_out/${1:-whiten6}
A=1084701955; B=1101479171; C=1168588035; D=1135033603
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "whiten or batched or flat" > $O/t0.log 2>&1 || { tail -40 $O/t0.log; exit 1; }
tail -1 $O/t0.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_spectrum_gpu.py tests/test_pipeline_gpu.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "fft4 or strip or pad" > $O/t2.log 2>&1 || { tail -30 $O/t2.log; exit 1; }
tail -1 $O/t2.log
timeout -k 10 300 python tools/expt/whiten_bench.py --log2n 20 --dms 32 > $O/wb.log 2>&1 || { tail -10 $O/wb.log; exit 1; }
tail -2 $O/wb.log
for rep in 1 2; do
  for f in $A $B $C $D; do
    timeout -k 10 300 python bench.py --log2n 20 --dms-per-gpu 32 --steps 10 --warmup 2 --fft4-flags $f > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    grep "^{" $O/b.log >> $O/b20_$f.jsonl
    echo "2^20 flags $f: $(grep -o '"value": [0-9.]*' $O/b.log)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py --log2n 20 --dms-per-gpu 32 --steps 10 --warmup 2 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
echo DONE
