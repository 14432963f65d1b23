#!/bin/bash
# Round 3: fused pass B numerics + kernel timings (fused vs unfused, harmonic
# sum on natural vs blocked spectra).
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "fused or blocked_layout or fft4_interbin or prethreshold or fft4_pruned" > gpurun_out/r3/pytest_fused.log 2>&1 \
  || { echo PYTEST_FAIL; tail -40 gpurun_out/r3/pytest_fused.log; exit 1; }
tail -3 gpurun_out/r3/pytest_fused.log
timeout -k 10 200 python -u tools/kbench_fused.py --K 32 --reps 10 > gpurun_out/r3/kbench_fused.txt 2>&1 \
  || { echo KBENCH_FAIL; tail -20 gpurun_out/r3/kbench_fused.txt; exit 1; }
cat gpurun_out/r3/kbench_fused.txt
# same-box ABBA bench: default flags vs + kFft4FusedR2c
D=212227; F=$((212227 | 2097152))
for fl in $D $F $F $D; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --fft4-flags $fl > gpurun_out/r3/bench_$fl.log 2>&1 \
    || { echo BENCH_FAIL $fl; tail -20 gpurun_out/r3/bench_$fl.log; exit 1; }
  echo "flags=$fl $(tail -1 gpurun_out/r3/bench_$fl.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
