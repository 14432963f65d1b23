#!/bin/bash
# Round-6 A/B on one box: numerics tests of the fused FFT passes, per-kernel
# times (kbench) and the trace of both flag sets, then the bench with each
# flag set (ABAB).  tools/expt/gpu/gpu_ab6.sh OUT OLD_FLAGS NEW_FLAGS [test files]
set -o pipefail
O=gpurun_out/${1:-ab6}; A=$2; B=$3; shift 3
mkdir -p $O
export TMPDIR=/tmp
T="${@:-tests/test_spectrum_gpu.py tests/test_screen_gpu.py}"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread $T > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for f in $A $B; do
  timeout -k 10 200 python tools/kbench_fused.py --flags $f > $O/kb_$f.log 2>&1 || { tail -5 $O/kb_$f.log; exit 1; }
  cat $O/kb_$f.log
done
for f in $A $B; do
  timeout -k 10 200 python tools/expt/fft4_trace.py $f > $O/trace_$f.log 2>&1 || { tail -5 $O/trace_$f.log; exit 1; }
done
for rep in 1 2; do
  for f in $A $B; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --fft4-flags $f > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    grep "^{" $O/b.log >> $O/bench_$f.jsonl
    echo "flags $f: $(grep "^{" $O/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
echo DONE
