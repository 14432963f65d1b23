#!/bin/bash
# Harmonic exact-path change: screen / spectrum tests, benches (noise,
# peak-heavy x2), fft4 phase trace and kernel microbenchmarks.
set -o pipefail
O=gpurun_out/${1:-r5e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_screen_gpu.py tests/test_spectrum_gpu.py > $O/t1.log 2>&1 || { tail -30 $O/t1.log; exit 1; }
tail -1 $O/t1.log
for c in "--steps 10 --warmup 2" "--steps 10 --warmup 2 --peak-heavy" "--steps 10 --warmup 2" "--steps 10 --warmup 2 --peak-heavy"; do
  timeout -k 10 300 python bench.py $c > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  grep "^{" $O/b.log >> $O/bench.jsonl
  echo "$c: $(grep "^{" $O/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 200 python tools/expt/fft4_trace.py > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
grep -v amdgpu.ids $O/trace.log
timeout -k 10 200 python tools/kbench.py > $O/kbench.log 2>&1 || { tail -5 $O/kbench.log; exit 1; }
tail -12 $O/kbench.log
echo DONE
