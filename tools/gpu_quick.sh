#!/bin/bash
# Quick A/B: fft4 phase trace, kernel microbenchmarks, 2 noise benches.
set -o pipefail
O=gpurun_out/${1:-quick}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/expt/fft4_trace.py > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
grep -v amdgpu.ids $O/trace.log | head -8
timeout -k 10 200 python tools/kbench.py > $O/kbench.log 2>&1 || { tail -5 $O/kbench.log; exit 1; }
grep "colpass\|rowpass_spectrum\|screened" $O/kbench.log
for c in "--steps 10 --warmup 2" "--steps 10 --warmup 2"; do
  timeout -k 10 300 python bench.py $c > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  grep "^{" $O/b.log >> $O/bench.jsonl
  echo "$c: $(grep "^{" $O/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
echo DONE
