#!/bin/bash
# Quick check after a kernel change: the given GPU test files (default: the
# spectrum / screen / kernel numerics), kernel microbenchmarks, two noise and
# one peak-heavy bench.  tools/expt/gpu/gpu_quick.sh OUTNAME [test files...]
set -o pipefail
O=gpurun_out/${1:-quick}; shift
mkdir -p $O
export TMPDIR=/tmp
T="${@:-tests/test_spectrum_gpu.py tests/test_screen_gpu.py}"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread $T > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 200 python tools/kbench.py > $O/kbench.log 2>&1 || { tail -5 $O/kbench.log; exit 1; }
grep "colpass\|rowpass_spectrum\|screened" $O/kbench.log
for c in "--steps 10 --warmup 2" "--steps 10 --warmup 2 --peak-heavy" "--steps 10 --warmup 2"; do
  timeout -k 10 300 python bench.py $c > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  grep "^{" $O/b.log >> $O/bench.jsonl
  echo "$c: $(grep "^{" $O/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
echo DONE
