#!/bin/bash
# One-exchange pass B without its waterfall loops vs the Stockham pass B.
set -o pipefail
O=gpurun_out/r3onexrow
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "fft4" > $O/pytest.log 2>&1 \
  || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/kbench.py --K 64 --reps 6 --flags 1073954051,1074478339 > $O/kbench.txt 2>&1 || { echo KB_FAIL; tail -20 $O/kbench.txt; exit 1; }
grep -E "colpass|rowpass" $O/kbench.txt
for r in 1 2; do
  for f in 1073954051 1074478339; do
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --fft4-flags $f > $O/bench_${f}_$r.log 2>&1 || { echo BENCH_FAIL $f; tail -20 $O/bench_${f}_$r.log; exit 1; }
    echo -n "flags $f rep $r: "; grep '^{"metric"' $O/bench_${f}_$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
  done
done
echo DONE
