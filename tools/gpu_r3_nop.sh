#!/bin/bash
# Compiler-visible packed add/sub (fewer s_nop)  vs HEAD
# (ab_old/): numerics, golden pipeline, kbench, ABAB bench.
set -o pipefail
O=gpurun_out/r3nop
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_kernels_gpu.py tests/test_pipeline_gpu.py -k "r2c or interbin or fft4 or golden or fft_modes or headline or injected or harmonic" > $O/pytest.log 2>&1 \
  || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in new old; do
  D=.; [ $v = old ] && D=ab_old
  timeout -k 10 300 python -u $D/tools/kbench.py --K 64 --reps 6 --flags 1073954051 > $O/kbench_$v.txt 2>&1 || { echo KB_FAIL; tail -20 $O/kbench_$v.txt; exit 1; }
  echo "$v:"; grep -E "colpass|rowpass|tiled" $O/kbench_$v.txt
done
for r in 1 2; do
  for v in new old; do
    D=.; [ $v = old ] && D=ab_old
    timeout -k 10 300 python -u $D/bench.py --steps 10 --warmup 3 > $O/bench_${v}_$r.log 2>&1 || { echo BENCH_FAIL $v; tail -20 $O/bench_${v}_$r.log; exit 1; }
    echo -n "$v rep $r: "; grep '^{"metric"' $O/bench_${v}_$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
  done
done
echo DONE
