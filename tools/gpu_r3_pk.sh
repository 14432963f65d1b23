#!/bin/bash
# Packed-f32 FFT arithmetic (cplx_pk.hpp) vs the scalar build (ab_scalar/):
# kernel GPU tests, pass-A phase split and kbench for both, ABAB bench.
set -o pipefail
O=gpurun_out/r3pk
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_pipeline_gpu.py > $O/pytest.log 2>&1 \
  || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in pk scalar; do
  D=.; [ $v = scalar ] && D=ab_scalar
  timeout -k 10 200 python -u $D/tools/expt/passa_phases.py --extra 0 > $O/passa_$v.txt 2>&1 || { echo PHASES_FAIL $v; tail -20 $O/passa_$v.txt; exit 1; }
  echo "== $v"; cat $O/passa_$v.txt | grep extra
  timeout -k 10 200 python -u $D/tools/kbench.py --flags 212227 > $O/kbench_$v.txt 2>&1 || { echo KBENCH_FAIL $v; tail -20 $O/kbench_$v.txt; exit 1; }
  grep -E "colpass|rowpass|r2c|harmonic" $O/kbench_$v.txt
done
for r in 1 2; do
  for v in pk scalar; do
    D=.; [ $v = scalar ] && D=ab_scalar
    timeout -k 10 300 python -u $D/bench.py --steps 10 --warmup 3 > $O/bench_${v}_$r.log 2>&1 || { echo BENCH_FAIL $v; tail -20 $O/bench_${v}_$r.log; exit 1; }
    echo -n "$v rep $r: "; grep '^{"metric"' $O/bench_${v}_$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
  done
done
echo DONE
