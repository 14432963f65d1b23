#!/bin/bash
# Strip-layout pass-A input (kFft4StripInput): fft4 numerics for every flag
# set, pass-A phase split with and without, ABAB bench.
set -o pipefail
O=gpurun_out/r3strip
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "fft4 or whitener or batched or flat" > $O/pytest.log 2>&1 \
  || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u tools/expt/passa_phases.py --extra 0,1073741824 > $O/passa.txt 2>&1 || { echo PHASES_FAIL; tail -20 $O/passa.txt; exit 1; }
grep extra $O/passa.txt
for r in 1 2; do
  for f in 212227 1073954051; do
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --fft4-flags $f > $O/bench_${f}_$r.log 2>&1 || { echo BENCH_FAIL $f; tail -20 $O/bench_${f}_$r.log; exit 1; }
    echo -n "flags $f rep $r: "; grep '^{"metric"' $O/bench_${f}_$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
  done
done
echo DONE
