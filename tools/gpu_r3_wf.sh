#!/bin/bash
# Pass A without waterfall loops (uniform buffer resource), constant-memory
# trace pointer and DFT-ordered loads vs HEAD (ab_old/): numerics, phase
# split at K = 256, ABAB bench.
set -o pipefail
O=gpurun_out/r3wf
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "fft4 or whitener or batched or flat or fold" > $O/pytest.log 2>&1 \
  || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in new old; do
  D=.; [ $v = old ] && D=ab_old
  timeout -k 10 200 python -u $D/tools/expt/passa_phases.py --K 256 --reps 4 --only-full --extra 0,512 > $O/passa_$v.txt 2>&1 || { echo PHASES_FAIL $v; tail -20 $O/passa_$v.txt; exit 1; }
  echo "$v: $(grep extra $O/passa_$v.txt)"
done
for r in 1 2; do
  for v in new old newprio; do
    D=.; [ $v = old ] && D=ab_old
    F=""; [ $v = newprio ] && F="--fft4-flags 1073954563"
    timeout -k 10 300 python -u $D/bench.py --steps 10 --warmup 3 $F > $O/bench_${v}_$r.log 2>&1 || { echo BENCH_FAIL $v; tail -20 $O/bench_${v}_$r.log; exit 1; }
    echo -n "$v rep $r: "; grep '^{"metric"' $O/bench_${v}_$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
  done
done
echo DONE
