#!/bin/bash
set -o pipefail
O=gpurun_out/r4cl2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_peakcluster_gpu.py tests/test_harmdistill_gpu.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for n in 4200 9000 12000; do timeout -k 10 120 python -u tools/expt/cluster_bench.py --dense --trace --n $n > $O/cbt_$n.log 2>&1 || { echo CB_FAIL; tail -5 $O/cbt_$n.log; exit 1; }; tail -2 $O/cbt_$n.log; done
timeout -k 10 120 python -u tools/expt/cluster_bench.py --n 4200 > $O/cbs.log 2>&1 || { echo CBS_FAIL; tail -5 $O/cbs.log; exit 1; }; tail -1 $O/cbs.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --signal > $O/bench_signal.log 2>&1 || { echo SIG_FAIL; tail -20 $O/bench_signal.log; exit 1; }
grep '^{"metric"' $O/bench_signal.log | cut -c1-120
echo DONE
