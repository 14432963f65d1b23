#!/bin/bash
# Cluster sort with register stages (PSOUP_CLUSTER_RSORT=1, opt-in) vs the
# all-LDS default: exactness tests under both, microbenchmark, peak-heavy bench.
set -o pipefail
O=gpurun_out/r3csort
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread tests/test_peakcluster_gpu.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
PSOUP_CLUSTER_RSORT=1 timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread tests/test_peakcluster_gpu.py > $O/pytest_rsort.log 2>&1 || { echo PYTEST_RSORT_FAIL; grep -E "FAILED|Error" $O/pytest_rsort.log | head; tail -30 $O/pytest_rsort.log; exit 1; }
tail -1 $O/pytest_rsort.log
for v in 0 1; do
  for n in 4200 2000 9000; do
    echo -n "rsort=$v n=$n: "; PSOUP_CLUSTER_RSORT=$v timeout -k 10 120 python3 tools/expt/cluster_bench.py --n $n > $O/cb_${v}_$n.log 2>&1 || { echo CB_FAIL; tail -20 $O/cb_${v}_$n.log; exit 1; }
    tail -1 $O/cb_${v}_$n.log
  done
done
for r in 1 2; do
  for v in 0 1; do
    PSOUP_CLUSTER_RSORT=$v timeout -k 10 300 python -u bench.py --signal --steps 5 --warmup 2 > $O/sig_${v}_$r.log 2>&1 || { echo SIG_FAIL; tail -20 $O/sig_${v}_$r.log; exit 1; }
    echo -n "signal rsort=$v $r: "; grep '^{"metric"' $O/sig_${v}_$r.log | cut -c1-130
  done
done
echo DONE
