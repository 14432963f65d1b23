#!/bin/bash
set -o pipefail
O=gpurun_out/r3cl
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_peakcluster_gpu.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for th in 1024 512; do
  for st in 1 2 3 4 99; do
    PSOUP_CLUSTER_TH=$th PSOUP_CLUSTER_STOP=$st timeout -k 10 120 python -u tools/expt/cluster_bench.py >> $O/cluster.txt 2>&1 || { echo CB_FAIL; tail -20 $O/cluster.txt; exit 1; }
  done
done
cat $O/cluster.txt
echo DONE
