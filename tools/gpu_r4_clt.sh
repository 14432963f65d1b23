#!/bin/bash
set -o pipefail
O=gpurun_out/r4clt
mkdir -p $O
export TMPDIR=/tmp
for n in 4200 9000 12000; do timeout -k 10 120 python -u tools/expt/cluster_bench.py --dense --trace --n $n > $O/cbt_$n.log 2>&1 || { echo CB_FAIL; tail -5 $O/cbt_$n.log; exit 1; }; tail -2 $O/cbt_$n.log; done
echo DONE
