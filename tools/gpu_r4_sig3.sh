#!/bin/bash
# Peak-heavy bench after the capacity-cut chunk fix, then noise bench, dense cluster bench.
set -o pipefail
O=gpurun_out/r4sig3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --signal > $O/bench_signal.log 2>&1 || { echo SIG_FAIL; tail -20 $O/bench_signal.log; exit 1; }
grep '^{"metric"' $O/bench_signal.log | cut -c1-120; grep '^{"metric"' $O/bench_signal.log | grep -o '"peaks_per_dm.*'
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-120
for n in 4200 9000; do timeout -k 10 120 python -u tools/expt/cluster_bench.py --dense --n $n > $O/cbd_$n.log 2>&1 || { echo CB_FAIL; tail -5 $O/cbd_$n.log; exit 1; }; tail -1 $O/cbd_$n.log; done
echo DONE
