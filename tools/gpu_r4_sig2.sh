#!/bin/bash
# Peak-heavy bench: merge split, per-block trace, kernel trace.
set -o pipefail
O=gpurun_out/r4sig2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_peakcluster_gpu.py tests/test_harmdistill_gpu.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for n in 2000 4200 9000; do timeout -k 10 120 python -u tools/expt/cluster_bench.py --n $n > $O/cb_$n.log 2>&1 || { echo CB_FAIL; tail -5 $O/cb_$n.log; exit 1; }; tail -1 $O/cb_$n.log; done
PSOUP_BLOCK_TRACE=$O/blocks.jsonl timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --signal > $O/bench_signal.log 2>&1 || { echo SIG_FAIL; tail -20 $O/bench_signal.log; exit 1; }
grep '^{"metric"' $O/bench_signal.log | cut -c1-120; grep '^{"metric"' $O/bench_signal.log | grep -o '"peaks_per_dm.*'
tail -3 $O/blocks.jsonl | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o sig -- python3 bench.py --signal --steps 4 --warmup 2 > $O/sig.log 2>&1 || { echo PROF_FAIL; tail -20 $O/sig.log; exit 1; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
cp $T $O/kernel_trace.csv
echo DONE
