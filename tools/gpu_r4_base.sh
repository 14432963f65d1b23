#!/bin/bash
# Round-4 opening measurements on one MI355X: headline bench (noise and
# peak-heavy), 2^20 bench, and the golden tutorial command (5 repetitions,
# native and Python) for the per-stage comparison with the reference's
# published 2x C2070 execution times.
set -o pipefail
O=gpurun_out/r4base
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-160
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --signal > $O/bench_signal.log 2>&1 || { echo SIG_FAIL; tail -20 $O/bench_signal.log; exit 1; }
grep '^{"metric"' $O/bench_signal.log | cut -c1-160
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --log2n 20 > $O/bench20.log 2>&1 || { echo B20_FAIL; tail -20 $O/bench20.log; exit 1; }
grep '^{"metric"' $O/bench20.log | cut -c1-160
for i in 1 2 3 4 5; do
  timeout -k 10 120 ./bin/peasoup -i tests/data/tutorial.fil -o $O/golden_native_$i --dm_end 250 --acc_start -5 --acc_end 5 -n 4 --npdmp 10 > $O/golden_native_$i.log 2>&1 || { echo GOLDEN_NATIVE_FAIL; tail -20 $O/golden_native_$i.log; exit 1; }
done
for i in 1 2 3 4 5; do
  timeout -k 10 180 python -u -m peasoup_amd -i tests/data/tutorial.fil -o $O/golden_py_$i --dm_end 250 --acc_start -5 --acc_end 5 -n 4 --npdmp 10 > $O/golden_py_$i.log 2>&1 || { echo GOLDEN_PY_FAIL; tail -20 $O/golden_py_$i.log; exit 1; }
done
grep -h -A7 "<execution_times>" $O/golden_native_*/overview.xml | grep -v execution_times | tr -s ' ' | paste -sd' ' | head -c 2000
echo
echo DONE
