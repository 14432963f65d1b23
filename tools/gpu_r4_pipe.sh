#!/bin/bash
set -o pipefail
O=gpurun_out/r4pipe
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --signal > $O/bench_signal.log 2>&1 || { echo SIG_FAIL; tail -20 $O/bench_signal.log; exit 1; }
grep '^{"metric"' $O/bench_signal.log | cut -c1-120; grep -o '"search_s_per_step.*' $O/bench_signal.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --signal --serial-merge > $O/bench_signal_serial.log 2>&1 || { echo SIG2_FAIL; tail -20 $O/bench_signal_serial.log; exit 1; }
grep '^{"metric"' $O/bench_signal_serial.log | cut -c1-120
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-120
echo DONE
