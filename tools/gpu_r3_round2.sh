#!/bin/bash
# Round-3 evidence run: full GPU suite, bench (noise / signal), kernel-stat
# profile, roctx marker trace of the native pipeline, configs 4 and 5.
set -o pipefail
O=gpurun_out/r3b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest -m gpu -x -v --timeout 280 --timeout-method thread tests/ > $O/pytest_gpu.log 2>&1 \
  || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-400
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --signal > $O/bench_signal.log 2>&1 || { echo SIGNAL_FAIL; tail -20 $O/bench_signal.log; exit 1; }
grep '^{"metric"' $O/bench_signal.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 bench.py --steps 5 --warmup 1 > $O/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof_bench.log; exit 1; }
grep '^{"metric"' $O/prof_bench.log | cut -c1-200
timeout -k 10 300 python -u tools/baseline_configs.py --configs 4,5 --out $O/configs.jsonl > $O/configs.log 2>&1 || { echo CONFIGS_FAIL; tail -30 $O/configs.log; exit 1; }
cut -c1-600 $O/configs.jsonl
F=$(ls gpurun_out/configs/cfg45_20_multi.fil)
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d $O/prof_marker -o marker -- ./bin/peasoup -i $F -o $O/out_marker --dm_end 100 --acc_start -500 --acc_end 500 -n 3 --npdmp 32 > $O/prof_marker.log 2>&1 || { echo MARKER_FAIL; tail -20 $O/prof_marker.log; exit 1; }
tail -3 $O/prof_marker.log
echo DONE
