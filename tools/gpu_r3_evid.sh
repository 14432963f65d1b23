#!/bin/bash
# Round-3 evidence (second pass): --signal sweep, bench kernel stats, configs
# 4/5 (filterbank in /tmp, not under gpurun_out), roctx marker trace of bin/peasoup.
set -o pipefail
O=gpurun_out/r3c
W=/tmp/psoup_cfg
mkdir -p $O $W
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_kernels_gpu.py -k "1024ch or fold" > $O/pytest_k.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
O=$O bash tools/gpu_r3_sig.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 bench.py --steps 5 --warmup 1 > $O/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof_bench.log; exit 1; }
grep '^{"metric"' $O/prof_bench.log | cut -c1-200
timeout -k 10 400 python -u tools/baseline_configs.py --configs 4,5 --workdir $W --out $O/configs.jsonl > $O/configs.log 2>&1 || { echo CONFIGS_FAIL; tail -30 $O/configs.log; exit 1; }
cut -c1-400 $O/configs.jsonl
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d $O/prof_marker -o marker -- ./bin/peasoup -i $W/cfg45_20_multi.fil -o $W/out_marker --dm_end 100 --acc_start -500 --acc_end 500 -n 3 --npdmp 32 > $O/prof_marker.log 2>&1 || { echo MARKER_FAIL; tail -20 $O/prof_marker.log; exit 1; }
find $O/prof_marker -name "*stats*"
echo DONE
