#!/bin/bash
# Long series after the external-row path: 2^26 (default plan) and 2^27
# (+-100 m/s^2 so a step stays under a minute), one DM per step, with kernel
# tables; the external-row tests.   tools/expt/gpu/gpu_long8.sh OUT
set -o pipefail
O=gpurun_out/${1:-long8}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "beyond_one_grid or rows or packed2 or dedisp" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 500 python -u bench.py --log2n 26 --dms-per-gpu 1 --steps 2 --warmup 1 > $O/b26.log 2>&1 || { tail -20 $O/b26.log; exit 1; }
grep '^{"metric"' $O/b26.log > $O/b26.json; grep -o '"value": [0-9.]*' $O/b26.json
timeout -k 10 600 python -u bench.py --log2n 27 --acc 100 --dms-per-gpu 1 --steps 1 --warmup 1 > $O/b27.log 2>&1 || { tail -20 $O/b27.log; exit 1; }
grep '^{"metric"' $O/b27.log > $O/b27.json; grep -o '"value": [0-9.]*\|"accel_trials_per_dm": [0-9]*' $O/b27.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof27 -o b --output-format csv -- python3 bench.py --log2n 27 --acc 100 --dms-per-gpu 1 --steps 1 --warmup 0 > $O/prof27.log 2>&1 || { tail -20 $O/prof27.log; exit 1; }
rm -f $O/prof27/b_kernel_trace.csv
python3 tools/prof_summary.py $O/prof27/b_kernel_stats.csv 6
echo DONE
