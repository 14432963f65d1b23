#!/bin/bash
# After the FFT4 flag prune: kernel tests (all flag sets, no skips), short bench,
# 2^20 bench + kernel stats; then the async/golden/config script.
set -o pipefail
O=gpurun_out/r4prune
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_kernels_gpu.py > $O/pytest_kernels.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest_kernels.log | head; tail -30 $O/pytest_kernels.log; exit 1; }
tail -1 $O/pytest_kernels.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-200
timeout -k 10 300 python -u bench.py --log2n 20 --dms-per-gpu 32 --steps 20 --warmup 3 > $O/bench20.log 2>&1 || { echo BENCH20_FAIL; tail -20 $O/bench20.log; exit 1; }
grep '^{"metric"' $O/bench20.log | cut -c1-1200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof20 -o run -- python3 bench.py --log2n 20 --dms-per-gpu 32 --steps 20 --warmup 3 > $O/prof20.log 2>&1 || { echo PROF20_FAIL; tail -20 $O/prof20.log; exit 1; }
find $O/prof20 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/k20_stats.csv
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r4prune/k20_stats.csv')))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:18]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):6d} {100*float(r['TotalDurationNs'])/tot:5.1f}% {r['Name'][:90]}")
PY
bash tools/gpu_r4_async.sh
