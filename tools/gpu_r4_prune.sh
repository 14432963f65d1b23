#!/bin/bash
# After the FFT4 flag prune: kernel tests (all flag sets, no skips), short bench,
# 2^20 bench + kernel stats; then the async/golden/config script.
set -o pipefail
O=gpurun_out/r4prune
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_screen_gpu.py tests/test_kernels_gpu.py > $O/pytest_kernels.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest_kernels.log | head; tail -30 $O/pytest_kernels.log; exit 1; }
tail -1 $O/pytest_kernels.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-200
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --harm-flags 2597 > $O/bench_noscreen.log 2>&1 || { echo BENCH_NS_FAIL; tail -20 $O/bench_noscreen.log; exit 1; }
grep '^{"metric"' $O/bench_noscreen.log | cut -c1-200
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --harm-flags 2601 > $O/bench_fromx.log 2>&1 || { echo BENCH_FX_FAIL; tail -20 $O/bench_fromx.log; exit 1; }
grep '^{"metric"' $O/bench_fromx.log | cut -c1-200
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench2.log 2>&1 || { echo BENCH2_FAIL; tail -20 $O/bench2.log; exit 1; }
grep '^{"metric"' $O/bench2.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof23 -o run -- python3 bench.py --steps 5 --warmup 1 > $O/prof23.log 2>&1 || { echo PROF23_FAIL; tail -20 $O/prof23.log; exit 1; }
find $O/prof23 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/k23_stats.csv
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
timeout -k 10 300 python -u bench.py --signal --steps 4 --warmup 2 > $O/bench_sig.log 2>&1 || { echo BENCH_SIG_FAIL; tail -20 $O/bench_sig.log; exit 1; }
grep '^{"metric"' $O/bench_sig.log | cut -c1-200
timeout -k 10 300 python -u bench.py --signal --steps 4 --warmup 2 --harm-flags 2597 > $O/bench_sig_ns.log 2>&1 || { echo BENCH_SIGNS_FAIL; tail -20 $O/bench_sig_ns.log; exit 1; }
grep '^{"metric"' $O/bench_sig_ns.log | cut -c1-200
timeout -k 10 300 python -u bench.py --signal --steps 4 --warmup 2 --harm-flags 2601 > $O/bench_sig_fx.log 2>&1 || { echo BENCH_SIGFX_FAIL; tail -20 $O/bench_sig_fx.log; exit 1; }
grep '^{"metric"' $O/bench_sig_fx.log | cut -c1-200
timeout -k 10 300 python -u tools/kbench.py --K 32 --reps 10 --flags 1073954051 > $O/kbench.log 2>&1 || { echo KBENCH_FAIL; tail -20 $O/kbench.log; exit 1; }
cat $O/kbench.log | tail -14
echo DONE
