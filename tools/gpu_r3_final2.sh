#!/bin/bash
# Round-3 final check of the tree: GPU suite, smoke, bench x2 + kernel stats,
# same-box A/B against the previous commit's build (ab_old/), configs 3-5.
set -o pipefail
O=gpurun_out/r3final2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 280 --timeout-method thread tests/ > $O/pytest_gpu.log 2>&1 \
  || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  for v in new old; do
    D=.; [ $v = old ] && D=ab_old
    timeout -k 10 300 python -u $D/bench.py --steps 20 --warmup 5 > $O/bench_${v}_$r.log 2>&1 || { echo BENCH_FAIL $v; tail -20 $O/bench_${v}_$r.log; exit 1; }
    echo -n "$v rep $r: "; grep '^{"metric"' $O/bench_${v}_$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 bench.py --steps 5 --warmup 1 > $O/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof_bench.log; exit 1; }
grep '^{"metric"' $O/prof_bench.log | cut -c1-200
timeout -k 10 300 python -u bench.py --signal --steps 5 --warmup 2 > $O/bench_signal.log 2>&1 || { echo SIG_FAIL; tail -20 $O/bench_signal.log; exit 1; }
grep '^{"metric"' $O/bench_signal.log | cut -c1-200
timeout -k 10 400 python3 tools/baseline_configs.py --configs 4 --sky single --workdir /tmp/cfg --out $O/configs.jsonl > $O/c4.log 2>&1 || { echo C4_FAIL; tail -20 $O/c4.log; exit 1; }
timeout -k 10 400 python3 tools/baseline_configs.py --configs 3,5 --workdir /tmp/cfg --out $O/configs.jsonl > $O/c5.log 2>&1 || { echo C5_FAIL; tail -20 $O/c5.log; exit 1; }
cut -c1-400 $O/configs.jsonl
echo DONE
