#!/bin/bash
# Config 4 after the setup-time table build / buffer reserve and the
# submit-then-pull block order: host timeline, configs 4 (x2) and 5, GPU tests
# of the search drivers, bench.
set -o pipefail
O=gpurun_out/r3c4f
mkdir -p $O
export TMPDIR=/tmp
rm -f $O/blocks.jsonl
PSOUP_BLOCK_TRACE=$O/blocks.jsonl timeout -k 10 400 python3 tools/baseline_configs.py --configs 4 --sky single --workdir /tmp/cfg --out $O/c4.jsonl > $O/c4.log 2>&1 || { echo C4_FAIL; tail -20 $O/c4.log; exit 1; }
timeout -k 10 400 python3 tools/baseline_configs.py --configs 4 --sky single --workdir /tmp/cfg --out $O/c4.jsonl > $O/c4b.log 2>&1 || { echo C4_FAIL; tail -20 $O/c4b.log; exit 1; }
timeout -k 10 400 python3 tools/baseline_configs.py --configs 4,5 --workdir /tmp/cfg --out $O/c45.jsonl > $O/c45.log 2>&1 || { echo C45_FAIL; tail -20 $O/c45.log; exit 1; }
cut -c1-330 $O/c4.jsonl $O/c45.jsonl
timeout -k 10 500 python -u -m pytest -m gpu -x -v --timeout 280 --timeout-method thread tests/test_pipeline_gpu.py tests/test_models_gpu.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-200
timeout -k 10 300 python -u bench.py --signal --steps 5 --warmup 2 > $O/bench_signal.log 2>&1 || { echo SIG_FAIL; tail -20 $O/bench_signal.log; exit 1; }
grep '^{"metric"' $O/bench_signal.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], {k:v for k,v in d["config"].items() if k.endswith("step")})'
echo DONE
