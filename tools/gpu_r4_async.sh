#!/bin/bash
# BASELINE configs 4/5 (Python driver), config 5 at 2^23, config 4 single sky, golden command x5 (native + Python).
set -o pipefail
O=gpurun_out/r4async
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_pipeline_gpu.py tests/test_models_gpu.py > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python3 tools/baseline_configs.py --configs 4,5 --workdir /tmp/cfg --out $O/c45.jsonl > $O/c45.log 2>&1 || { echo C45_FAIL; tail -20 $O/c45.log; exit 1; }
python3 -c "
import json
for l in open('$O/c45.jsonl'):
    d=json.loads(l); r=d['rank_stats'][0]
    print(d['config'], d['timers_s'], {k: r[k] for k in ('host_s','accd_s','tail_s','gpu_distilled','host_distilled')})
"
timeout -k 10 500 python3 tools/baseline_configs.py --configs 4,5 --native --workdir /tmp/cfg --out $O/c45_native.jsonl > $O/c45n.log 2>&1 || { echo C45N_FAIL; tail -20 $O/c45n.log; exit 1; }
cut -c1-400 $O/c45_native.jsonl
timeout -k 10 500 python3 tools/baseline_configs.py --configs 4 --sky single --workdir /tmp/cfg --out $O/c4single.jsonl > $O/c4s.log 2>&1 || { echo C4S_FAIL; tail -20 $O/c4s.log; exit 1; }
python3 -c "
import json
for l in open('$O/c4single.jsonl'):
    d=json.loads(l); print('single', d['config'], d['timers_s'])
"
timeout -k 10 600 python3 tools/baseline_configs.py --configs 5 --log2n 23 --workdir /tmp/cfg23 --out $O/c5_23.jsonl > $O/c5_23.log 2>&1 || { echo C5_23_FAIL; tail -20 $O/c5_23.log; exit 1; }
cut -c1-300 $O/c5_23.jsonl
for i in 1 2 3 4 5; do
  timeout -k 10 120 ./bin/peasoup -i tests/data/tutorial.fil -o $O/golden_native_$i --dm_end 250 --acc_start -5 --acc_end 5 -n 4 --npdmp 10 > $O/golden_native_$i.log 2>&1 || { echo GOLDEN_NATIVE_FAIL; tail -20 $O/golden_native_$i.log; exit 1; }
done
for i in 1 2 3 4 5; do
  timeout -k 10 180 python -u -m peasoup_amd -i tests/data/tutorial.fil -o $O/golden_py_$i --dm_end 250 --acc_start -5 --acc_end 5 -n 4 --npdmp 10 > $O/golden_py_$i.log 2>&1 || { echo GOLDEN_PY_FAIL; tail -20 $O/golden_py_$i.log; exit 1; }
done
for f in $O/golden_native_*/overview.xml $O/golden_py_*/overview.xml; do echo $f; grep -A6 "<execution_times>" $f | grep -v execution_times | tr -s ' ' | paste -sd' '; done
echo DONE
