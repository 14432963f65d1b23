#!/bin/bash
# BASELINE configs 4/5 (Python and native drivers, 2^20) and the shorter
# bench sizes, written under gpurun_out/$1.
set -o pipefail
O=gpurun_out/${1:-configs}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 tools/baseline_configs.py --configs 4,5 --workdir /tmp/cfg --out $O/c45.jsonl > $O/c45.log 2>&1 || { echo C45_FAIL; tail -20 $O/c45.log; exit 1; }
python3 -c "
import json
for l in open('$O/c45.jsonl'):
    d=json.loads(l); print('py', d['config'], d['timers_s'])
"
timeout -k 10 500 python3 tools/baseline_configs.py --configs 4,5 --native --workdir /tmp/cfg --out $O/c45_native.jsonl > $O/c45n.log 2>&1 || { echo C45N_FAIL; tail -20 $O/c45n.log; exit 1; }
python3 -c "
import json
for l in open('$O/c45_native.jsonl'):
    d=json.loads(l); print('native', d['config'], d['timers_s'], {k: round(v, 4) for k, v in d['performance'].items() if k.endswith('_s')})
"
for l in 20 21 22; do
  timeout -k 10 300 python -u bench.py --log2n $l --dms-per-gpu 32 --steps 5 --warmup 1 > $O/bench_$l.log 2>&1 || { echo BENCH_${l}_FAIL; tail -20 $O/bench_$l.log; exit 1; }
  grep '^{"metric"' $O/bench_$l.log | cut -c100-200
done
echo DONE
