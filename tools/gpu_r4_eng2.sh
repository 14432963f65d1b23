#!/bin/bash
# Engines 1 vs 3 (Python driver), configs 4/5 many-pulsar sky and 4 single pulsar, alternating, two rounds.
set -o pipefail
O=gpurun_out/r4eng2
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for e in 1 3; do
    PSOUP_ENGINES=$e timeout -k 10 300 python3 tools/baseline_configs.py --configs 4,5 --workdir /tmp/cfg --out $O/c45_e${e}_r$r.jsonl > $O/c45_e${e}_r$r.log 2>&1 || { echo C45_FAIL $e; tail -20 $O/c45_e${e}_r$r.log; exit 1; }
    PSOUP_ENGINES=$e timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --sky single --workdir /tmp/cfg --out $O/c4s_e${e}_r$r.jsonl > $O/c4s_e${e}_r$r.log 2>&1 || { echo C4S_FAIL $e; tail -20 $O/c4s_e${e}_r$r.log; exit 1; }
    python3 -c "
import json
for f in ['$O/c45_e${e}_r$r.jsonl','$O/c4s_e${e}_r$r.jsonl']:
    for l in open(f):
        d=json.loads(l); print('engines $e round $r', f.split('/')[-1][:4], d['config'], 'search', d['timers_s']['searching'], 'total', d['timers_s']['total'])
"
  done
done
echo DONE
