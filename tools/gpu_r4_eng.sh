#!/bin/bash
# Config 4 search time vs engines per GPU (Python driver and native), after the round-4 kernels.
set -o pipefail
O=gpurun_out/r4eng
mkdir -p $O
export TMPDIR=/tmp
for e in 1 2 3 4; do
  PSOUP_ENGINES=$e timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --workdir /tmp/cfg --out $O/c4_py_e$e.jsonl > $O/c4_py_e$e.log 2>&1 || { echo C4_FAIL $e; tail -20 $O/c4_py_e$e.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_py_e$e.jsonl').readline()); print('python engines $e', d['timers_s'])"
done
for e in 1 2 3; do
  PSOUP_ENGINES=$e timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --native --workdir /tmp/cfg --out $O/c4_nat_e$e.jsonl > $O/c4_nat_e$e.log 2>&1 || { echo C4N_FAIL $e; tail -20 $O/c4_nat_e$e.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_nat_e$e.jsonl').readline()); print('native engines $e', d['timers_s'])"
done
echo DONE
