#!/bin/bash
# Config 4 (Python) with 2 / 4 / 8 acceleration-distillation host workers
# (PSOUP_ACCD_THREADS), alternating, and one kernel trace's idle gaps at 8.
set -o pipefail
O=gpurun_out/${1:-accd}
mkdir -p $O /tmp/cfgw
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --workdir /tmp/cfgw > $O/warm.log 2>&1 || { tail -10 $O/warm.log; exit 1; }
for rep in 1 2; do
  for w in 2 4 8; do
    PSOUP_ACCD_THREADS=$w timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --workdir /tmp/cfgw --out $O/c4_w$w.jsonl > $O/c4.log 2>&1 || { tail -10 $O/c4.log; exit 1; }
  done
done
for w in 2 4 8; do python3 tools/summarize_jsonl.py $O/c4_w$w.jsonl timers_s.searching timers_s.total rank_stats.0.accd_s; done
echo DONE
