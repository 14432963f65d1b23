#!/bin/bash
# Config 4 (Python, static shard) with 32 / 64 / 128-DM blocks, alternating.
set -o pipefail
O=gpurun_out/${1:-chunk}
mkdir -p $O /tmp/cfgw
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --workdir /tmp/cfgw > $O/warm.log 2>&1 || { tail -10 $O/warm.log; exit 1; }
for rep in 1 2; do
  for c in 32 64 128; do
    PSOUP_STATIC_CHUNK=$c timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --workdir /tmp/cfgw --out $O/c4_$c.jsonl > $O/c4.log 2>&1 || { tail -10 $O/c4.log; exit 1; }
  done
done
for c in 32 64 128; do echo "chunk $c:"; python3 tools/summarize_jsonl.py $O/c4_$c.jsonl timers_s.searching timers_s.total candidates best.snr; done
echo DONE
