#!/bin/bash
# 2^20 sub-batch size A/B (32 DMs x 13 trials per step, one 416-trial batch):
# auto (256), 208 (two equal halves), 128, 104 and none, alternating.
set -o pipefail
O=gpurun_out/${1:-sub20}
mkdir -p $O
for rep in 1 2 3; do
  for sb in -1 208 128 104 0; do
    timeout -k 10 300 python3 bench.py --log2n 20 --dms-per-gpu 32 --steps 20 --warmup 3 --sub-batch $sb > $O/b.log 2>&1 || { tail -10 $O/b.log; exit 1; }
    grep '^{"metric"' $O/b.log >> $O/sb$sb.jsonl
  done
done
for sb in -1 208 128 104 0; do echo "sub $sb: $(python3 -c "import json; print([json.loads(x)['value'] for x in open('$O/sb$sb.jsonl')])")"; done
echo DONE
