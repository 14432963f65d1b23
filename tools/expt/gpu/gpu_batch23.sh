#!/bin/bash
# Headline batch size A/B on one box: the default (1376 = 5480 trials / 4
# batches), 2048 (3 batches) and 1024 (6 batches), alternating.
set -o pipefail
O=gpurun_out/${1:-batch23}
mkdir -p $O
for rep in 1 2 3; do
  for k in 0 2048 1024; do
    timeout -k 10 300 python3 bench.py --accel-batch $k > $O/b.log 2>&1 || { tail -10 $O/b.log; exit 1; }
    grep '^{"metric"' $O/b.log >> $O/k$k.jsonl
  done
done
for k in 0 2048 1024; do echo "batch $k: $(python3 -c "import json; print([json.loads(x)['value'] for x in open('$O/k$k.jsonl')])")"; done
echo DONE
