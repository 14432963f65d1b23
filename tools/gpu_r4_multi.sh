#!/bin/bash
# Two ranks on the one GPU (gloo collectives): the bench's multi-rank path (candidate gather, merge) end to end.
set -o pipefail
O=gpurun_out/r4multi
mkdir -p $O
export TMPDIR=/tmp
PSOUP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 4 --warmup 2 > $O/bench2.log 2>&1 || { echo MULTI_FAIL; tail -30 $O/bench2.log; exit 1; }
grep '^{"metric"' $O/bench2.log | cut -c1-400
echo DONE
