#!/bin/bash
# Multi-rank rehearsal on one GPU (gloo, every rank on GPU 0): bench.py at
# world 2 and 4 (noise and --signal), under gpurun_out/$1.  The timings are
# of ranks sharing one GPU; what they check is the merge path (gather to rank
# 0, merge there) and its cost per step.  World 4 uses 512-trial batches:
# four ranks' default batch budgets (each sized from the free memory it saw at
# start-up) do not fit one GPU together.
set -o pipefail
O=gpurun_out/${1:-multirank}
mkdir -p $O
export TMPDIR=/tmp PSOUP_DIST_BACKEND=gloo
for w in 2 4; do
  for sig in "" "--peak-heavy"; do
    tag=w${w}${sig:+_signal}
    timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 --master-port $((29600 + w)) bench.py --gpus $w --steps 3 --warmup 1 $sig $([ $w -gt 2 ] && echo --accel-batch 512) > $O/$tag.log 2>&1 || { echo FAIL_$tag; tail -20 $O/$tag.log; exit 1; }
    grep '^{"metric"' $O/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$tag', d['value'], d['ms_per_step'], 'merge', c['merge_s_per_step'], 'work', c['merge_work_s_per_step'], c['merge_split_s'], 'blob', c['candidate_blob_bytes'])"
  done
done
