#!/bin/bash
# Headline scaling curve on ONE node: bench.py at 1/2/4/8 ranks (one rank per
# GPU under torch.distributed.run, RCCL over xGMI), one JSON line per N.
#   tools/expt/gpu/scale8.sh [steps] [warmup] [extra bench.py args...]
# Needs >= 8 visible MI355X for the N = 8 point (smaller N run regardless).
set -o pipefail
STEPS=${1:-10}; WARM=${2:-2}; shift 2 2>/dev/null
NGPU=$(python -c 'import torch; print(torch.cuda.device_count())')
mkdir -p gpurun_out/scale8
for N in 1 2 4 8; do
  if [ "$N" -gt "$NGPU" ]; then echo "{\"n_gpus\": $N, \"skipped\": \"only $NGPU GPUs visible\"}"; continue; fi
  PORT=$((29600 + N))
  if [ "$N" -eq 1 ]; then
    timeout -k 10 900 python bench.py --gpus 1 --steps "$STEPS" --warmup "$WARM" "$@" \
      > gpurun_out/scale8/bench_n$N.log 2>&1 || { echo "{\"n_gpus\": $N, \"failed\": true}"; tail -5 gpurun_out/scale8/bench_n$N.log >&2; exit 1; }
  else
    timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
      --master-port "$PORT" bench.py --gpus "$N" --steps "$STEPS" --warmup "$WARM" "$@" \
      > gpurun_out/scale8/bench_n$N.log 2>&1 || { echo "{\"n_gpus\": $N, \"failed\": true}"; tail -5 gpurun_out/scale8/bench_n$N.log >&2; exit 1; }
  fi
  grep '^{"metric"' gpurun_out/scale8/bench_n$N.log | tail -1
done
