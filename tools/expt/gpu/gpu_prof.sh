#!/bin/bash
# rocprofv3 kernel-trace + stats of the headline bench (1 GPU).
# usage: tools/expt/gpu/gpu_prof.sh [outdir-name] [extra bench args...]
set -o pipefail
name=${1:-prof}; shift || true
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/$name
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$name -o bench --output-format csv -- python3 bench.py --steps 2 --warmup 1 "$@" > gpurun_out/$name/bench.log 2>&1
rc=$?
echo rc=$rc
tail -1 gpurun_out/$name/bench.log
exit $rc
