#!/bin/bash
# rocprofv3 kernel-trace + stats of the headline bench (1 GPU)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof/bench.log 2>&1
echo rc=$?
ls -R gpurun_out/prof | head -20
