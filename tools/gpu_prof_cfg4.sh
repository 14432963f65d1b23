#!/bin/bash
# Config 4 (2026 DMs x 13 accelerations at 2^20, 1 GPU): plain run, then a
# rocprofv3 kernel trace of a second run (the synthetic .fil is reused).
set -o pipefail
mkdir -p gpurun_out/cfg4prof
timeout -k 10 300 python tools/baseline_configs.py --configs 4 --workdir /tmp/cfg4 --out gpurun_out/cfg4prof/plain.jsonl > gpurun_out/cfg4prof/plain.log 2>&1 || { echo PLAIN_FAIL; tail -20 gpurun_out/cfg4prof/plain.log; exit 1; }
tail -1 gpurun_out/cfg4prof/plain.jsonl
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/cfg4prof -o cfg4 --output-format csv -- python3 tools/baseline_configs.py --configs 4 --workdir /tmp/cfg4 --out gpurun_out/cfg4prof/prof.jsonl > gpurun_out/cfg4prof/prof.log 2>&1
echo rc=$?
tail -1 gpurun_out/cfg4prof/prof.jsonl; rm -f gpurun_out/cfg4prof/*kernel_trace.csv.gz
