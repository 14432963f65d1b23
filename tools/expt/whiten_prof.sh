#!/bin/bash
# Isolated per-DM work at 2^20 (tools/expt/whiten_bench.py), plain and under rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out/whiten
timeout -k 10 300 python -u tools/expt/whiten_bench.py "$@" > gpurun_out/whiten/plain.txt 2>&1 || { echo FAIL; tail -20 gpurun_out/whiten/plain.txt; exit 1; }
cat gpurun_out/whiten/plain.txt | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/whiten -o w --output-format csv -- python3 tools/expt/whiten_bench.py "$@" > gpurun_out/whiten/prof.txt 2>&1
echo rc=$?
rm -f gpurun_out/whiten/w_kernel_trace.csv
