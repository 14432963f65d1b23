#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --log2n 20 --steps 2 --warmup 1 > gpurun_out/bench20.log 2>&1 || { echo B20_FAIL; tail -30 gpurun_out/bench20.log; exit 1; }
tail -2 gpurun_out/bench20.log
timeout -k 10 400 python bench.py > gpurun_out/bench23.log 2>&1 || { echo B23_FAIL; tail -30 gpurun_out/bench23.log; exit 1; }
tail -2 gpurun_out/bench23.log
