#!/bin/bash
# Sub-batch pipeline sweep: headline bench with PSOUP_SUB_BATCH = each arg
# (0 = off), plus the multi-stream search equality test first.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_pipeline_gpu.py -x -q > gpurun_out/pytest_pipe.log 2>&1 || { echo PIPE_FAIL; tail -40 gpurun_out/pytest_pipe.log; exit 1; }
tail -1 gpurun_out/pytest_pipe.log
for sb in "$@"; do
  PSOUP_SUB_BATCH=$sb timeout -k 10 300 python bench.py --steps 2 --warmup 1 > gpurun_out/bench_sb$sb.log 2>&1 || { echo BENCH_FAIL $sb; tail -30 gpurun_out/bench_sb$sb.log; exit 1; }
  echo -n "sub=$sb "; tail -1 gpurun_out/bench_sb$sb.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
done
