#!/bin/bash
# Final-tree evidence: per-step kernel tables (noise and --signal) and the per-rank step cost of an 8-rank job.
set -o pipefail
O=gpurun_out/r4trace_noise bash tools/gpu_r4_trace.sh || exit 1
O=gpurun_out/r4trace_signal bash tools/gpu_r4_trace.sh --signal || exit 1
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --as-rank 8:0,1,4,7 > gpurun_out/r4trace_noise/as_rank.log 2>&1 || { echo ASRANK_FAIL; tail -20 gpurun_out/r4trace_noise/as_rank.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4trace_noise/as_rank.log | cut -c1-300
echo DONE
