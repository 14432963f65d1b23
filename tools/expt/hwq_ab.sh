#!/bin/bash
# Same-box bench A/B: HIP hardware queues per process (GPU_MAX_HW_QUEUES, default 4)
# x sub-batch streams (PSOUP_SUB_STREAMS), interleaved.  Args: "HWQ:STREAMS" ...
set -o pipefail
mkdir -p gpurun_out/hwq
for r in 1 2; do
  for cfg in "$@"; do
    q=${cfg%%:*}; ns=${cfg##*:}
    GPU_MAX_HW_QUEUES=$q PSOUP_SUB_STREAMS=$ns timeout -k 10 300 python bench.py --steps 3 > gpurun_out/hwq/q${q}_s${ns}_$r.log 2>&1 || { echo FAIL $cfg; tail -5 gpurun_out/hwq/q${q}_s${ns}_$r.log; exit 1; }
    echo -n "hwq=$q streams=$ns rep=$r "; tail -1 gpurun_out/hwq/q${q}_s${ns}_$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
  done
done
