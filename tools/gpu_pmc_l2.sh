#!/bin/bash
# L2 hit/miss + SQ busy counters per hot kernel (kernel-trace only).
set -o pipefail
name=${1:-pmcl2}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/$name
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_WAVES -d gpurun_out/$name/l2 -o p --output-format csv -- python3 tools/kbench.py --K 32 --reps 2 --flags 15619 > gpurun_out/$name/l2.log 2>&1 || { echo L2_FAIL; tail -5 gpurun_out/$name/l2.log; exit 1; }
echo PMC_OK
