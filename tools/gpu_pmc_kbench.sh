#!/bin/bash
# SQ counters for the hot kernels via the microbenchmark (kernel-trace only, no other tracing).
set -o pipefail
name=${1:-pmck}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/$name
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU -d gpurun_out/$name/sq -o p --output-format csv -- python3 tools/kbench.py --K 32 --reps 3 --flags 275 > gpurun_out/$name/sq.log 2>&1 || { echo SQ_FAIL; tail -5 gpurun_out/$name/sq.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM -d gpurun_out/$name/lds -o p --output-format csv -- python3 tools/kbench.py --K 32 --reps 3 --flags 275 > gpurun_out/$name/lds.log 2>&1 || { echo LDS_FAIL; tail -5 gpurun_out/$name/lds.log; exit 1; }
echo PMC_OK
