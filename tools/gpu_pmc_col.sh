#!/bin/bash
# Memory-side counters of the fft4 column pass (kbench, kernel-trace only, one pass per group).
set -o pipefail
name=${1:-pmc_col}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/$name
run() {
  local g=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/$name/$g -o p --output-format csv -- python3 tools/kbench.py --K 32 --reps 2 --flags 81155 > gpurun_out/$name/$g.log 2>&1 || { echo "PMC_FAIL $g"; tail -5 gpurun_out/$name/$g.log; exit 1; }
}
run a TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum
run b TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum
run c TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum
run d SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
python3 tools/pmc_summary.py $(find gpurun_out/$name -name "*counter_collection.csv") --match colpass,rowpass > gpurun_out/$name/summary.txt 2>&1 || true
echo PMC_OK
