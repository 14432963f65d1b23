#!/bin/bash
# SQ/TCC counters of the default fft4 passes, r2c and harmonic kernels (kbench, kernel-trace only).
set -o pipefail
name=${1:-pmc_fft}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/$name
run() {  # group-name counters...
  local g=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/$name/$g -o p --output-format csv -- python3 tools/kbench.py --K 32 --reps 2 --flags 81155 > gpurun_out/$name/$g.log 2>&1 || { echo "PMC_FAIL $g"; tail -5 gpurun_out/$name/$g.log; exit 1; }
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU
run b SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM
run c TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
run d FETCH_SIZE
run e WRITE_SIZE
python3 tools/pmc_summary.py $(find gpurun_out/$name -name "*counter_collection.csv") --match colpass,rowpass,r2c_interbin_tiled,harmonic_peaks > gpurun_out/$name/summary.txt 2>&1 || true
echo PMC_OK
