#!/bin/bash
# Counter passes over tools/kbench.py (K trials per launch, 2^23): SQ
# instruction/wait mix and TCC memory-side traffic of the search kernels.
set -o pipefail
name=${1:-pmckb}; shift || true
export TMPDIR=/tmp
mkdir -p gpurun_out/$name
timeout -k 10 300 python3 tools/kbench.py --K 32 --reps 5 "$@" > gpurun_out/$name/kbench.log 2>&1 || { echo KBENCH_FAIL; tail -5 gpurun_out/$name/kbench.log; exit 1; }
cat gpurun_out/$name/kbench.log
run() {  # pass-name counters...
  local p=$1; shift
  timeout -k 10 -s KILL 240 rocprofv3 --pmc "$@" -d gpurun_out/$name/$p -o p --output-format csv -- python3 tools/kbench.py --K 32 --reps 2 > gpurun_out/$name/$p.log 2>&1 || { echo "PASS $p FAIL"; tail -5 gpurun_out/$name/$p.log; return 1; }
}
run a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE && \
run b SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM && \
run c TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_HIT_sum && \
run d TCC_MISS_sum TCC_REQ_sum TA_BUSY_avr TD_BUSY_avr && \
python3 tools/pmc_summary.py gpurun_out/$name/*/p_counter_collection.csv --match fft4_col,fft4_rowpass_kernel,fft4_rowpass_spectrum,r2c_interbin_tiled,harmonic_peaks_q8
