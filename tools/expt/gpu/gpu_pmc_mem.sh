#!/bin/bash
# Memory-pipeline counters (TA/TCP/TD/UTCL1/TCC) of the production bench kernels, one pass each.
set -o pipefail
name=${1:-pmcmem}; shift || true
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/$name
run() {  # pass-name counters...
  local p=$1; shift
  timeout -k 10 -s KILL 180 rocprofv3 --pmc "$@" -d gpurun_out/$name/$p -o p --output-format csv -- python3 bench.py --steps 1 --warmup 0 --sub-batch 0 --dms-per-gpu 1 > gpurun_out/$name/$p.log 2>&1 || { echo "PASS $p FAIL"; tail -5 gpurun_out/$name/$p.log; return 1; }
}
run a TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE && \
run b TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_TCR_TCP_STALL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum && \
run c TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_TAG_STALL_sum TCC_BUSY_sum && \
python3 tools/pmc_summary.py gpurun_out/$name/*/p_counter_collection.csv --match fft4_col,fft4_row,r2c_inter,harmonic_peaks
