#!/bin/bash
# Counter passes over one bench step (DMS DMs x 685 trials at 2^23; default 8,
# the headline bench's step):
# memory-side traffic (TCC_EA0 read/write requests, DRAM vs Infinity-Cache
# hits) and the SQ instruction/wait mix of every search kernel.  One rocprofv3
# --pmc run per pass (no other trace domains), each under its own time limit.
set -o pipefail
name=${1:-pmcbench}; shift || true
DMS=${DMS:-8}
export TMPDIR=/tmp
mkdir -p gpurun_out/$name
run() {  # pass-name counters...
  local p=$1; shift
  timeout -k 10 -s KILL 240 rocprofv3 --pmc "$@" -d gpurun_out/$name/$p -o p --output-format csv -- python3 bench.py --steps 1 --warmup 0 --dms-per-gpu $DMS > gpurun_out/$name/$p.log 2>&1 || { echo "PASS $p FAIL"; tail -5 gpurun_out/$name/$p.log; return 1; }
}
run m1 TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum && \
run m2 TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum && \
run s1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE && \
python3 tools/pmc_summary.py gpurun_out/$name/m1/p_counter_collection.csv gpurun_out/$name/m2/p_counter_collection.csv --match fft4_col,fft4_rowpass_spectrum,harmonic_peaks_q8,dedisperse --per $((DMS * 685)) > gpurun_out/$name/per_trial.txt && cat gpurun_out/$name/per_trial.txt && python3 tools/pmc_summary.py gpurun_out/$name/s1/p_counter_collection.csv --match fft4_col,fft4_rowpass_spectrum,harmonic_peaks_q8,dedisperse > gpurun_out/$name/sq_per_dispatch.txt
