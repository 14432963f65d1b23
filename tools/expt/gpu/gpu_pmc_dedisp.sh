#!/bin/bash
# PMC passes over tools/dedisp_bench.py (MFMA / LDS packed-byte kernels).
set -o pipefail
name=${1:-pmc_dd}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/$name
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU -d gpurun_out/$name/sq -o p --output-format csv -- python3 tools/dedisp_bench.py --samples 2 --reps 1 > gpurun_out/$name/sq.log 2>&1 || { echo SQ_FAIL; tail -20 gpurun_out/$name/sq.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE -d gpurun_out/$name/tcc -o p --output-format csv -- python3 tools/dedisp_bench.py --samples 2 --reps 1 > gpurun_out/$name/tcc.log 2>&1 || { echo TCC_FAIL; tail -20 gpurun_out/$name/tcc.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE TCC_MISS_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE -d gpurun_out/$name/wr -o p --output-format csv -- python3 tools/dedisp_bench.py --samples 2 --reps 1 > gpurun_out/$name/wr.log 2>&1 || { echo WR_FAIL; tail -20 gpurun_out/$name/wr.log; exit 1; }
echo PMC_OK
