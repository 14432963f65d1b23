#!/bin/bash
# Cluster kernel on RFI-like dense segments: timing and SQ counters.
set -o pipefail
O=gpurun_out/r4clpmc
mkdir -p $O
export TMPDIR=/tmp
for n in 4200 9000 12000; do timeout -k 10 120 python -u tools/expt/cluster_bench.py --dense --n $n --nseg 2048 > $O/cbd_$n.log 2>&1 || { echo CB_FAIL; tail -5 $O/cbd_$n.log; exit 1; }; tail -1 $O/cbd_$n.log; done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU -d $O/sq -o p --output-format csv -- python3 tools/expt/cluster_bench.py --dense --n 9000 --reps 2 > $O/sq.log 2>&1 || { echo SQ_FAIL; tail -5 $O/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM -d $O/lds -o p --output-format csv -- python3 tools/expt/cluster_bench.py --dense --n 9000 --reps 2 > $O/lds.log 2>&1 || { echo LDS_FAIL; tail -5 $O/lds.log; exit 1; }
python3 tools/pmc_summary.py $(find $O/sq $O/lds -name "*counter_collection.csv") --match "peak_cluster_kernel<14000,peak_cluster_kernel<4096,seg_scatter" > $O/pmc.txt; cat $O/pmc.txt
echo DONE
