#!/bin/bash
# Pass-A phase stamps (default / compute-only), SQ counters of pass A, and a
# kernel trace of config 5 (fold stage).
set -o pipefail
O=gpurun_out/r3tr
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/expt/fft4_trace.py > $O/trace_default.txt 2>&1 && cat $O/trace_default.txt || { echo TRACE_FAIL; tail $O/trace_default.txt; exit 1; }
timeout -k 10 120 python -u tools/expt/fft4_trace.py 212419 > $O/trace_compute.txt 2>&1 && cat $O/trace_compute.txt || { echo TRACE2_FAIL; tail $O/trace_compute.txt; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU --kernel-trace --output-format csv -d $O/pmc_a -o pa -- python3 tools/expt/passa_phases.py --only-full --extra 0,192 > $O/pmc_a.log 2>&1 || { echo PMC_FAIL; tail $O/pmc_a.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 tools/baseline_configs.py --configs 5 --workdir /tmp/cfg --out $O/c5.jsonl > $O/c5.log 2>&1 || { echo C5_FAIL; tail -20 $O/c5.log; exit 1; }
cut -c1-900 $O/c5.jsonl
echo DONE
