#!/bin/bash
# Evidence for docs/PERF_NOTES.md: fft4 phase timeline, per-kernel microbenchmark,
# load/store-pattern microbenchmarks, r2c+harmonic grouping.
set -o pipefail
mkdir -p gpurun_out/evidence
timeout -k 10 200 python tools/expt/fft4_trace.py > gpurun_out/evidence/fft4_trace.txt 2>&1 || { echo TRACE_FAIL; exit 1; }
timeout -k 10 200 python tools/kbench.py --K 32 --reps 20 --flags 81155 > gpurun_out/evidence/kbench.txt 2>&1 || { echo KB_FAIL; exit 1; }
timeout -k 10 100 ./tools/expt/bin/load_pattern 32 > gpurun_out/evidence/load_pattern.txt 2>&1 || { echo LP_FAIL; exit 1; }
timeout -k 10 100 ./tools/expt/bin/store_pattern 32 > gpurun_out/evidence/store_pattern.txt 2>&1 || { echo SP_FAIL; exit 1; }
timeout -k 10 200 python tools/expt/harm_group.py > gpurun_out/evidence/harm_group.txt 2>&1 || { echo HG_FAIL; exit 1; }
timeout -k 10 300 python tools/mallbench.py --Ks 1,4,8,32 > gpurun_out/evidence/mallbench.txt 2>&1 || { echo MB_FAIL; exit 1; }
echo EVIDENCE_OK
