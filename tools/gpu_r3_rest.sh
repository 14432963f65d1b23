#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread \
  tests/test_pipeline_gpu.py::test_headline_shape_binary_pulsar_and_fft_modes > gpurun_out/r3/pytest_headline.log 2>&1 \
  || { echo PYTEST_FAIL; tail -30 gpurun_out/r3/pytest_headline.log; exit 1; }
tail -1 gpurun_out/r3/pytest_headline.log
timeout -k 10 300 python -u tools/dedisp_bench.py --ndm 2000 --log2n 20 --reps 3 > gpurun_out/r3/dedisp_bench.jsonl 2>&1 || { echo DEDISP_FAIL; tail -20 gpurun_out/r3/dedisp_bench.jsonl; exit 1; }
cat gpurun_out/r3/dedisp_bench.jsonl
timeout -k 10 300 bash tools/scale8.sh 5 1 > gpurun_out/r3/scale8_n1.txt 2>&1 || { echo SCALE_FAIL; cat gpurun_out/r3/scale8_n1.txt; exit 1; }
cut -c1-160 gpurun_out/r3/scale8_n1.txt
export TMPDIR=/tmp
PSOUP_FORCE_PG=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29777 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/prof_forcepg -o forcepg -- python bench.py --steps 3 --warmup 1 > gpurun_out/r3/bench_forcepg.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/r3/bench_forcepg.log; exit 1; }
grep '^{"metric"' gpurun_out/r3/bench_forcepg.log | cut -c1-200
timeout -k 10 120 python -u tools/expt/fft4_trace.py > gpurun_out/r3/fft4_trace_default.txt 2>&1 && cat gpurun_out/r3/fft4_trace_default.txt
