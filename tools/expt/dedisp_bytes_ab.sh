#!/bin/bash
# LDS dedispersion: byte-lane sums vs 16-bit perm sums (PSOUP_DEDISP_LDS_BYTES), bit-exactness tests first.
set -o pipefail
mkdir -p gpurun_out/ddb
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "dedisp or golden or mfma" > gpurun_out/ddb/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/ddb/pytest.log; exit 1; }
tail -1 gpurun_out/ddb/pytest.log
for b in 0 1 0 1; do
  PSOUP_DEDISP_LDS_BYTES=$b timeout -k 10 200 python tools/dedisp_bench.py --samples 2 --reps 3 > gpurun_out/ddb/bench_$b.txt 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/ddb/bench_$b.txt; exit 1; }
  echo -n "bytes=$b "; tail -1 gpurun_out/ddb/bench_$b.txt
done
