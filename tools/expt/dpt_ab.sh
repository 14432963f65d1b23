#!/bin/bash
# Headline bench A/B of the LDS dedispersion's DMs per wave for the 8-DM chunk
# (PSOUP_DEDISP_LDS_DPT=4 forces the 16-DM workgroups), after the dedispersion tests.
set -o pipefail
mkdir -p gpurun_out/dpt
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "dedisp or golden or mfma" > gpurun_out/dpt/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/dpt/pytest.log; exit 1; }
tail -1 gpurun_out/dpt/pytest.log
for r in 1 2; do
  for d in 4 0; do
    if [ $d = 0 ]; then unset PSOUP_DEDISP_LDS_DPT; else export PSOUP_DEDISP_LDS_DPT=$d; fi
    timeout -k 10 300 python bench.py --steps 3 > gpurun_out/dpt/d${d}_$r.log 2>&1 || { echo FAIL $d; tail -5 gpurun_out/dpt/d${d}_$r.log; exit 1; }
    echo -n "dpt_env=$d rep=$r "; tail -1 gpurun_out/dpt/d${d}_$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
  done
done
