#!/bin/bash
# External-row FFT path (2^26 and up): its tests, the transposing r2c alone,
# the 2^26 bench and its kernel table.   tools/expt/gpu/gpu_rows26.sh OUT
set -o pipefail
O=gpurun_out/${1:-rows26}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "rows or fft4_resample_spectrum" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 200 python tools/expt/r2c_rows_probe.py > $O/probe.log 2>&1 || { tail -10 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log
timeout -k 10 500 python -u bench.py --log2n 26 --dms-per-gpu 1 --steps 2 --warmup 1 > $O/b26.log 2>&1 || { tail -20 $O/b26.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/b26.log
bash tools/expt/gpu/gpu_prof26.sh ${1:-rows26}/prof
