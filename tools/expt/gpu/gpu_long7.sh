#!/bin/bash
# Long-series pass A changes: fused-FFT numerics tests (2^25 included), the
# 2^25 phase trace, one bench step at 2^25, the Stockham wide-store A/B at
# 2^20 / 2^22 / 2^25 and the 2^20 bench.   tools/expt/gpu/gpu_long7.sh OUT
set -o pipefail
O=gpurun_out/${1:-long7}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_spectrum_gpu.py -k "fft4 or resample or spectrum" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for L in 20 22 25; do
  for f in 1076313347 1084701955; do
    timeout -k 10 120 python tools/kbench_fused.py --log2n $L --K 16 --flags $f > $O/kb.log 2>&1 || { tail -5 $O/kb.log; exit 1; }
    grep flags= $O/kb.log | tee -a $O/kb_ab.txt
  done
done
timeout -k 10 200 python tools/expt/fft4_trace.py -1 25 > $O/trace25.log 2>&1 || { tail -5 $O/trace25.log; exit 1; }
grep -v amdgpu.ids $O/trace25.log | head -8
timeout -k 10 400 python bench.py --log2n 25 --dms-per-gpu 1 --steps 2 --warmup 1 > $O/bench25.log 2>&1 || { tail -20 $O/bench25.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"accel_trials_per_dm": [0-9]*' $O/bench25.log | tr '\n' ' '; echo
timeout -k 10 300 python bench.py --log2n 20 --dms-per-gpu 32 --steps 10 --warmup 2 > $O/b20.log 2>&1 || { tail -5 $O/b20.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/b20.log | tr '\n' ' '; echo
echo DONE
