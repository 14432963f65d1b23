# One-exchange pass A: numerics (fft4 GPU tests incl. flag sets 212227 and
# 474371), per-kernel times, phase trace, then same-box bench A/B.
set -o pipefail
mkdir -p gpurun_out/onex
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "fft4 or whiten" -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/onex/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/onex/tests.log; exit 1; }
tail -2 gpurun_out/onex/tests.log
timeout -k 10 200 python tools/kbench.py --K 32 --flags 81155,212227 > gpurun_out/onex/kb.txt 2>&1 || exit 1
grep -E "colpass|rowpass" gpurun_out/onex/kb.txt
timeout -k 10 100 python tools/expt/fft4_trace.py 212227 > gpurun_out/onex/trace.txt 2>&1 || exit 1
head -8 gpurun_out/onex/trace.txt
for r in 1 2; do
  for fl in 81155 212227; do
    timeout -k 10 300 python bench.py --steps 5 --fft4-flags $fl > gpurun_out/onex/b_${fl}_$r.log 2>&1 || exit 1
    echo -n "$fl "; tail -n 1 gpurun_out/onex/b_${fl}_$r.log | python -c 'import sys,json; print(json.loads(sys.stdin.read())["value"])'
  done
done
