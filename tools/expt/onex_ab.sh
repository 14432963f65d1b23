# One-exchange passes: numerics (fft4 GPU tests), per-kernel times, phase
# trace, then same-box bench A/B of flag sets ($@, default 212227 736515).
set -o pipefail
mkdir -p gpurun_out/onex
FL=${@:-212227 736515}
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "fft4 or whiten" -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/onex/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/onex/tests.log; exit 1; }
tail -2 gpurun_out/onex/tests.log
timeout -k 10 200 python tools/kbench.py --K 32 --flags $(echo $FL | tr ' ' ',') > gpurun_out/onex/kb.txt 2>&1 || exit 1
grep -E "colpass|rowpass" gpurun_out/onex/kb.txt
for r in 1 2; do
  for fl in $FL; do
    timeout -k 10 300 python bench.py --steps 5 --fft4-flags $fl > gpurun_out/onex/b_${fl}_$r.log 2>&1 || exit 1
    echo -n "$fl "; tail -n 1 gpurun_out/onex/b_${fl}_$r.log | python -c 'import sys,json; print(json.loads(sys.stdin.read())["value"])'
  done
done
