set -o pipefail
mkdir -p gpurun_out/dd27
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py -k "beyond_one_grid or dedisp or mfma or packed" > gpurun_out/dd27/t.log 2>&1; tail -3 gpurun_out/dd27/t.log
