#!/bin/bash
# Round 3: multi-GPU code paths on one GPU (forced RCCL process group, native
# oversubscribed device workers, 4-rank dynamic schedule), scale8 at N=1,
# rocprof kernel trace of the RCCL-forced bench, pass-A phase trace.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_models_gpu.py::test_forced_rccl_process_group_world1 \
  tests/test_models_gpu.py::test_dynamic_schedule_four_ranks_many_chunks \
  tests/test_pipeline_gpu.py::test_native_oversubscribed_device_workers_match_one \
  > gpurun_out/r3/pytest_multi.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/r3/pytest_multi.log; exit 1; }
tail -5 gpurun_out/r3/pytest_multi.log
timeout -k 10 300 bash tools/scale8.sh 5 1 > gpurun_out/r3/scale8_n1.txt 2>&1 || { echo SCALE_FAIL; cat gpurun_out/r3/scale8_n1.txt; exit 1; }
cat gpurun_out/r3/scale8_n1.txt | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PSOUP_FORCE_PG=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29777 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/prof_forcepg -o forcepg -- python bench.py --steps 3 --warmup 1 > gpurun_out/r3/bench_forcepg.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/r3/bench_forcepg.log; exit 1; }
tail -1 gpurun_out/r3/bench_forcepg.log | cut -c1-200
timeout -k 10 120 python -u tools/expt/fft4_trace.py > gpurun_out/r3/fft4_trace_default.txt 2>&1 && cat gpurun_out/r3/fft4_trace_default.txt
