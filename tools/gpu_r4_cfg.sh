#!/bin/bash
# Peak-heavy byte-identity test; configs 4/5; signal trace; golden command x5 (native + Python).
set -o pipefail
O=gpurun_out/r4cfg
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread "tests/test_pipeline_gpu.py::test_peak_heavy_candidates_equal_across_clustering_paths" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python3 tools/baseline_configs.py --configs 4,5 --workdir /tmp/cfg --out $O/c45.jsonl > $O/c45.log 2>&1 || { echo C45_FAIL; tail -20 $O/c45.log; exit 1; }
cut -c1-400 $O/c45.jsonl
for i in 1 2 3 4 5; do
  timeout -k 10 120 ./bin/peasoup -i tests/data/tutorial.fil -o $O/golden_native_$i --dm_end 250 --acc_start -5 --acc_end 5 -n 4 --npdmp 10 > $O/golden_native_$i.log 2>&1 || { echo GOLDEN_NATIVE_FAIL; tail -20 $O/golden_native_$i.log; exit 1; }
done
for i in 1 2 3; do
  timeout -k 10 180 python -u -m peasoup_amd -i tests/data/tutorial.fil -o $O/golden_py_$i --dm_end 250 --acc_start -5 --acc_end 5 -n 4 --npdmp 10 > $O/golden_py_$i.log 2>&1 || { echo GOLDEN_PY_FAIL; tail -20 $O/golden_py_$i.log; exit 1; }
done
grep -h -A7 "<execution_times>" $O/golden_native_*/overview.xml | grep -v execution_times | tr -s ' ' | paste -sd' ' | cut -c1-1500
echo
O=gpurun_out/r4trace_sig3 bash tools/gpu_r4_trace.sh --signal
echo DONE
