#!/bin/bash
# The golden command x5 (native + Python) for the stage-time comparison (tools/golden_times.py).
set -o pipefail
O=gpurun_out/r4golden
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3 4 5; do
  timeout -k 10 120 ./bin/peasoup -i tests/data/tutorial.fil -o $O/golden_native_$i --dm_end 250 --acc_start -5 --acc_end 5 -n 4 --npdmp 10 --trace_json $O/trace_native_$i.json > $O/golden_native_$i.log 2>&1 || { echo GOLDEN_NATIVE_FAIL; tail -20 $O/golden_native_$i.log; exit 1; }
done
for i in 1 2 3 4 5; do
  timeout -k 10 180 python -u -m peasoup_amd -i tests/data/tutorial.fil -o $O/golden_py_$i --dm_end 250 --acc_start -5 --acc_end 5 -n 4 --npdmp 10 > $O/golden_py_$i.log 2>&1 || { echo GOLDEN_PY_FAIL; tail -20 $O/golden_py_$i.log; exit 1; }
done
python3 tools/golden_times.py $O/golden_native_* -- $O/golden_py_*
echo DONE
