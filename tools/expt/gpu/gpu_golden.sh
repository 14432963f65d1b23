#!/bin/bash
# The golden command (tests/data/tutorial.fil, the reference's example run) x5
# through the native CLI and the Python driver, with --trace_json, under
# gpurun_out/$1; then the stage table (tools/golden_times.py).
set -o pipefail
O=gpurun_out/${1:-golden}
mkdir -p $O
export TMPDIR=/tmp
ARGS="-i tests/data/tutorial.fil --dm_end 250 --acc_start -5 --acc_end 5 -n 4 --npdmp 10"
for i in 1 2 3 4 5; do
  timeout -k 10 120 ./bin/peasoup $ARGS -o $O/golden_native_$i --trace_json $O/trace_native_$i.json > $O/golden_native_$i.log 2>&1 || { echo GOLDEN_NATIVE_FAIL; tail -20 $O/golden_native_$i.log; exit 1; }
done
for i in 1 2 3 4 5; do
  timeout -k 10 180 python -u -m peasoup_amd $ARGS -o $O/golden_py_$i --trace_json $O/trace_py_$i.json > $O/golden_py_$i.log 2>&1 || { echo GOLDEN_PY_FAIL; tail -20 $O/golden_py_$i.log; exit 1; }
done
cmp $O/golden_native_2/candidates.peasoup $O/golden_py_2/candidates.peasoup && echo "candidates identical"
python3 tools/golden_times.py $O/golden_native_* -- $O/golden_py_* > $O/golden_times.md
cat $O/golden_times.md
python3 -c "
import json
for f in ('$O/trace_native_3.json', '$O/trace_py_3.json'):
    try:
        d = json.load(open(f))
    except Exception as e:
        print(f, e); continue
    print(f, {k: round(v, 4) for k, v in d.get('performance', {}).items() if isinstance(v, (int, float)) and k.endswith('_s')})
"
