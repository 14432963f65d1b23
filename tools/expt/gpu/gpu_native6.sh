#!/bin/bash
# Native CLI vs Python driver: pipeline GPU tests, then config 4 alternating
# Python / native three times each.   tools/expt/gpu/gpu_native6.sh OUT
set -o pipefail
O=gpurun_out/${1:-native6}
mkdir -p $O /tmp/cfgwork
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pipeline_gpu.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "dedisp or packed or mfma or valu" > $O/t2.log 2>&1 || { tail -30 $O/t2.log; exit 1; }
tail -1 $O/t2.log
timeout -k 10 300 python tools/dedisp_bench.py --log2n 20 --ndm 2000 > $O/ddb.log 2>&1 || { tail -10 $O/ddb.log; exit 1; }
grep -o '"d0": [0-9]*\|"mfma_ms": [0-9.]*\|"packed2_ms": [0-9.]*\|"bit_exact": [a-z]*' $O/ddb.log | paste - - - - | head -8
tail -1 $O/ddb.log | cut -c1-400
for i in 1 2 3; do
  timeout -k 10 300 python tools/baseline_configs.py --configs 4 --workdir /tmp/cfgwork --out $O/c4_python.jsonl > $O/c4p.log 2>&1 || { tail -20 $O/c4p.log; exit 1; }
  timeout -k 10 300 python tools/baseline_configs.py --configs 4 --native --workdir /tmp/cfgwork --out $O/c4_native.jsonl > $O/c4n.log 2>&1 || { tail -20 $O/c4n.log; exit 1; }
done
python tools/summarize_jsonl.py $O/c4_python.jsonl timers_s.searching timers_s.dedispersion timers_s.total wall_s
python tools/summarize_jsonl.py $O/c4_native.jsonl timers_s.searching timers_s.dedispersion timers_s.total wall_s performance.device_init_s
echo DONE
