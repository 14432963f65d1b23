#!/bin/bash
# Dedispersion change check: bit-exact kernel tests, the whole-list kernel
# bench at 2^20 (config 4's list), the 2^20 and 2^23 benches, config 4.
set -o pipefail
O=gpurun_out/${1:-dd6}
mkdir -p $O /tmp/cfgwork
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "dedisp or packed or mfma or valu" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python tools/dedisp_bench.py --log2n 20 --ndm 2000 > $O/ddb.log 2>&1 || { tail -10 $O/ddb.log; exit 1; }
tail -1 $O/ddb.log | cut -c1-600
grep -c '"bit_exact": true' $O/ddb.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --log2n 20 --dms-per-gpu 32 --steps 10 --warmup 2 > $O/b20.log 2>&1 || { tail -5 $O/b20.log; exit 1; }
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/b20.log | tr '\n' ' '; echo
done
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/b23.log 2>&1 || { tail -5 $O/b23.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/b23.log | tr '\n' ' '; echo
for i in 1 2; do
  timeout -k 10 300 python tools/baseline_configs.py --configs 4 --workdir /tmp/cfgwork --out $O/c4_python.jsonl > $O/c4p.log 2>&1 || { tail -20 $O/c4p.log; exit 1; }
done
python tools/summarize_jsonl.py $O/c4_python.jsonl timers_s.searching timers_s.dedispersion timers_s.total
echo DONE
