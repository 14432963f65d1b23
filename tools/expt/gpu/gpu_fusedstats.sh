#!/bin/bash
# Dereddening + interbin statistics in one pass (PSOUP_WHITEN_FUSED_STATS):
# kernel / engine / pipeline GPU tests, then bench A/B at 2^20 / 2^21 / 2^22
# and config 4, alternating on one box.
set -o pipefail
O=gpurun_out/${1:-fusedstats}
mkdir -p $O /tmp/cfgw
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_kernels_gpu.py tests/test_spectrum_gpu.py tests/test_pipeline_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for l in 20 21 22; do
    for v in 0 1; do
      PSOUP_WHITEN_FUSED_STATS=$v timeout -k 10 300 python3 bench.py --log2n $l --dms-per-gpu 32 --steps 10 --warmup 2 > $O/b.log 2>&1 || { tail -10 $O/b.log; exit 1; }
      grep '^{"metric"' $O/b.log >> $O/bench_${l}_$v.jsonl
    done
  done
done
for rep in 1 2; do
  for v in 0 1; do
    PSOUP_WHITEN_FUSED_STATS=$v timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --workdir /tmp/cfgw --out $O/c4_$v.jsonl > $O/c.log 2>&1 || { tail -10 $O/c.log; exit 1; }
  done
done
for l in 20 21 22; do for v in 0 1; do echo "2^$l fused=$v: $(python3 -c "import json; print([json.loads(x)['value'] for x in open('$O/bench_${l}_$v.jsonl')])")"; done; done
for v in 0 1; do echo "c4 fused=$v"; python3 tools/summarize_jsonl.py $O/c4_$v.jsonl timers_s.searching; done
echo DONE
