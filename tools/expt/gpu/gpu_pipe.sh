#!/bin/bash
# Block pipeline (search_launch / whitening of the next block / search_finish)
# A/B: model + pipeline tests, config 4 and the 2^20 / 2^23 benches with
# PSOUP_BLOCK_PIPELINE=0 / 1 alternating.
set -o pipefail
O=gpurun_out/${1:-pipe}
mkdir -p $O /tmp/cfgw
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_models_gpu.py tests/test_pipeline_gpu.py tests/test_failure.py tests/test_checkpoint.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --workdir /tmp/cfgw > $O/warm.log 2>&1 || { tail -10 $O/warm.log; exit 1; }
for rep in 1 2; do
  for p in 0 1; do
    PSOUP_BLOCK_PIPELINE=$p timeout -k 10 300 python3 tools/baseline_configs.py --configs 4,5 --workdir /tmp/cfgw --out $O/c45_p$p.jsonl > $O/c.log 2>&1 || { tail -10 $O/c.log; exit 1; }
    PSOUP_BLOCK_PIPELINE=$p timeout -k 10 300 python bench.py --log2n 20 --dms-per-gpu 32 --steps 10 --warmup 2 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "2^20 pipeline=$p: $(grep -o '"value": [0-9.]*' $O/b.log)"
    PSOUP_BLOCK_PIPELINE=$p timeout -k 10 300 python bench.py > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "2^23 pipeline=$p: $(grep -o '"value": [0-9.]*' $O/b.log)"
  done
done
for p in 0 1; do echo "pipeline=$p"; python3 tools/summarize_jsonl.py $O/c45_p$p.jsonl config timers_s.searching timers_s.total candidates best.snr; done
echo DONE
