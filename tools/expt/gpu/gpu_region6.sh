#!/bin/bash
# Hashed peak-record regions: clustering / screen / distillation / pipeline
# tests, config 3 as ranks 0/3/7 of 8 with default regions and one region,
# config 4, and the headline bench.   tools/expt/gpu/gpu_region6.sh OUT
set -o pipefail
O=gpurun_out/${1:-region6}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_peakcluster_gpu.py tests/test_screen_gpu.py tests/test_harmdistill_gpu.py tests/test_pipeline_gpu.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 200 python tools/baseline_configs.py --configs 3 --as-rank 8:0,3,7 --workdir /tmp/w --out $O/c3.jsonl > $O/c3.log 2>&1 || { tail -20 $O/c3.log; exit 1; }
python tools/summarize_jsonl.py $O/c3.jsonl as_rank search_s rank_stats.peaks rank_stats.overflows
for i in 1 2; do
  timeout -k 10 200 python tools/baseline_configs.py --configs 4 --workdir /tmp/w --out $O/c4.jsonl > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
done
python tools/summarize_jsonl.py $O/c4.jsonl timers_s.searching timers_s.total
timeout -k 10 300 python bench.py > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
echo "2^23: $(grep -o '"value": [0-9.]*' $O/b.log)"
timeout -k 10 300 python bench.py --signal > $O/bs.log 2>&1 || { tail -5 $O/bs.log; exit 1; }
echo "2^23 peak-heavy: $(grep -o '"value": [0-9.]*' $O/bs.log)"
echo DONE
