#!/bin/bash
# GPU peak clustering: kernel + engine equality tests, signal sweep, configs 4/5
set -o pipefail
O=${O:-gpurun_out/r3d}
W=/tmp/psoup_cfg
mkdir -p $O $W
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_peakcluster_gpu.py > $O/pytest_pc.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_pc.log; exit 1; }
tail -3 $O/pytest_pc.log
O=$O bash tools/gpu_r3_sig.sh || exit 1
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-300
timeout -k 10 400 python -u tools/baseline_configs.py --configs 4,5 --workdir $W --out $O/configs.jsonl > $O/configs.log 2>&1 || { echo CONFIGS_FAIL; tail -30 $O/configs.log; exit 1; }
python -c "
import json
for l in open('$O/configs.jsonl'):
    d=json.loads(l); print(d['config'], d['wall_s'], d['timers_s'], d['candidates'], d.get('folded'), d['rank_stats'][0]['peaks'], d['rank_stats'][0]['host_s'], d['rank_stats'][0].get('harm_in'), d['rank_stats'][0].get('harm_out'), d.get('fold_stats'), d['best'])
"
echo DONE
