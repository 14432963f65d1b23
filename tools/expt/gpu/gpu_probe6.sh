#!/bin/bash
# Round-6 probes: the config-3 rank rehearsal and the bench at long series.
#   tools/expt/gpu/gpu_probe6.sh OUT [bench log2n values...]
set -o pipefail
O=gpurun_out/${1:-probe6}; shift
mkdir -p $O /tmp/cfgwork
export TMPDIR=/tmp
timeout -k 10 600 python tools/baseline_configs.py --configs 3 --as-rank 8:0,3,7 --workdir /tmp/cfgwork --out $O/cfg3_as8.jsonl > $O/cfg3.log 2>&1 || { tail -20 $O/cfg3.log; exit 1; }
python tools/summarize_jsonl.py $O/cfg3_as8.jsonl as_rank warmup accel_trials accel_slices search_s wall_s timers_s.total
for L in "$@"; do
  timeout -k 10 600 python bench.py --log2n $L --steps 3 --warmup 1 > $O/bench_$L.log 2>&1 || { tail -20 $O/bench_$L.log; exit 1; }
  grep '^{' $O/bench_$L.log | cut -c1-300
done
echo DONE
