#!/bin/bash
# Long series: kernel tables of one bench step at 2^25 and 2^26 (one DM per
# step) and the config-3 rank rehearsal.  tools/expt/gpu/gpu_long6.sh OUT
set -o pipefail
O=gpurun_out/${1:-long6}
mkdir -p $O /tmp/cfgwork
export TMPDIR=/tmp
timeout -k 10 300 python tools/baseline_configs.py --configs 3 --as-rank 8:0,3,7 --workdir /tmp/cfgwork --out $O/cfg3_as8.jsonl > $O/cfg3.log 2>&1 || { tail -20 $O/cfg3.log; exit 1; }
python tools/summarize_jsonl.py $O/cfg3_as8.jsonl as_rank warmup accel_trials accel_slices search_s wall_s timers_s.total
for L in 25 26; do
  echo "log2n $L"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof$L -o b --output-format csv -- python3 bench.py --log2n $L --dms-per-gpu 1 --steps 1 --warmup 1 > $O/bench_$L.log 2>&1 || { echo FAIL $L; tail -20 $O/bench_$L.log; exit 1; }
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"fft_mode": [0-9]*\|"accel_trials_per_dm": [0-9]*' $O/bench_$L.log | tr '\n' ' '; echo
  f=$(find $O/prof$L -name '*kernel_stats.csv' | head -1)
  python tools/prof_summary.py $f 12
done
echo DONE
