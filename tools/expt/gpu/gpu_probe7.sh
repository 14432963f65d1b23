#!/bin/bash
# Round-6 probes: 2^20 step kernel table, 2^25 fused-pass phase traces,
# native vs Python config 4 (3 runs each).   tools/expt/gpu/gpu_probe7.sh OUT
set -o pipefail
O=gpurun_out/${1:-probe7}
mkdir -p $O /tmp/cfgwork
export TMPDIR=/tmp
timeout -k 10 200 python tools/expt/fft4_trace.py -1 25 > $O/trace25.log 2>&1 || { tail -5 $O/trace25.log; exit 1; }
grep -v amdgpu.ids $O/trace25.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof20 -o b --output-format csv -- python3 bench.py --log2n 20 --dms-per-gpu 32 --steps 4 --warmup 1 > $O/bench20.log 2>&1 || { tail -20 $O/bench20.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/bench20.log | tr '\n' ' '; echo
python tools/prof_summary.py $(find $O/prof20 -name '*kernel_stats.csv' | head -1) 24
for i in 1 2 3; do
  timeout -k 10 300 python tools/baseline_configs.py --configs 4 --workdir /tmp/cfgwork --out $O/c4_python.jsonl > $O/c4p.log 2>&1 || { tail -20 $O/c4p.log; exit 1; }
  timeout -k 10 300 python tools/baseline_configs.py --configs 4 --native --workdir /tmp/cfgwork --out $O/c4_native.jsonl > $O/c4n.log 2>&1 || { tail -20 $O/c4n.log; exit 1; }
done
python tools/summarize_jsonl.py $O/c4_python.jsonl desc timers_s.searching timers_s.total wall_s
python tools/summarize_jsonl.py $O/c4_native.jsonl desc timers_s.searching timers_s.total wall_s performance.code_objects_deferred performance.device_init_s
echo DONE
