#!/bin/bash
# Every BASELINE.json configuration on the current tree, one GPU, written under
# gpurun_out/$1 (summarised in profiles/r6_configs/SUMMARY.md):
#   configs 1-3 (Python; config 3 = 1 DM x 685 accelerations at 2^23), config 3
#   as ranks 0/3/7 of an 8-rank run (acceleration slices), configs 4/5 three
#   times each through Python and bin/peasoup, config 4 as ranks 0/3/7, the
#   golden command, bench at 2^20..2^23, and rocprofv3 kernel tables of
#   configs 3 and 4.
set -o pipefail
O=gpurun_out/${1:-configs6}
W=/tmp/cfgwork
mkdir -p $O $W
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step() { echo "[$(date +%T)] $*"; }
step configs 1-3
timeout -k 10 400 python3 tools/baseline_configs.py --configs 1,2,3 --workdir $W --out $O/c123.jsonl > $O/c123.log 2>&1 || { tail -20 $O/c123.log; exit 1; }
step config 3 as ranks 0,3,7 of 8
timeout -k 10 400 python3 tools/baseline_configs.py --configs 3 --as-rank 8:0,3,7 --workdir $W --out $O/c3_as8.jsonl > $O/c3_as8.log 2>&1 || { tail -20 $O/c3_as8.log; exit 1; }
for i in 1 2 3; do
  step configs 4,5 python run $i
  timeout -k 10 400 python3 tools/baseline_configs.py --configs 4,5 --workdir $W --out $O/c45_py.jsonl > $O/c45p.log 2>&1 || { tail -20 $O/c45p.log; exit 1; }
  step configs 4,5 native run $i
  timeout -k 10 400 python3 tools/baseline_configs.py --configs 4,5 --native --workdir $W --out $O/c45_native.jsonl > $O/c45n.log 2>&1 || { tail -20 $O/c45n.log; exit 1; }
done
step config 4 as ranks 0,3,7 of 8
timeout -k 10 400 python3 tools/baseline_configs.py --configs 4 --as-rank 8:0,3,7 --workdir $W --out $O/c4_as8.jsonl > $O/c4_as8.log 2>&1 || { tail -20 $O/c4_as8.log; exit 1; }
step golden command
bash tools/expt/gpu/gpu_golden.sh ${1:-configs6}/golden > $O/golden.log 2>&1 || { tail -20 $O/golden.log; exit 1; }
for l in 20 21 22; do
  step bench 2^$l
  timeout -k 10 300 python3 bench.py --log2n $l --dms-per-gpu 32 --steps 10 --warmup 2 > $O/bench_$l.log 2>&1 || { tail -10 $O/bench_$l.log; exit 1; }
  grep '^{"metric"' $O/bench_$l.log > $O/bench_$l.json
done
step bench 2^23
timeout -k 10 300 python3 bench.py > $O/bench_23.log 2>&1 || { tail -10 $O/bench_23.log; exit 1; }
grep '^{"metric"' $O/bench_23.log > $O/bench_23.json
step rocprof config 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o c3 --output-format csv -- python3 tools/baseline_configs.py --configs 3 --workdir $W > $O/prof_c3.log 2>&1 || { tail -10 $O/prof_c3.log; exit 1; }
step rocprof config 4
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o c4 --output-format csv -- python3 tools/baseline_configs.py --configs 4 --workdir $W > $O/prof_c4.log 2>&1 || { tail -10 $O/prof_c4.log; exit 1; }
rm -f $O/prof_c3/*kernel_trace.csv $O/prof_c4/*kernel_trace.csv
step DONE
