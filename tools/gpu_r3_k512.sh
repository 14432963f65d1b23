#!/bin/bash
# New 2^23 defaults (K = 512, no sub-batches): GPU suite, default bench x2,
# shorter series with/without sub-batches, config 4 on the single-pulsar data.
set -o pipefail
O=gpurun_out/r3k512
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 280 --timeout-method thread tests/ > $O/pytest_gpu.log 2>&1 \
  || { echo PYTEST_FAIL; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_$r.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench_$r.log; exit 1; }
  grep '^{"metric"' $O/bench_$r.log | cut -c1-160; grep '^{"metric"' $O/bench_$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["config"]["accel_batch"], d["config"]["sub_batch"])'
done
for lg in 22 20; do
  for sb in -1 0; do
    tag="n${lg}_sb${sb}"
    timeout -k 10 300 python -u bench.py --log2n $lg --dms-per-gpu 32 --steps 5 --warmup 2 --sub-batch $sb > $O/$tag.log 2>&1 || { echo BENCH_FAIL $tag; tail -20 $O/$tag.log; exit 1; }
    echo -n "$tag: "; grep '^{"metric"' $O/$tag.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["accel_batch"], d["config"]["sub_batch"])'
  done
done
for th in 1024 512; do
  tag="sig_th$th"
  PSOUP_CLUSTER_TH=$th timeout -k 10 300 python -u bench.py --signal --steps 5 --warmup 2 > $O/$tag.log 2>&1 || { echo BENCH_FAIL $tag; tail -20 $O/$tag.log; exit 1; }
  echo -n "$tag: "; grep '^{"metric"' $O/$tag.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["accel_batch"], d["config"]["sub_batch"], d["config"]["host_distill_s_per_step"])'
done
bash tools/gpu_r3_cfg4.sh
