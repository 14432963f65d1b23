#!/bin/bash
# A/B on one box: step pipeline vs serial steps (noise, peak-heavy, 2^20);
# peak clustering replay after the XCD-spread segment order; cluster tests.
set -o pipefail
O=gpurun_out/${1:-r5d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_peakcluster_gpu.py tests/test_pipeline_gpu.py -k "cluster or peak_heavy" > $O/t1.log 2>&1 || { tail -30 $O/t1.log; exit 1; }
tail -1 $O/t1.log
xz -dk gpurun_out/r5c1/peaks_sig.bin.xz -c > /tmp/peaks_sig.bin && timeout -k 10 120 python tools/expt/cluster_replay.py /tmp/peaks_sig.bin --trace 2>&1 | grep -v amdgpu.ids | tee $O/replay.log
for c in "--steps 10 --warmup 2" "--steps 10 --warmup 2 --serial-steps" "--steps 10 --warmup 2 --peak-heavy" "--steps 10 --warmup 2 --peak-heavy --serial-steps" "--log2n 20 --dms-per-gpu 32 --steps 20 --warmup 3" "--log2n 20 --dms-per-gpu 32 --steps 20 --warmup 3 --serial-steps" "--steps 10 --warmup 2"; do
  timeout -k 10 300 python bench.py $c > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  grep "^{" $O/b.log >> $O/bench.jsonl
  echo "$c: $(grep "^{" $O/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
echo DONE
