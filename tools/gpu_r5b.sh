#!/bin/bash
# Round-5 batch: kernel tests (dedispersion incl. packed 2-bit, peak
# clustering, spectrum), search_iter/pipeline tests, dedispersion bench,
# benches (noise, peak-heavy, 2^20) and a peak-record dump for replay.
set -o pipefail
O=gpurun_out/${1:-r5b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_peakcluster_gpu.py tests/test_spectrum_gpu.py -k "dedisp or packed2 or cluster or spectrum or resident" > $O/t1.log 2>&1 || { tail -30 $O/t1.log; exit 1; }
tail -2 $O/t1.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_pipeline_gpu.py -k "search_iter or headline or peak_heavy or direct_and_mfma" > $O/t2.log 2>&1 || { tail -30 $O/t2.log; exit 1; }
tail -2 $O/t2.log
timeout -k 10 300 python tools/dedisp_bench.py --ndm 2026 --samples 6 > $O/dedisp.log 2>&1 || { tail -20 $O/dedisp.log; exit 1; }
tail -1 $O/dedisp.log
for c in "--steps 10 --warmup 2" "--steps 10 --warmup 2 --peak-heavy" "--log2n 20 --dms-per-gpu 32 --steps 20 --warmup 3"; do
  timeout -k 10 300 python bench.py $c > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  grep "^{" $O/b.log >> $O/bench.jsonl
  grep "^{" $O/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['search_s_per_step'], d['config']['merge_s_per_step'])"
done
PSOUP_DUMP_PEAKS=$O/peaks_sig.bin PSOUP_DUMP_PEAKS_MIN=2000000 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --peak-heavy > $O/dump.log 2>&1 || { tail -5 $O/dump.log; exit 1; }
ls -la $O/peaks_sig.bin && timeout -k 10 120 python tools/expt/cluster_replay.py $O/peaks_sig.bin --trace 2>&1 | tee $O/replay.log
xz -T4 $O/peaks_sig.bin
echo DONE
