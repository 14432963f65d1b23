#!/bin/bash
# Round-5 profile batch: dedispersion test + bench, peak-heavy replay, kernel
# traces of the noise / peak-heavy benches with idle-gap analysis.
set -o pipefail
O=gpurun_out/${1:-r5c}
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "dedisp or packed2" > $O/t1.log 2>&1 || { tail -30 $O/t1.log; exit 1; }
tail -1 $O/t1.log
timeout -k 10 300 python tools/dedisp_bench.py --ndm 2026 --samples 2 > $O/dedisp.log 2>&1 || { tail -20 $O/dedisp.log; exit 1; }
tail -1 $O/dedisp.log
PSOUP_DUMP_PEAKS=$O/peaks_sig.bin PSOUP_DUMP_PEAKS_MIN=1000000 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --peak-heavy > $O/dump.log 2>&1 || { tail -5 $O/dump.log; exit 1; }
timeout -k 10 120 python tools/expt/cluster_replay.py $O/peaks_sig.bin --trace > $O/replay.log 2>&1 || { tail -5 $O/replay.log; exit 1; }
cat $O/replay.log | grep -v amdgpu.ids
xz -T4 $O/peaks_sig.bin
for tag in noise sig; do
  extra=""; [ $tag = sig ] && extra="--peak-heavy"
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/p_$tag -o run -- python3 $R/bench.py --steps 4 --warmup 1 $extra > $R/$O/p_$tag.log 2>&1) || { echo PROF_FAIL; tail -5 $O/p_$tag.log; exit 1; }
  python3 tools/step_kernels.py $O/p_$tag/run_kernel_trace.csv --skip 1 --steps 3 > $O/k_$tag.md 2>&1
  python3 tools/expt/trace_gaps.py $O/p_$tag/run_kernel_trace.csv > $O/gaps_$tag.txt 2>&1
  head -14 $O/k_$tag.md; head -12 $O/gaps_$tag.txt
  rm -f $O/p_$tag/run_kernel_trace.csv.gz; gzip $O/p_$tag/run_kernel_trace.csv
done
echo DONE
