# Record regions (SearchParams.peak_region_log2) against one counter, same box.
mkdir -p gpurun_out/abr
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_peakcluster_gpu.py tests/test_harmdistill_gpu.py > gpurun_out/abr/t.log 2>&1 || { tail -40 gpurun_out/abr/t.log; exit 1; }
tail -1 gpurun_out/abr/t.log
for g in 6 0 6 0; do
  PSOUP_PEAK_REGION_LOG2=$g timeout -k 10 300 python bench.py --steps 10 --warmup 2 --signal > gpurun_out/abr/s_$g.log 2>&1 || { tail -20 gpurun_out/abr/s_$g.log; exit 1; }
  echo "signal regions 2^$g: $(grep -o '"value": [0-9.]*' gpurun_out/abr/s_$g.log)"
done
PSOUP_PEAK_REGION_LOG2=8 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --signal > gpurun_out/abr/s_8.log 2>&1 || { tail -20 gpurun_out/abr/s_8.log; exit 1; }
echo "signal regions 2^8: $(grep -o '"value": [0-9.]*' gpurun_out/abr/s_8.log)"
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/abr/noise.log 2>&1 || { tail -20 gpurun_out/abr/noise.log; exit 1; }
echo "noise: $(grep -o '"value": [0-9.]*' gpurun_out/abr/noise.log)"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/abr/psig -o b --output-format csv -- python3 bench.py --steps 6 --warmup 2 --signal > gpurun_out/abr/psig.log 2>&1
