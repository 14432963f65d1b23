# Auto acceleration batch at 2^23 against explicit batch sizes, same box.
mkdir -p gpurun_out/abb
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "auto or batch" > gpurun_out/abb/t.log 2>&1 || { tail -30 gpurun_out/abb/t.log; exit 1; }
tail -1 gpurun_out/abb/t.log
for r in 1 2; do
  for a in 0 1024 2048; do
    if [ $a = 0 ]; then opt=""; else opt="--accel-batch $a"; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 $opt > gpurun_out/abb/b_${a}_$r.log 2>&1 || { tail -20 gpurun_out/abb/b_${a}_$r.log; exit 1; }
    echo "batch $a: $(grep -o '"value": [0-9.]*' gpurun_out/abb/b_${a}_$r.log) $(grep -o '"accel_batch": [0-9]*' gpurun_out/abb/b_${a}_$r.log)"
  done
done
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --signal > gpurun_out/abb/sig.log 2>&1 || { tail -20 gpurun_out/abb/sig.log; exit 1; }
echo "signal: $(grep -o '"value": [0-9.]*' gpurun_out/abb/sig.log)"
