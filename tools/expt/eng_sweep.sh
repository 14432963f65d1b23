set -o pipefail
mkdir -p gpurun_out/eng
for e in 1 2 3; do
  PSOUP_ENGINES=$e timeout -k 10 300 python tools/baseline_configs.py --configs 4,5 --workdir /tmp/cfgs --out gpurun_out/eng/cfg_e$e.jsonl > gpurun_out/eng/cfg_e$e.log 2>&1 || exit 1
done
for e in 1 2; do
  PSOUP_ENGINES=$e timeout -k 10 300 python bench.py --steps 3 > gpurun_out/eng/bench_e$e.log 2>&1 || exit 1
done
