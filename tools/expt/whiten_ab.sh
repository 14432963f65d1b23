# same-box A/B of the whitening front end on bench.py (2 interleaved rounds)
set -o pipefail
mkdir -p gpurun_out/wab
for r in 1 2; do
  for v in batch k1 rocfft; do
    case $v in
      batch) env_="" ;;
      k1) env_="PSOUP_PREPARE_MAX=1" ;;
      rocfft) env_="PSOUP_WHITEN_ROCFFT=1" ;;
    esac
    env $env_ timeout -k 10 300 python bench.py --steps 5 > gpurun_out/wab/${v}_$r.log 2>&1 || exit 1
    echo -n "$v $r "; tail -1 gpurun_out/wab/${v}_$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"])'
  done
done
