# Same-box A/B of the working tree against a snapshot build in abtmp/old
# (abtmp/old/bench.py imports abtmp/old/peasoup_amd): tests first, then
# interleaved benches.  usage: tools/expt/ab_tree.sh <name> <pytest -k expr> [bench args...]
name=$1; kx=$2; shift 2
mkdir -p gpurun_out/$name
[ -z "$kx" ] || timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread ${TESTS:-tests/test_spectrum_gpu.py tests/test_kernels_gpu.py} -k "$kx" > gpurun_out/$name/t.log 2>&1 || { tail -40 gpurun_out/$name/t.log; exit 1; }
[ -z "$kx" ] || tail -1 gpurun_out/$name/t.log
for r in 1 2; do
  for v in new old; do
    if [ $v = new ]; then b=bench.py; else b=abtmp/old/bench.py; fi
    timeout -k 10 300 python $b --steps 10 --warmup 2 "$@" > gpurun_out/$name/b_${v}_$r.log 2>&1 || { tail -20 gpurun_out/$name/b_${v}_$r.log; exit 1; }
    echo "$v $r: $(grep -o '"value": [0-9.]*' gpurun_out/$name/b_${v}_$r.log)"
  done
done
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  for v in new old; do
    if [ $v = new ]; then b=bench.py; else b=abtmp/old/bench.py; fi
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$name/p_$v -o b --output-format csv -- python3 $b --steps 6 --warmup 2 "$@" > gpurun_out/$name/p_$v.log 2>&1 || exit 1
  done
fi
