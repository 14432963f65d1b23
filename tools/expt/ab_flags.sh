# Same-box A/B of fft4 flag sets: the default D against D | $ADD, interleaved.
# usage: ADD=<bits> tools/expt/ab_flags.sh <name> [bench args...]
name=$1; shift
mkdir -p gpurun_out/$name
D=$(python -c "import peasoup_amd._C as C; print(C.kernels.fft4_flags())")
for r in 1 2; do
  for f in $D $((D | ADD)); do
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --fft4-flags $f "$@" > gpurun_out/$name/b_${f}_$r.log 2>&1 || { tail -20 gpurun_out/$name/b_${f}_$r.log; exit 1; }
    echo "flags $f run $r: $(grep -o '"value": [0-9.]*' gpurun_out/$name/b_${f}_$r.log)"
  done
done
