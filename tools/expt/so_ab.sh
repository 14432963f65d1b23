# Same-box A/B of bench.py: the tree's build (A) vs an alternative _C .so (B),
# interleaved: bash tools/expt/so_ab.sh ab_so/_C_alt.so REPS
set -o pipefail
alt=$1; reps=${2:-3}
mkdir -p gpurun_out/soab
rm -rf /tmp/soab_tree && mkdir -p /tmp/soab_tree && cp -r peasoup_amd bench.py /tmp/soab_tree/
cp "$alt" /tmp/soab_tree/peasoup_amd/_C.cpython-310-x86_64-linux-gnu.so
for r in $(seq 1 $reps); do
  timeout -k 10 300 python bench.py --steps 5 > gpurun_out/soab/a_$r.log 2>&1 || exit 1
  (cd /tmp/soab_tree && timeout -k 10 300 python bench.py --steps 5) > gpurun_out/soab/b_$r.log 2>&1 || exit 1
  echo -n "A "; tail -n 1 gpurun_out/soab/a_$r.log | python -c 'import sys,json; print(json.loads(sys.stdin.read())["value"])'
  echo -n "B "; tail -n 1 gpurun_out/soab/b_$r.log | python -c 'import sys,json; print(json.loads(sys.stdin.read())["value"])'
done
