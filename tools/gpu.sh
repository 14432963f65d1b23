#!/bin/bash
# One entry point for the GPU-box jobs (run through gpurun; every step has its
# own time limit and the steps are chained so that a failure ends the job).
# Output goes under gpurun_out/NAME; the summaries that matter are copied to
# profiles/ by hand.
#
#   tools/gpu.sh round   NAME [bench args]   GPU tests, smoke(), bench, rocprofv3 kernel stats of the bench
#   tools/gpu.sh tests   NAME [pytest args]  pytest -m gpu (one process)
#   tools/gpu.sh bench   NAME [bench args]   bench.py once
#   tools/gpu.sh prof    NAME [bench args]   rocprofv3 --kernel-trace --stats of bench.py
#   tools/gpu.sh pmc     NAME [bench args]   three counter passes (SQ / TCC fetch / writes + LDS), kernel trace only
#   tools/gpu.sh ab      NAME REPS L DMS FLAGS...  same-box A/B of fft4 flag sets, interleaved (2^L, DMS per step)
#   tools/gpu.sh configs NAME                every BASELINE configuration (profiles/r6_configs/SUMMARY.md)
#   tools/gpu.sh golden  NAME                the golden command x5 per driver + the stage table
#
# (One-off lease wrappers of earlier rounds: tools/expt/gpu/.)
set -o pipefail
task=${1:?task}; name=${2:?name}; shift 2
O=gpurun_out/$name
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step() { echo "[$(date +%T)] $*"; }
PYTEST="python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread"

case $task in
  tests)
    timeout -k 10 1100 $PYTEST tests -m gpu "$@" > "$O/pytest_gpu.log" 2>&1 || { echo TESTS_FAIL; tail -40 "$O/pytest_gpu.log"; exit 1; }
    tail -2 "$O/pytest_gpu.log"
    ;;
  bench)
    timeout -k 10 400 python bench.py "$@" > "$O/bench.log" 2>&1 || { echo BENCH_FAIL; tail -30 "$O/bench.log"; exit 1; }
    tail -1 "$O/bench.log"
    ;;
  prof)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O" -o bench --output-format csv -- python3 bench.py --steps 2 --warmup 1 "$@" > "$O/bench.log" 2>&1 || { echo PROF_FAIL; tail -20 "$O/bench.log"; exit 1; }
    tail -1 "$O/bench.log"
    rm -f "$O"/bench_kernel_trace.csv
    python3 tools/prof_summary.py "$O"/bench_kernel_stats.csv > "$O/kernels.md" 2>/dev/null || true
    ;;
  pmc)
    run_pass() {  # pass-name counters...
      local p=$1; shift
      timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d "$O/$p" -o p --output-format csv -- python3 bench.py --steps 1 --warmup 0 $BARGS > "$O/$p.log" 2>&1 || { echo "PMC_${p}_FAIL"; tail -20 "$O/$p.log"; exit 1; }
    }
    BARGS="$*"
    run_pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU
    run_pass tcc FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE
    run_pass wr WRITE_SIZE TCC_MISS_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
    echo PMC_OK
    ;;
  ab)
    reps=${1:?reps}; l=${2:?log2n}; dms=${3:?dms}; shift 3
    for r in $(seq 1 "$reps"); do
      for f in "$@"; do
        timeout -k 10 300 python bench.py --log2n "$l" --dms-per-gpu "$dms" --fft4-flags "$f" > "$O/b.log" 2>&1 || { echo "FAIL $f"; tail -5 "$O/b.log"; exit 1; }
        grep '^{"metric"' "$O/b.log" >> "$O/ab_$f.jsonl"
        echo "2^$l flags $f rep $r: $(grep -o '"value": [0-9.]*' "$O/b.log")"
      done
    done
    ;;
  configs)
    W=/tmp/cfgwork
    mkdir -p $W
    step configs 1-3
    timeout -k 10 400 python3 tools/baseline_configs.py --configs 1,2,3 --workdir $W --out "$O/c123.jsonl" > "$O/c123.log" 2>&1 || { tail -20 "$O/c123.log"; exit 1; }
    step config 3 as ranks 0,3,7 of 8
    timeout -k 10 400 python3 tools/baseline_configs.py --configs 3 --as-rank 8:0,3,7 --workdir $W --out "$O/c3_as8.jsonl" > "$O/c3_as8.log" 2>&1 || { tail -20 "$O/c3_as8.log"; exit 1; }
    for i in 1 2 3; do
      step configs 4,5 python run $i
      timeout -k 10 400 python3 tools/baseline_configs.py --configs 4,5 --workdir $W --out "$O/c45_py.jsonl" > "$O/c45p.log" 2>&1 || { tail -20 "$O/c45p.log"; exit 1; }
      step configs 4,5 native run $i
      timeout -k 10 400 python3 tools/baseline_configs.py --configs 4,5 --native --workdir $W --out "$O/c45_native.jsonl" > "$O/c45n.log" 2>&1 || { tail -20 "$O/c45n.log"; exit 1; }
    done
    step config 4 as ranks 0,3,7 of 8
    timeout -k 10 400 python3 tools/baseline_configs.py --configs 4 --as-rank 8:0,3,7 --workdir $W --out "$O/c4_as8.jsonl" > "$O/c4_as8.log" 2>&1 || { tail -20 "$O/c4_as8.log"; exit 1; }
    step golden command
    bash tools/gpu.sh golden "$name/golden" > "$O/golden.log" 2>&1 || { tail -20 "$O/golden.log"; exit 1; }
    for l in 20 21 22; do
      step bench 2^$l
      timeout -k 10 300 python3 bench.py --log2n $l --dms-per-gpu 32 --steps 10 --warmup 2 > "$O/bench_$l.log" 2>&1 || { tail -10 "$O/bench_$l.log"; exit 1; }
      grep '^{"metric"' "$O/bench_$l.log" > "$O/bench_$l.json"
    done
    step bench 2^23
    timeout -k 10 300 python3 bench.py > "$O/bench_23.log" 2>&1 || { tail -10 "$O/bench_23.log"; exit 1; }
    grep '^{"metric"' "$O/bench_23.log" > "$O/bench_23.json"
    for c in 3 4; do
      step rocprof config $c
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_c$c" -o c$c --output-format csv -- python3 tools/baseline_configs.py --configs $c --workdir $W > "$O/prof_c$c.log" 2>&1 || { tail -10 "$O/prof_c$c.log"; exit 1; }
      rm -f "$O/prof_c$c"/*kernel_trace.csv
    done
    step DONE
    ;;
  golden)
    ARGS="-i tests/data/tutorial.fil --dm_end 250 --acc_start -5 --acc_end 5 -n 4 --npdmp 10"
    for i in 1 2 3 4 5; do
      timeout -k 10 120 ./bin/peasoup $ARGS -o "$O/golden_native_$i" --trace_json "$O/trace_native_$i.json" > "$O/golden_native_$i.log" 2>&1 || { echo GOLDEN_NATIVE_FAIL; tail -20 "$O/golden_native_$i.log"; exit 1; }
    done
    for i in 1 2 3 4 5; do
      timeout -k 10 180 python -u -m peasoup_amd $ARGS -o "$O/golden_py_$i" --trace_json "$O/trace_py_$i.json" > "$O/golden_py_$i.log" 2>&1 || { echo GOLDEN_PY_FAIL; tail -20 "$O/golden_py_$i.log"; exit 1; }
    done
    cmp "$O/golden_native_2/candidates.peasoup" "$O/golden_py_2/candidates.peasoup" && echo "candidates identical"
    python3 tools/golden_times.py "$O"/golden_native_* -- "$O"/golden_py_* > "$O/golden_times.md"
    cat "$O/golden_times.md"
    ;;
  round)
    bash tools/gpu.sh tests "$name" || exit 1
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo SMOKE_FAIL; tail -30 "$O/smoke.log"; exit 1; }
    tail -1 "$O/smoke.log"
    bash tools/gpu.sh bench "$name" "$@" || exit 1
    bash tools/gpu.sh prof "$name/prof" "$@" || exit 1
    ;;
  *)
    echo "unknown task $task"; exit 2
    ;;
esac
