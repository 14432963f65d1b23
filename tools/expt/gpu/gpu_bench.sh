#!/bin/bash
# GPU-box helper: default bench (noise + signal) and a rocprofv3 kernel-stats
# run of the bench, written under gpurun_out/$1.  Extra args go to bench.py.
set -o pipefail
O=gpurun_out/${1:-bench}
shift || true
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 "$@" > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | cut -c1-400
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --signal "$@" > $O/bench_signal.log 2>&1 || { echo BENCH_SIG_FAIL; tail -20 $O/bench_signal.log; exit 1; }
grep '^{"metric"' $O/bench_signal.log | cut -c1-300
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 "$@" > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
find $O/prof -name '*kernel_stats.csv' | head -3
echo DONE
