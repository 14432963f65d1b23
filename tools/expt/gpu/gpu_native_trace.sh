#!/bin/bash
# HIP API + kernel trace (rocprofv3, no counters) of one native golden run,
# after one untraced warm-up run, under gpurun_out/$1.
set -o pipefail
O=gpurun_out/${1:-ntrace}
mkdir -p $O
export TMPDIR=/tmp
ARGS="-i tests/data/tutorial.fil --dm_end 250 --acc_start -5 --acc_end 5 -n 4 --npdmp 10"
timeout -k 10 120 ./bin/peasoup $ARGS -o $O/warm > $O/warm.log 2>&1 || { echo WARM_FAIL; tail -20 $O/warm.log; exit 1; }
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $O/prof -o run -- ./bin/peasoup $ARGS -o $O/traced --trace_json $O/trace.json > $O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof.log; exit 1; }
python3 -c "
import json
d = json.load(open('$O/trace.json'))
print({k: round(v, 4) for k, v in d['performance'].items() if k.startswith('phase_')})
"
head -25 $O/prof/run_hip_api_stats.csv | cut -d, -f1-6
