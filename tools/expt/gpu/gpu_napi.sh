#!/bin/bash
# Native config 4 under a HIP API trace (host time per runtime call).
set -o pipefail
O=gpurun_out/${1:-napi}
mkdir -p $O /tmp/cfgw
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --native --workdir /tmp/cfgw --out $O/warm.jsonl > $O/warm.log 2>&1 || { tail -10 $O/warm.log; exit 1; }
ARGS=$(python3 -c "import json; print(' '.join(json.loads(open('$O/warm.jsonl').readline())['argv']))")
PSOUP_SCHED_TRACE=$O/sched.csv timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -d $O/ht -o ht --output-format csv -- ./bin/peasoup $ARGS > $O/run.log 2>&1 || { tail -10 $O/run.log; exit 1; }
gzip -f $O/ht/ht_hip_api_trace.csv $O/ht/ht_kernel_trace.csv
echo DONE
