#!/bin/bash
# Native config 4 under a kernel trace, block pipeline off / on: GPU busy and
# idle gaps over the search (tools/trace_gaps.py).
set -o pipefail
O=gpurun_out/${1:-ntrace}
mkdir -p $O /tmp/cfgw
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --native --workdir /tmp/cfgw --out $O/warm.jsonl > $O/warm.log 2>&1 || { tail -10 $O/warm.log; exit 1; }
ARGS=$(python3 -c "import json; print(' '.join(json.loads(open('$O/warm.jsonl').readline())['argv']))")
echo "bin/peasoup $ARGS"
for p in 0 1; do
  PSOUP_BLOCK_PIPELINE=$p timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p$p -o p$p --output-format csv -- ./bin/peasoup $ARGS > $O/p$p.log 2>&1 || { tail -10 $O/p$p.log; exit 1; }
  python3 tools/trace_gaps.py $O/p$p/p${p}_kernel_trace.csv > $O/gaps_p$p.txt
  echo "== pipeline $p"; head -25 $O/gaps_p$p.txt
  gzip -f $O/p$p/p${p}_kernel_trace.csv
done
echo DONE
