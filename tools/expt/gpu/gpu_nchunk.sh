#!/bin/bash
# Native config 4 with 32- / 64-DM chunks (PSOUP_CHUNK_DMS), alternating.
set -o pipefail
O=gpurun_out/${1:-nchunk}
mkdir -p $O /tmp/cfgw
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --native --workdir /tmp/cfgw > $O/warm.log 2>&1 || { tail -10 $O/warm.log; exit 1; }
for rep in 1 2 3; do
  for c in 32 64; do
    PSOUP_CHUNK_DMS=$c timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --native --workdir /tmp/cfgw --out $O/n_$c.jsonl > $O/n.log 2>&1 || { tail -10 $O/n.log; exit 1; }
  done
done
for c in 32 64; do echo "chunk $c"; python3 tools/summarize_jsonl.py $O/n_$c.jsonl timers_s.searching timers_s.dedispersion timers_s.total performance.phase_search_s; done
echo DONE
