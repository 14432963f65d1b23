#!/bin/bash
# Config 4 (Python, 3 runs) and its GPU idle gaps after the CandidateBag
# growth fix; config 5 once.
set -o pipefail
O=gpurun_out/${1:-c4ext}
mkdir -p $O /tmp/cfgw
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --workdir /tmp/cfgw > $O/warm.log 2>&1 || { tail -10 $O/warm.log; exit 1; }
for i in 1 2 3; do
  timeout -k 10 300 python3 tools/baseline_configs.py --configs 4,5 --workdir /tmp/cfgw --out $O/c45.jsonl > $O/c45.log 2>&1 || { tail -10 $O/c45.log; exit 1; }
done
python3 tools/summarize_jsonl.py $O/c45.jsonl config timers_s.searching timers_s.total rank_stats.0.accd_s candidates
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c4 -o c4 --output-format csv -- python3 tools/baseline_configs.py --configs 4 --workdir /tmp/cfgw > $O/c4.log 2>&1 || { tail -10 $O/c4.log; exit 1; }
python3 tools/trace_gaps.py $O/c4/c4_kernel_trace.csv > $O/c4_gaps.txt
head -8 $O/c4_gaps.txt
gzip -f $O/c4/c4_kernel_trace.csv
echo DONE
