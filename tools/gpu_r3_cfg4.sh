#!/bin/bash
# Config 4 on the round-2 data (one pulsar in noise), Python and native,
# with a kernel trace of the Python run.
set -o pipefail
O=gpurun_out/r3cfg4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o c4 -- python3 tools/baseline_configs.py --configs 4 --sky single --workdir /tmp/cfg --out $O/c4.jsonl > $O/c4.log 2>&1 || { echo C4_FAIL; tail -20 $O/c4.log; exit 1; }
cut -c1-1500 $O/c4.jsonl
timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --sky single --workdir /tmp/cfg --out $O/c4b.jsonl > $O/c4b.log 2>&1 || { echo C4B_FAIL; tail -20 $O/c4b.log; exit 1; }
cut -c1-700 $O/c4b.jsonl
timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --sky single --native --workdir /tmp/cfg --out $O/c4n.jsonl > $O/c4n.log 2>&1 || { echo C4N_FAIL; tail -20 $O/c4n.log; exit 1; }
cut -c1-900 $O/c4n.jsonl
echo DONE
