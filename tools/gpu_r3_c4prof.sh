#!/bin/bash
# Config 4 (2026 DMs x 13 accelerations at 2^20, one pulsar) kernel statistics.
set -o pipefail
O=gpurun_out/r3c4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/baseline_configs.py --configs 4 --sky single --workdir /tmp/cfg --out $O/c4_plain.jsonl > $O/c4_plain.log 2>&1 || { echo C4_FAIL; tail -20 $O/c4_plain.log; exit 1; }
cut -c1-400 $O/c4_plain.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c4 -- python3 tools/baseline_configs.py --configs 4 --sky single --workdir /tmp/cfg --out $O/c4_prof.jsonl > $O/c4_prof.log 2>&1 || { echo PROF_FAIL; tail -20 $O/c4_prof.log; exit 1; }
cut -c1-400 $O/c4_prof.jsonl
echo DONE
