#!/bin/bash
# Config 4 host timeline per 32-DM block (PSOUP_BLOCK_TRACE), plain run.
set -o pipefail
O=gpurun_out/r3c4t
mkdir -p $O
export TMPDIR=/tmp
PSOUP_BLOCK_TRACE=$O/blocks.jsonl timeout -k 10 400 python3 tools/baseline_configs.py --configs 4 --sky single --workdir /tmp/cfg --out $O/c4.jsonl > $O/c4.log 2>&1 || { echo C4_FAIL; tail -20 $O/c4.log; exit 1; }
cut -c1-300 $O/c4.jsonl
echo DONE
