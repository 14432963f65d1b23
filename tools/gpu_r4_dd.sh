#!/bin/bash
# Whole-DM-list dedispersion timing (config-4 list: 2000 DMs, 1024 ch, 2-bit, 2^20).
set -o pipefail
O=gpurun_out/r4dd
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/dedisp_bench.py --ndm 2000 --log2n 20 --reps 3 > $O/dd.log 2>&1 || { echo DD_FAIL; tail -20 $O/dd.log; exit 1; }
grep -v amdgpu.ids $O/dd.log | tail -4 | cut -c1-600
echo DONE
