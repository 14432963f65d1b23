#!/bin/bash
set -o pipefail
O=gpurun_out/r4dbg
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/expt/screen_debug.py > $O/dbg.log 2>&1 || { echo DBG_FAIL; tail -30 $O/dbg.log; exit 1; }
cat $O/dbg.log | grep -v amdgpu.ids
