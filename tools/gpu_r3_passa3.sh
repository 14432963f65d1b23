#!/bin/bash
set -o pipefail
O=${O:-gpurun_out/r3k}
mkdir -p $O
timeout -k 10 200 python -u tools/expt/passa_phases.py --extra 0,8388608 > $O/passa_wide.txt 2>&1 || { echo PHASES_FAIL; tail -20 $O/passa_wide.txt; exit 1; }
cat $O/passa_wide.txt
