#!/bin/bash
set -o pipefail
O=${O:-gpurun_out/r3h}
mkdir -p $O
timeout -k 10 200 python -u tools/expt/passa_phases.py --extra 0,262144,4096,8192,32 > $O/passa_phases.txt 2>&1 || { echo PHASES_FAIL; tail -20 $O/passa_phases.txt; exit 1; }
cat $O/passa_phases.txt
