#!/bin/bash
set -o pipefail
O=${O:-gpurun_out/r3j}
mkdir -p $O
timeout -k 10 200 python -u tools/expt/passa_phases.py --only-full --extra 0,4194304,21971200,38748416,55525632,72302848,105857280 > $O/passa_stagger.txt 2>&1 || { echo PHASES_FAIL; tail -20 $O/passa_stagger.txt; exit 1; }
cat $O/passa_stagger.txt
