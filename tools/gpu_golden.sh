#!/bin/bash
# Quick GPU check: native CLI on the reference tutorial filterbank.
set -e
mkdir -p gpurun_out/golden
timeout -k 10 300 ./bin/peasoup -i tests/data/tutorial.fil -o gpurun_out/golden --dm_end 250 --acc_start -5 --acc_end 5 -n 4 --npdmp 10 -v > gpurun_out/golden/log.txt 2>&1
