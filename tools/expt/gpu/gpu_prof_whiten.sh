#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for f in 1084701955 1101479171; do
mkdir -p gpurun_out/pw_$f
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pw_$f -o bench --output-format csv -- python3 bench.py --log2n 20 --dms-per-gpu 32 --steps 10 --warmup 2 --fft4-flags $f > gpurun_out/pw_$f/bench.log 2>&1 || exit 1
done
echo DONE
