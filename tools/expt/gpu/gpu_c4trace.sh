#!/bin/bash
# Config 4 (Python driver) under a kernel trace: GPU busy / idle over the
# search (tools/trace_gaps.py), and the same for the 2^20 bench.
set -o pipefail
O=gpurun_out/${1:-c4trace}
mkdir -p $O /tmp/cfgw
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --workdir /tmp/cfgw > $O/warm.log 2>&1 || { tail -10 $O/warm.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c4 -o c4 --output-format csv -- python3 tools/baseline_configs.py --configs 4 --workdir /tmp/cfgw > $O/c4.log 2>&1 || { tail -10 $O/c4.log; exit 1; }
python3 tools/trace_gaps.py $O/c4/c4_kernel_trace.csv > $O/c4_gaps.txt
head -30 $O/c4_gaps.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/b20 -o b20 --output-format csv -- python3 bench.py --log2n 20 --dms-per-gpu 32 --steps 10 --warmup 2 > $O/b20.log 2>&1 || { tail -10 $O/b20.log; exit 1; }
python3 tools/trace_gaps.py $O/b20/b20_kernel_trace.csv > $O/b20_gaps.txt
head -30 $O/b20_gaps.txt
gzip -f $O/c4/c4_kernel_trace.csv $O/b20/b20_kernel_trace.csv
echo DONE
