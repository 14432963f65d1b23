#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/coinc /tmp/cfg5
timeout -k 10 300 python tools/baseline_configs.py --configs 1 --workdir /tmp/cfg5 > /dev/null 2>&1
timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'tools'); sys.argv=['x']
import baseline_configs as b
from peasoup_amd.parallel import dist as pdist
class A: pass
a=A(); a.workdir='/tmp/cfg5'; a.log2n=20
print(b._make_fb(a, pdist.init()))
" > gpurun_out/coinc/mk.txt 2>&1 || { tail -20 gpurun_out/coinc/mk.txt; exit 1; }
timeout -k 10 200 python -u tools/expt/coinc_timing.py /tmp/cfg5/cfg45_20.fil > gpurun_out/coinc/timing.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/coinc/timing.txt; exit $rc
