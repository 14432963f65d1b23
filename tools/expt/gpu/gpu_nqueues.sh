#!/bin/bash
# Native config 4: HIP launch cost and search time with the default hardware
# queues (4), with host-memory kernel arguments, with 8 queues and with
# ROC_ACTIVE_WAIT_TIMEOUT=0.
set -o pipefail
O=gpurun_out/${1:-nqueues}
mkdir -p $O /tmp/cfgw
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --native --workdir /tmp/cfgw --out $O/warm.jsonl > $O/warm.log 2>&1 || { tail -10 $O/warm.log; exit 1; }
ARGS=$(python3 -c "import json; print(' '.join(json.loads(open('$O/warm.jsonl').readline())['argv']))")
for v in default ka0 q8 aw0; do
  case $v in default) E="";; ka0) E="HIP_FORCE_DEV_KERNARG=0";; q8) E="GPU_MAX_HW_QUEUES=8";; aw0) E="ROC_ACTIVE_WAIT_TIMEOUT=0";; esac
  env $E timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d $O/$v -o t --output-format csv -- ./bin/peasoup $ARGS > $O/$v.log 2>&1 || { tail -10 $O/$v.log; exit 1; }
  echo "== $v"; python3 tools/expt/launch_stats.py $O/$v/t_hip_api_trace.csv $O/$v/t_kernel_trace.csv | head -6
  rm -f $O/$v/t_hip_api_trace.csv $O/$v/t_kernel_trace.csv
done
for rep in 1 2 3; do
  for v in default ka0 q8 aw0; do
    case $v in default) E="";; ka0) E="HIP_FORCE_DEV_KERNARG=0";; q8) E="GPU_MAX_HW_QUEUES=8";; aw0) E="ROC_ACTIVE_WAIT_TIMEOUT=0";; esac
    env $E timeout -k 10 300 python3 tools/baseline_configs.py --configs 4 --native --workdir /tmp/cfgw --out $O/c4_$v.jsonl > $O/n.log 2>&1 || { tail -10 $O/n.log; exit 1; }
  done
done
for v in default ka0 q8 aw0; do echo "== $v"; python3 tools/summarize_jsonl.py $O/c4_$v.jsonl timers_s.searching performance.phase_search_s; done
echo DONE
