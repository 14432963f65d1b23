#!/bin/bash
# The native eager code-object test, the first chunk's launch time with
# deferred loading forced on (what the test guards against), and the launch
# microbenchmark plain and under the profiler.
set -o pipefail
O=gpurun_out/${1:-warm}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_pipeline_gpu.py -k "code_objects or block_pipeline" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for dl in 0 1; do
  HIP_ENABLE_DEFERRED_LOADING=$dl PSOUP_SCHED_TRACE=$O/sched_dl$dl.csv timeout -k 10 120 ./bin/peasoup -i tests/data/tutorial.fil -o /tmp/wo$dl --dm_end 250 --acc_start -5 --acc_end 5 -n 4 --npdmp 10 --trace_json $O/t_dl$dl.json > $O/dl$dl.log 2>&1 || { tail -5 $O/dl$dl.log; exit 1; }
  python3 - <<PY
ev=[l.split(",") for l in open("$O/sched_dl$dl.csv").read().splitlines()[2:]]
l=[float(e[0]) for e in ev if e[2]=="launch0"]; p=[float(e[0]) for e in ev if e[2]=="peek0"]
print("deferred=$dl first launch->peek ms", round(p[0]-l[0],3), "later", [round(b-a,3) for a,b in zip(l[1:],p[1:])])
PY
done
timeout -k 5 60 ./bin/expt/launch_cost > $O/lc_plain.txt 2>&1 && timeout -k 5 120 rocprofv3 --hip-trace --kernel-trace -d $O/prof -o p --output-format csv -- ./bin/expt/launch_cost > $O/lc_profiled.txt 2>&1 || exit 1
rm -rf $O/prof
paste -d'|' $O/lc_plain.txt $O/lc_profiled.txt | cut -c1-200
echo DONE
