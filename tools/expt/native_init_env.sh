#!/bin/bash
# Native golden run under the HIP code-object loading modes: the phase
# timers (trace_json) and the process wall time, 3 runs each, interleaved.
mkdir -p gpurun_out/init
A="-i tests/data/tutorial.fil --dm_end 250 --acc_start -5 --acc_end 5 -n 4 --npdmp 10"
for r in 1 2 3; do
for env in "HIP_ENABLE_DEFERRED_LOADING=1" "HIP_ENABLE_DEFERRED_LOADING=0"; do
  t0=$(date +%s.%N)
  env $env timeout -k 10 60 ./bin/peasoup $A -o /tmp/go --trace_json /tmp/t.json > /dev/null 2>&1 || { echo FAIL; exit 1; }
  t1=$(date +%s.%N)
  python3 -c "
import json; d=json.load(open('/tmp/t.json'))
p=d['performance']; print('$env', 'wall', round($t1-$t0,3), 'total', round(d['timers_s']['total'],4), 'device_init', round(p['phase_device_init_s'],4))"
done
done
