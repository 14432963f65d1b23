#!/bin/bash
# Pass A at K = 512: phase split, load-priority experiment, bench A/B; PMC
# bytes per kernel of the bench (one stream).
set -o pipefail
O=gpurun_out/r3prio
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/expt/passa_phases.py --K 256 --reps 4 --extra 0,512 > $O/passa.txt 2>&1 || { echo PHASES_FAIL; tail -20 $O/passa.txt; exit 1; }
grep extra $O/passa.txt
for r in 1 2; do
  for f in 1073954051 1073954563; do
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --fft4-flags $f > $O/bench_${f}_$r.log 2>&1 || { echo BENCH_FAIL $f; tail -20 $O/bench_${f}_$r.log; exit 1; }
    echo -n "flags $f rep $r: "; grep '^{"metric"' $O/bench_${f}_$r.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
  done
done
bash tools/gpu_pmc.sh r3prio/pmc --dms-per-gpu 2 && python3 tools/pmc_summary.py gpurun_out/r3prio/pmc/*/p_counter_collection.csv --match fft4,r2c_inter,harmonic_peaks,dedisperse > $O/pmc_summary.txt 2>&1; cat $O/pmc_summary.txt | head -80
echo DONE
