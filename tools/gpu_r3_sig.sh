#!/bin/bash
# --signal bench sweep over the RFI amplitude (peaks per DM vs throughput)
set -o pipefail
O=${O:-gpurun_out/r3c}
mkdir -p $O
for amp in 0 0.02 0.05 0.1 0.3; do
  timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --signal --rfi-amp $amp > $O/sig_$amp.log 2>&1 || { echo SIG_FAIL $amp; tail -20 $O/sig_$amp.log; exit 1; }
  echo "amp $amp"; grep '^{"metric"' $O/sig_$amp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], c['peaks_per_dm'], c['host_distill_s_per_step'], c['candidates_after_distill'])"
done
