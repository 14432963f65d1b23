#!/bin/bash
# 8-rank rehearsal of the distributed search on one GPU (gloo transport):
# dynamic DM queue vs static shards vs one rank, candidates compared byte for byte.
set -o pipefail
mkdir -p gpurun_out/dyn8
FIL=tests/data/tutorial.fil
for mode in dynamic static; do
  PSOUP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29541 -m peasoup_amd -i $FIL -o /tmp/dyn8_$mode --dm_end 1000 -n 4 --npdmp 8 --dm_schedule $mode --trace_json gpurun_out/dyn8/trace_$mode.json > gpurun_out/dyn8/$mode.log 2>&1 || { echo FAIL $mode; tail -20 gpurun_out/dyn8/$mode.log; exit 1; }
done
timeout -k 10 300 python -m peasoup_amd -i $FIL -o /tmp/dyn8_single --dm_end 1000 -n 4 --npdmp 8 --trace_json gpurun_out/dyn8/trace_single.json > gpurun_out/dyn8/single.log 2>&1 || { echo FAIL single; tail -20 gpurun_out/dyn8/single.log; exit 1; }
cmp /tmp/dyn8_dynamic/candidates.peasoup /tmp/dyn8_single/candidates.peasoup && echo "dynamic == single"
cmp /tmp/dyn8_static/candidates.peasoup /tmp/dyn8_single/candidates.peasoup && echo "static == single"
python3 - <<'PY'
import json
for m in ("dynamic", "static"):
    d = json.load(open(f"gpurun_out/dyn8/trace_{m}.json"))
    print(m, "ndm", d["config"]["ndm"], "per-rank blocks/trials:",
          [(r.get("dm_blocks"), r.get("accel_trials_planned")) for r in d["devices"]],
          "search_s max %.3f" % max(r["search_s"] for r in d["devices"]))
PY
