#!/bin/bash
# 64-lane epochs before the solo dispatch (bench --epochs) at the default
# first-epoch budget, on the three bench workloads: bash tools/gpu/ep3_sweep_r05.sh
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ep3_sweep_r05.jsonl
: > $out
for wl in "crc32:" "qsort:--workload qsort" "intmix:--workload intmix --trials 125000"; do
  name=${wl%%:*}; args=${wl#*:}
  for ep in 2 3 2 3; do
    timeout -k 10 300 python -u bench.py --workloads "" --no-cpu-baseline --steps 6 --epochs $ep $args > gpurun_out/ep_one.json 2> gpurun_out/ep_one.err || exit $?
    python - "$name" "$ep" >> $out <<'PY'
import json, sys
d = json.load(open("gpurun_out/ep_one.json"))
print(json.dumps({"workload": sys.argv[1], "epochs": int(sys.argv[2]), "ms_per_step": round(d["ms_per_step"], 4), "value": round(d["value"])}))
PY
    tail -n 1 $out
  done
done
