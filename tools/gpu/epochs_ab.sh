#!/bin/bash
# Epoch schedules on the bench configuration: bash tools/gpu/epochs_ab.sh TAG "EPOCHS:ITERS ..." [WORKLOADS]
set -o pipefail
mkdir -p gpurun_out
TAG=$1; W=${3:-}
O=gpurun_out/epochs_$TAG.jsonl
: > $O
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
for v in $2; do
    ep=${v%%:*}; it=${v#*:}
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --workloads "$W" --extra-parity 0 --epochs $ep --epoch-iters $it \
        > gpurun_out/epochs_${TAG}_$ep_$it.json 2> gpurun_out/epochs_$TAG.err || exit $?
    python - >> $O <<PY
import json
d = json.loads(open("gpurun_out/epochs_${TAG}_$ep_$it.json").read().strip().splitlines()[-1])
r = {"epochs": $ep, "iters": $it, "crc32_ms": round(d["ms_per_step"], 3), "crc32": round(d["value"])}
for k, w in d.get("workloads", {}).items():
    r[k] = round(w["value"]); r[k + "_ms"] = round(w["ms_per_step"], 2)
print(json.dumps(r))
PY
done
cat $O
