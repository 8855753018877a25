#!/bin/bash
# Alternating bench runs of the headline workload under different bench.py
# argument sets (engine knobs): bash tools/gpu/sweep_args.sh TAG ROUNDS "name=ARGS" ...
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
out=gpurun_out/sweep_$TAG.jsonl
: > $out
for r in $(seq $ROUNDS); do
    for spec in "$@"; do
        name=${spec%%=*}; args=${spec#*=}
        timeout -k 10 300 python -u bench.py --workloads "" --no-cpu-baseline --steps 10 $args \
            > gpurun_out/sw_one.json 2> gpurun_out/sw_one.err || exit $?
        python - "$name" >> $out <<'PY'
import json, sys
d = json.load(open("gpurun_out/sw_one.json"))
pk = d["roofline"]["per_kernel"]
print(json.dumps({"cfg": sys.argv[1], "ms_per_step": round(d["ms_per_step"], 4), "value": round(d["value"]),
                  "per_kernel_ms": {k: round(v["ms_per_step"], 3) for k, v in pk.items()}}))
PY
    done
done
cat $out
