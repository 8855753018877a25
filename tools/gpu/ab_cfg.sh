#!/bin/bash
# A/B of library builds x engine flags on one bench workload, alternating:
#   bash tools/gpu/ab_cfg.sh TAG ROUNDS "name=LIB:FLAGS" ...
# LIB: "default" (libshrewd_fi.so) or a variant directory under shrewd_amd/_lib/;
# FLAGS: FI_CFG_* bits added through SHREWD_FI_EXTRA_FLAGS (0: none).
# AB_ARGS: extra bench.py arguments (e.g. "--workload qsort --steps 5").
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
out=gpurun_out/ab_cfg_$TAG.jsonl
: > $out
for r in $(seq $ROUNDS); do
    for spec in "$@"; do
        name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%:*}; flags=${rest#*:}
        if [ "$lib" = default ]; then unset SHREWD_FI_LIB; else export SHREWD_FI_LIB=$PWD/shrewd_amd/_lib/$lib/libshrewd_fi.so; fi
        export SHREWD_FI_EXTRA_FLAGS=$flags
        timeout -k 10 300 python -u bench.py --workloads "" --no-cpu-baseline --steps 10 ${AB_ARGS} \
            > gpurun_out/ab_one.json 2> gpurun_out/ab_one.err || exit $?
        python - "$name" >> $out <<'PY'
import json, sys
d = json.load(open("gpurun_out/ab_one.json"))
pk = d["roofline"]["per_kernel"]
print(json.dumps({"cfg": sys.argv[1], "ms_per_step": round(d["ms_per_step"], 4), "value": round(d["value"]),
                  "parity": d.get("parity"),
                  "per_kernel_ms": {k: round(v["ms_per_step"], 3) for k, v in pk.items()},
                  "busy_ms": {k: v.get("device_busy_ms") for k, v in pk.items()}}))
PY
    done
done
unset SHREWD_FI_EXTRA_FLAGS
cat $out
