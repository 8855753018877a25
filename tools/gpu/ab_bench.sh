#!/bin/bash
# A/B of library builds on the bench's headline workload only (no CPU
# baseline, no further workloads), alternating: bash tools/gpu/ab_bench.sh TAG ROUNDS LIB [LIB ...]
# (libraries under shrewd_amd/_lib/; "default" = libshrewd_fi.so)
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
mkdir -p gpurun_out
out=gpurun_out/ab_bench_$TAG.jsonl
: > $out
for r in $(seq $ROUNDS); do
    for lib in "$@"; do
        if [ "$lib" = default ]; then unset SHREWD_FI_LIB; else export SHREWD_FI_LIB=$PWD/shrewd_amd/_lib/$lib; fi
        timeout -k 10 300 python -u bench.py --workloads "" --no-cpu-baseline --steps 10 ${AB_ARGS} > gpurun_out/ab_one.json 2> gpurun_out/ab_one.err || exit $?
        python - "$lib" >> $out <<'PY'
import json, sys
d = json.load(open("gpurun_out/ab_one.json"))
print(json.dumps({"lib": sys.argv[1], "ms_per_step": round(d["ms_per_step"], 4), "value": round(d["value"]),
                  "per_kernel_ms": {k: round(v["ms_per_step"], 3) for k, v in d["roofline"]["per_kernel"].items()}}))
PY
    done
done
cat $out
