#!/bin/bash
# Sweep trials per wave (first epoch) and per resumed wave on the default
# bench workload.  One bench line per setting -> gpurun_out/lanes_sweep.jsonl
set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
: > gpurun_out/lanes_sweep.jsonl
for cfg in "64 8" "64 16" "64 32" "64 64" "64 16" "64 8" "64 32"; do
    set -- $cfg
    echo "lanes=$1 resume=$2"
    timeout -k 10 150 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --lanes $1 --resume-lanes $2 \
        > gpurun_out/ls.json 2>> gpurun_out/lanes_sweep.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/ls.json')); print(json.dumps({'lanes': $1, 'resume': $2, 'value': d['value'], 'ms': d['ms_per_step'], 'kernel_ms': d['roofline']['avg_kernel_ms'], 'outcomes': d['outcomes']}))" \
        | tee -a gpurun_out/lanes_sweep.jsonl
done
