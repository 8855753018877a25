#!/bin/bash
# A/B of resume_lanes (trials per resumed wave) on the three campaign
# workloads; one bench line each -> gpurun_out/resume_ab.jsonl
set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
: > gpurun_out/resume_ab.jsonl
for w in qsort intmix crc32; do
  for r in 8 16 8 16; do
    echo "$w resume=$r"
    timeout -k 10 200 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --resume-lanes $r \
        > gpurun_out/ab.json 2>> gpurun_out/resume_ab.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print(json.dumps({'w': '$w', 'resume': $r, 'value': d['value'], 'ms': d['ms_per_step'], 'outcomes': d['outcomes']}))" \
        | tee -a gpurun_out/resume_ab.jsonl
  done
done
