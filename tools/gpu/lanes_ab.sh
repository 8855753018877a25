#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
: > gpurun_out/lanes_ab_r05.jsonl
for rep in 1 2; do for l in 64 32 16; do for w in crc32 qsort; do
  timeout -k 10 200 python -u bench.py --workloads "" --no-cpu-baseline --steps 10 --workload $w --lanes $l > gpurun_out/la.json 2>> gpurun_out/lanes_ab.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/la.json')); print(json.dumps({'w': '$w', 'lanes': $l, 'ms': round(d['ms_per_step'],3), 'pk': {k: round(v['ms_per_step'],3) for k,v in d['roofline']['per_kernel'].items()}}))" >> gpurun_out/lanes_ab_r05.jsonl
done; done; done
cat gpurun_out/lanes_ab_r05.jsonl
