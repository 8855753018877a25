#!/bin/bash
# Epoch/budget sweep of the bench configuration (run via gpurun).
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
out=gpurun_out/epoch_sweep.jsonl; : > $out
for cfg in "0 0" "2 4096" "2 1024" "2 16384" "3 4096" "2 256"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --epochs $1 --epoch-iters $2 > gpurun_out/es.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/es.json')); print(json.dumps({'epochs':$1,'iters':$2,'value':round(d['value']),'ms':round(d['ms_per_step'],2)}))" >> $out
  tail -1 $out
done
for w in qsort intmix; do
for cfg in "0 0" "2 4096" "2 16384"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --workload $w --seed 0x5EED0003 --steps 2 --epochs $1 --epoch-iters $2 > gpurun_out/es.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/es.json')); print(json.dumps({'w':'$w','epochs':$1,'iters':$2,'value':round(d['value']),'ms':round(d['ms_per_step'],2)}))" >> $out
  tail -1 $out
done; done
