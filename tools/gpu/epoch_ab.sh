#!/bin/bash
# crc32 bench over first-epoch budgets and epoch counts (run via gpurun)
set -o pipefail
mkdir -p gpurun_out/epoch_ab
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
for spec in "4096 2" "2048 2" "1024 2" "512 2" "8192 2" "1024 3"; do
    set -- $spec
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --epoch-iters $1 --epochs $2 > gpurun_out/epoch_ab/e$1_$2.json 2> gpurun_out/epoch_ab/e$1_$2.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/epoch_ab/e$1_$2.json')); print('iters $1 epochs $2', round(d['value']), round(d['ms_per_step'], 2))"
done
