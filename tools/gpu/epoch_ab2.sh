#!/bin/bash
# qsort / intmix / crc32-memory bench over first-epoch budgets (run via gpurun)
set -o pipefail
mkdir -p gpurun_out/epoch_ab
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
for w in qsort intmix; do
for it in 4096 1024 2048; do
    timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --epoch-iters $it > gpurun_out/epoch_ab/$w$it.json 2> gpurun_out/epoch_ab/$w$it.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/epoch_ab/$w$it.json')); print('$w iters $it', round(d['value']), round(d['ms_per_step'], 2))"
done
done
