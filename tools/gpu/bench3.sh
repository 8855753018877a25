#!/bin/bash
# crc32 (the bench config), qsort and intmix bench lines (run via gpurun).
set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
for w in crc32 qsort intmix; do
    timeout -k 10 300 python -u bench.py --workload $w --cpu-seconds 3 > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/bench_$w.json')); print('$w', round(d['value']), round(d['ms_per_step'], 2), d['parity'])"
done
