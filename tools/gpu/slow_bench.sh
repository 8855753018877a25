#!/bin/bash
# Tail trials alone on the solo kernel (default build), then the bench line
# for crc32 / qsort (run via gpurun).
set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
O=gpurun_out/slow.jsonl
: > $O
timeout -k 10 240 python -u tools/gpu/slow_trials.py crc32 0x5EED0002 regs_pc 70460 80709 >> $O 2>&1 &&
timeout -k 10 240 python -u tools/gpu/slow_trials.py qsort 0x5EED0002 regs_pc 46948 11487 >> $O 2>&1 &&
timeout -k 10 240 python -u tools/gpu/slow_trials.py intmix 0x5EED0002 regs_pc 64617 53499 34535 >> $O 2>&1 || { cat $O; exit 1; }
cat $O
for w in ${BENCH_WORKLOADS:-crc32 qsort}; do
    timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/bench_$w.json')); print('$w', round(d['value']), d['ms_per_step'], d['parity'])"
done
