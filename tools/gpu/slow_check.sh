#!/bin/bash
# Per-instruction cost of the tail trials, alone on the solo kernel: default
# build (translated), then the FI_PROF build without translation (phase stamps).
set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
O=gpurun_out/slow.jsonl
: > $O
for build in default prof; do
    if [ $build = prof ]; then export SHREWD_FI_LIB=$PWD/shrewd_amd/_lib/libshrewd_fi_prof.so SLOW_FLAGS=132; fi
    timeout -k 10 240 python -u tools/gpu/slow_trials.py qsort 0x5EED0003 regs_pc 69076 89586 56077 >> $O 2>&1 &&
    timeout -k 10 240 python -u tools/gpu/slow_trials.py intmix 0x5EED0003 regs_pc 1864 >> $O 2>&1 &&
    timeout -k 10 240 python -u tools/gpu/slow_trials.py crc32 0x5EED0002 regs_pc 80709 85533 >> $O 2>&1 || exit $?
    echo "== $build done" >> $O
done
cat $O
