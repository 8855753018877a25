#!/bin/bash
# The qsort / intmix tail trials alone on the solo kernel: default, without
# snapshot checks, and FI_PROF phase stamps of the interpreter (run via gpurun
# after building shrewd_amd/_lib/libshrewd_fi_prof.so with -DFI_PROF).
set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
O=gpurun_out/tail_probe.jsonl
: > $O
timeout -k 10 200 python -u tools/gpu/slow_trials.py qsort 0x5EED0002 regs_pc 40699 91915 >> $O 2>&1 &&
SLOW_FLAGS=130 timeout -k 10 200 python -u tools/gpu/slow_trials.py qsort 0x5EED0002 regs_pc 40699 >> $O 2>&1 &&
timeout -k 10 300 python -u tools/gpu/slow_trials.py intmix 0x5EED0002 regs_pc 64617 >> $O 2>&1 &&
SHREWD_FI_LIB=$PWD/shrewd_amd/_lib/libshrewd_fi_prof.so PROF_FLAGS=128 timeout -k 10 200 \
    python -u tools/gpu/prof_trial.py qsort 0x5EED0002 40699 >> $O 2>&1
rc=$?; cat $O; exit $rc
