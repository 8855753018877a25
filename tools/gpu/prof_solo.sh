#!/bin/bash
# FI_PROF phase cycles of tail trials on the solo kernel (interpreter only),
# run via gpurun after building shrewd_amd/_lib/libshrewd_fi_prof.so (-DFI_PROF).
set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_LIB=$PWD/shrewd_amd/_lib/libshrewd_fi_prof.so PROF_FLAGS=128
timeout -k 10 200 python -u tools/gpu/prof_trial.py crc32 0x5EED0002 80709 > gpurun_out/prof_solo.jsonl 2>&1 &&
timeout -k 10 200 python -u tools/gpu/prof_trial.py qsort 0x5EED0003 69076 56077 >> gpurun_out/prof_solo.jsonl 2>&1
rc=$?; cat gpurun_out/prof_solo.jsonl; exit $rc
