#!/bin/bash
# FI_PROF phase cycles of tail trials on the solo kernel (interpreter only),
# run via gpurun after building shrewd_amd/_lib/libshrewd_fi_prof.so (-DFI_PROF):
# python -c "from shrewd_amd import build as b; b.build(force=True, out='shrewd_amd/_lib/libshrewd_fi_prof.so', extra=['-DFI_PROF'])"
set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_LIB=$PWD/shrewd_amd/_lib/libshrewd_fi_prof.so PROF_FLAGS=128
timeout -k 10 200 python -u tools/gpu/prof_trial.py crc32 0x5EED0002 70460 > gpurun_out/prof_solo.jsonl 2>&1 &&
timeout -k 10 200 python -u tools/gpu/prof_trial.py qsort 0x5EED0002 46948 >> gpurun_out/prof_solo.jsonl 2>&1 &&
timeout -k 10 200 python -u tools/gpu/prof_trial.py intmix 0x5EED0002 53499 >> gpurun_out/prof_solo.jsonl 2>&1
rc=$?; cat gpurun_out/prof_solo.jsonl; exit $rc
