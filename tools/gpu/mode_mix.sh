#!/bin/bash
# mode_mix.py for several library builds: bash tools/gpu/mode_mix.sh TAG WORKLOAD LIB [LIB ...]
set -o pipefail
TAG=$1; W=$2; shift 2
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
for lib in "$@"; do
    if [ "$lib" = default ]; then unset SHREWD_FI_LIB; else export SHREWD_FI_LIB=$PWD/shrewd_amd/_lib/$lib; fi
    timeout -k 10 200 python -u tools/gpu/mode_mix.py $W >> gpurun_out/mode_mix_$TAG.jsonl 2>> gpurun_out/mode_mix_$TAG.err || exit $?
done
cat gpurun_out/mode_mix_$TAG.jsonl
