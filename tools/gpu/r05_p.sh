#!/bin/bash
# Round-5 check p: correctness of the round's kernel changes, slow trials per
# library build, the 1M census, the headline A/B.  bash tools/gpu/r05_p.sh TAG
set -o pipefail
TAG=${1:-r05p}
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache LS_TOP=6
bash tools/gpu/gpu_tests.sh ${TAG}_t "known_answer or m5_simulator or decode or rewritten or dynamic_loop or chunking or resource or odd_pc" || exit $?
for lib in ${SLOW_LIBS:-default base/libshrewd_fi.so}; do
    if [ "$lib" = default ]; then unset SHREWD_FI_LIB; else export SHREWD_FI_LIB=$PWD/shrewd_amd/_lib/$lib; fi
    echo "{\"lib\": \"$lib\"}" >> gpurun_out/${TAG}_slow.jsonl
    timeout -k 10 200 python -u tools/gpu/slow_trials.py qsort 0x5EED0003 regs_pc 631236 934410 >> gpurun_out/${TAG}_slow.jsonl 2>&1 || exit $?
    timeout -k 10 200 python -u tools/gpu/slow_trials.py intmix 0x5EED0002 regs_pc 53499 >> gpurun_out/${TAG}_slow.jsonl 2>&1 || exit $?
done
unset SHREWD_FI_LIB
timeout -k 10 200 python -u tools/gpu/launch_size.py qsort 1000000 0x5EED0003 1000000 > gpurun_out/${TAG}_census.jsonl 2> gpurun_out/${TAG}_census.err &&
timeout -k 10 200 python -u tools/gpu/launch_size.py intmix 1000000 0x5EED0003 1000000 >> gpurun_out/${TAG}_census.jsonl 2>> gpurun_out/${TAG}_census.err &&
bash tools/gpu/ab_bench.sh $TAG 2 default base/libshrewd_fi.so r04/libshrewd_fi.so &&
timeout -k 10 400 python -u bench.py --steps 10 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
