#!/bin/bash
# correctness of the assembly interpreter changes, then tail trials, census, headline A/B
set -o pipefail
TAG=${1:-r05t}
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache LS_TOP=6
bash tools/gpu/gpu_tests.sh ${TAG}_t "known_answer or rewritten or dynamic_loop or odd_pc or trials_bit_exact or solo or m5_sim" || exit $?
for t in 631236 934410; do timeout -k 10 200 python -u tools/gpu/slow_trials.py qsort 0x5EED0003 regs_pc $t >> gpurun_out/${TAG}_slow.jsonl 2>&1 || exit $?; done
timeout -k 10 200 python -u tools/gpu/slow_trials.py intmix 0x5EED0002 regs_pc 53499 64617 >> gpurun_out/${TAG}_slow.jsonl 2>&1 &&
timeout -k 10 200 python -u tools/gpu/slow_trials.py crc32 0x5EED0002 regs_pc 70460 >> gpurun_out/${TAG}_slow.jsonl 2>&1 &&
timeout -k 10 200 python -u tools/gpu/launch_size.py qsort 1000000 0x5EED0003 1000000 > gpurun_out/${TAG}_census.jsonl 2> gpurun_out/${TAG}_census.err &&
timeout -k 10 200 python -u tools/gpu/launch_size.py intmix 1000000 0x5EED0003 1000000 >> gpurun_out/${TAG}_census.jsonl 2>> gpurun_out/${TAG}_census.err &&
bash tools/gpu/ab_bench.sh $TAG 2 default base/libshrewd_fi.so r04/libshrewd_fi.so
