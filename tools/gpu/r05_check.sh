#!/bin/bash
# Round-5 check: slow-trial speeds, the 1M census (qsort, intmix) and the GPU
# test suite, outputs under gpurun_out/ with a tag.  bash tools/gpu/r05_check.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-r05}
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache LS_TOP=${LS_TOP:-12}
timeout -k 10 200 python -u tools/gpu/slow_trials.py qsort 0x5EED0003 regs_pc 934410 > gpurun_out/${TAG}_slow.jsonl 2>&1 &&
timeout -k 10 200 python -u tools/gpu/slow_trials.py intmix 0x5EED0002 regs_pc 53499 64617 >> gpurun_out/${TAG}_slow.jsonl 2>&1 &&
timeout -k 10 200 python -u tools/gpu/launch_size.py qsort 1000000 0x5EED0003 1000000 > gpurun_out/${TAG}_census.jsonl 2> gpurun_out/${TAG}_census.err &&
timeout -k 10 200 python -u tools/gpu/launch_size.py intmix 1000000 0x5EED0003 1000000 >> gpurun_out/${TAG}_census.jsonl 2>> gpurun_out/${TAG}_census.err &&
bash tools/gpu/gpu_tests.sh $TAG "$2"
