#!/bin/bash
# Round 6: tick-domain GPU tests, then the 100k crc32 tick campaign checked
# trial by trial against the oracle.  Usage (via gpurun): bash tools/gpu/r06_tick.sh TAG
set -o pipefail
TAG=${1:-r06t}
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 600 python -u -m pytest tests/test_gpu_tick.py -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_tick_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_tick_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_tick_$TAG.log
timeout -k 10 500 python -u tools/gpu/tick_campaign.py crc32 100000 > gpurun_out/tick_crc32_$TAG.jsonl 2>&1
rc=$?; tail -2 gpurun_out/tick_crc32_$TAG.jsonl; exit $rc
