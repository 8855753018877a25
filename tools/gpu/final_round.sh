#!/bin/bash
# End-of-round evidence (run via gpurun): the round profile of the bench
# configuration (tools/gpu/profile_round.sh TAG), then the 1M-trial intmix
# north-star campaign with its 10k-trial oracle check.
set -o pipefail
TAG=${1:-r02}
mkdir -p gpurun_out
bash tools/gpu/profile_round.sh $TAG || exit $?
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 400 python -u tools/gpu/north_star.py > gpurun_out/north_star_$TAG.jsonl 2> gpurun_out/north_star_$TAG.err
rc=$?; cat gpurun_out/north_star_$TAG.jsonl; exit $rc
