#!/bin/bash
# Escape census: campaigns C1-C5c with per-class escape
# breakdowns, then the 1M-trial intmix north-star run with a 100k-trial oracle
# check.  Usage (via gpurun): bash tools/gpu/census.sh TAG
set -o pipefail
TAG=${1:-r03}
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 500 python -u tools/campaigns.py $TAG > gpurun_out/campaigns_$TAG.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/gpu/north_star.py > gpurun_out/north_star_$TAG.jsonl 2> gpurun_out/north_star_$TAG.err
rc=$?; cat gpurun_out/north_star_$TAG.jsonl; exit $rc
