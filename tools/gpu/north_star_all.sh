#!/bin/bash
# N1 (BASELINE.json north star): 1M-trial crc32 and qsort campaigns (C2's
# MiBench-class kernels) with every trial checked against the oracle, and
# 1M intmix trials with 250k of them checked.  Run via gpurun.
set -o pipefail
TAG=${1:-r04}
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
for spec in crc32:1000000 qsort:1000000 intmix:250000; do
    w=${spec%%:*}; c=${spec#*:}
    timeout -k 10 600 python -u tools/gpu/north_star.py $w 1000000 0x5EED0003 $c > gpurun_out/north_star_${TAG}_$w.jsonl \
        2> gpurun_out/north_star_${TAG}_$w.err || exit $?
    tail -1 gpurun_out/north_star_${TAG}_$w.jsonl
done
