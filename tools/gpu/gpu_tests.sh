#!/bin/bash
# The GPU test suite (or a -k selection) with per-test time limits, output
# kept under gpurun_out/.  Usage (via gpurun): bash tools/gpu/gpu_tests.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-r03}
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
if [ -n "$2" ]; then SEL=(-k "$2"); else SEL=(); fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${SEL[@]}" \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu_$TAG.log; exit $rc
