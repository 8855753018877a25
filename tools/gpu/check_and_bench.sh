#!/bin/bash
# A pytest -m gpu selection (or all of it), then the default bench line
# (crc32 headline + qsort / intmix under "workloads").  Run via gpurun:
#   bash tools/gpu/check_and_bench.sh TAG ["pytest -k expr" | all | none]
set -o pipefail
TAG=${1:-r04}
SEL=${2:-all}
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
if [ "$SEL" != "none" ]; then
    if [ "$SEL" = "all" ]; then K=(); else K=(-k "$SEL"); fi
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" \
        > gpurun_out/pytest_gpu_$TAG.log 2>&1
    rc=$?; tail -3 gpurun_out/pytest_gpu_$TAG.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_$TAG.log | head -5
    [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python tools/bench_summary.py gpurun_out/bench_$TAG.json
