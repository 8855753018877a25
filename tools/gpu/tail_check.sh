#!/bin/bash
# Parity subset + residency diagnostics + default bench (run via gpurun).
set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_tail.log 2>&1 &&
timeout -k 10 300 bash tools/gpu/occ_check.sh > /dev/null 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_tail.json 2> gpurun_out/bench_tail.err
rc=$?; tail -3 gpurun_out/pytest_tail.log; grep -v '"wave"' gpurun_out/occ.jsonl | cut -c1-260; grep '"wave"' gpurun_out/occ.jsonl | cut -c1-200 | head -30; cut -c1-300 gpurun_out/bench_tail.json; exit $rc
