#!/bin/bash
# Full GPU check (run via gpurun): every -m gpu test, the default bench, the
# 100k-trial tail profiles and the single-trial path speeds of the slowest
# intmix trial.  TAG names the output files.
set -o pipefail
TAG=${1:-r02}
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
timeout -k 10 300 python -u tools/gpu/tail_profile.py crc32 0x5EED0002 100000 > gpurun_out/tail_crc32_$TAG.log 2>&1 &&
timeout -k 10 300 python -u tools/gpu/tail_profile.py intmix 0x5EED0003 100000 > gpurun_out/tail_intmix_$TAG.log 2>&1 &&
timeout -k 10 300 python -u tools/gpu/tail_profile.py qsort 0x5EED0003 100000 > gpurun_out/tail_qsort_$TAG.log 2>&1 &&
timeout -k 10 300 python -u tools/gpu/path_speed.py intmix 0x5EED0003 1864 > gpurun_out/path_speed_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$TAG.log; cut -c1-400 gpurun_out/bench_$TAG.json; head -2 gpurun_out/tail_*_$TAG.log | cut -c1-300
cat gpurun_out/path_speed_$TAG.log
exit $rc
