#!/bin/bash
# Solo-kernel check: path parity tests, bench, tail profiles (run via gpurun).
set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "execution_paths or translated_path or known_answer" > gpurun_out/pytest_solo.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_solo.json 2> gpurun_out/bench_solo.err &&
timeout -k 10 300 python -u tools/gpu/tail_profile.py crc32 0x5EED0002 100000 > gpurun_out/tail_crc32.log 2>&1 &&
timeout -k 10 300 python -u tools/gpu/tail_profile.py intmix 0x5EED0003 100000 > gpurun_out/tail_intmix.log 2>&1 &&
timeout -k 10 300 python -u tools/gpu/tail_profile.py qsort 0x5EED0003 100000 > gpurun_out/tail_qsort.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_solo.log; cat gpurun_out/bench_solo.json | cut -c1-400; head -2 gpurun_out/tail_*.log | cut -c1-400
exit $rc
