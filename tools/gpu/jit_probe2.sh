#!/bin/bash
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache_probe2 SHREWD_FI_TRACE=1
timeout -k 10 300 python -u -X faulthandler -m pytest -s tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "translated_path" > gpurun_out/jit_probe2.log 2>&1
echo "rc=$?"; grep -v "^  File\|^Extension\|^Thread\|^Current\|^$" gpurun_out/jit_probe2.log | tail -30
