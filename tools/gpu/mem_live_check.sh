#!/bin/bash
# Memory-fault parity (dead-word shortcut) then the C4 residency timelines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu \
  -k "trials_bit_exact or execution_paths or dead_memory or known_answer or chunking or argv or full_size" \
  > gpurun_out/pytest_mem.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_mem.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/mem_occ.jsonl
bash tools/gpu/mem_check.sh && grep -v '"wave"' gpurun_out/mem_occ.jsonl | cut -c1-200
