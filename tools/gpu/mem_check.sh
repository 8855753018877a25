#!/bin/bash
# Residency of memory-fault campaigns (C4): crc32 and qsort, bursts 1 and 8.
set -o pipefail
mkdir -p gpurun_out
for w in "crc32 0x5EED0003 100000 0 0x200000000 1" "crc32 0x5EED0003 100000 0 0x200000000 8" \
         "qsort 0x5EED0003 100000 0 0x200000000 1"; do
  timeout -k 10 240 python -u tools/gpu/occupancy.py $w >> gpurun_out/mem_occ.jsonl || exit $?
done
