set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 200 python -u tools/gpu/occupancy.py qsort 0x5EED0003 > gpurun_out/occ.jsonl 2>&1 &&
timeout -k 10 200 python -u tools/gpu/occupancy.py crc32 0x5EED0002 >> gpurun_out/occ.jsonl 2>&1 &&
timeout -k 10 200 python -u tools/gpu/occupancy.py intmix 0x5EED0003 >> gpurun_out/occ.jsonl 2>&1
rc=$?; cut -c1-400 gpurun_out/occ.jsonl; exit $rc
