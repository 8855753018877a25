set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 300 python -u tools/gpu/tail_profile.py crc32 0x5EED0002 100000 > gpurun_out/tail_crc32.log 2>&1 &&
timeout -k 10 300 python -u tools/gpu/tail_profile.py qsort 0x5EED0003 100000 > gpurun_out/tail_qsort.log 2>&1 &&
timeout -k 10 300 python -u tools/gpu/tail_profile.py intmix 0x5EED0003 100000 > gpurun_out/tail_intmix.log 2>&1
rc=$?; cat gpurun_out/tail_*.log | cut -c1-600; exit $rc
