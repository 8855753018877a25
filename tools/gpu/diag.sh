set -o pipefail
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 300 python -u tools/diag.py crc32 --trials 100000 --converged > gpurun_out/diag.log 2>&1; rc=$?
cut -c1-1500 gpurun_out/diag.log
exit $rc
