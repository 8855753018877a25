set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 200 python -u tools/diag.py crc32 --trials 64 100000 --converged > gpurun_out/diag_tx.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/diag_tx.log | cut -c1-3000
exit $rc
