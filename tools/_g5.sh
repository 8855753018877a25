set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for v in "" "--flags 8" "--epoch 65536"; do
  timeout -k 10 200 python -u tools/diag.py crc32 --trials 64 100000 --converged $v > gpurun_out/diag_tx.log 2>&1; rc=$?
  echo "== $v"; grep -E "longest|converged|\"n\": 100000, \"kind\": \"faults\"|surv" gpurun_out/diag_tx.log | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
done
