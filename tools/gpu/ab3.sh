set -o pipefail
mkdir -p gpurun_out; export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/gpu/ab_run.py spread > gpurun_out/ab_spread.log 2>&1 &&
timeout -k 10 200 python -u tools/gpu/ab_run.py fixed --flags 32 > gpurun_out/ab_fixed.log 2>&1; rc=$?
cat gpurun_out/ab_spread.log gpurun_out/ab_fixed.log; exit $rc
