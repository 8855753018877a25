set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_fp.log 2>&1 &&
timeout -k 10 300 bash tools/gpu/occ_check.sh > /dev/null 2>&1
rc=$?; tail -5 gpurun_out/pytest_fp.log; cut -c1-330 gpurun_out/occ.jsonl; exit $rc
