set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "execution_paths or known_answer or bit_exact" > gpurun_out/pytest_simt.log 2>&1 &&
timeout -k 10 600 python -u tools/gpu/simt_sweep.py > gpurun_out/simt_sweep.jsonl 2>&1
rc=$?; tail -3 gpurun_out/pytest_simt.log; cat gpurun_out/simt_sweep.jsonl; exit $rc
