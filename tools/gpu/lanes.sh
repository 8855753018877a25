set -o pipefail
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for L in 64 32 16 8; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --lanes $L > gpurun_out/bench_l$L.json 2>gpurun_out/bench_l$L.err || exit 1
  python -c "import json;b=json.load(open('gpurun_out/bench_l$L.json'));print($L, round(b['value']), b['ms_per_step'], b['roofline']['avg_kernel_ms'], b['roofline']['dispatches_per_step'], b['outcomes'])"
done
