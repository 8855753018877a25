set -o pipefail
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
for E in 4096 1024 2048 8192 16384; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --epoch-iters $E > gpurun_out/bench_e$E.json 2>gpurun_out/bench_e$E.err || exit 1
  python -c "import json;b=json.load(open('gpurun_out/bench_e$E.json'));print($E, round(b['value']), b['ms_per_step'], b['roofline']['avg_kernel_ms'])"
done
for W in qsort intmix; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --workload $W > gpurun_out/bench_$W.json 2>gpurun_out/bench_$W.err || exit 1
  python -c "import json;b=json.load(open('gpurun_out/bench_$W.json'));print('$W', round(b['value']), b['ms_per_step'], b['roofline']['avg_kernel_ms'], b['outcomes'])"
done
