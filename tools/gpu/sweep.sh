# bench sweep: tools/gpu/sweep.sh "<workloads>" "<resume lanes>" "<epochs>" [extra bench args]
set -o pipefail
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
for W in $1; do for RL in $2; do for EP in $3; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 --workload $W --resume-lanes $RL --epochs $EP $4 > gpurun_out/sw.json 2>gpurun_out/sw.err || { tail -5 gpurun_out/sw.err; exit 1; }
  python -c "import json;b=json.load(open('gpurun_out/sw.json'));print('$W rl=$RL ep=$EP', round(b['value']), round(b['ms_per_step'],1), round(b['roofline']['avg_kernel_ms'],2), list(b['outcomes'].values()))"
done; done; done
