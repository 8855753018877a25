set -o pipefail
mkdir -p gpurun_out; export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 200 python -u tools/gpu/ab_run.py w1 > gpurun_out/ab_w1.log 2>&1 &&
SHREWD_FI_WAVES_PER_EU=2 timeout -k 10 200 python -u tools/gpu/ab_run.py w2 > gpurun_out/ab_w2.log 2>&1 &&
SHREWD_FI_WAVES_PER_EU=2 timeout -k 10 200 python -u tools/gpu/ab_run.py w2r16 --resume-lanes 16 > gpurun_out/ab_w2r16.log 2>&1
rc=$?; cat gpurun_out/ab_w*.log; exit $rc
