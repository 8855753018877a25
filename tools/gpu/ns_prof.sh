set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 400 python -u tools/gpu/north_star.py > gpurun_out/north_star.jsonl 2> gpurun_out/north_star.err &&
bash tools/gpu/kernel_prof.sh r02e qsort 0x5EED0003
rc=$?; cat gpurun_out/north_star.jsonl; tail -3 gpurun_out/north_star.err; exit $rc
