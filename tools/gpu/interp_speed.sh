set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
SLOW_FLAGS=132 timeout -k 10 200 python -u tools/gpu/slow_trials.py crc32 0x5EED0002 regs_pc 70460 > gpurun_out/interp.jsonl 2>&1 &&
SLOW_FLAGS=132 timeout -k 10 200 python -u tools/gpu/slow_trials.py qsort 0x5EED0002 regs_pc 46948 >> gpurun_out/interp.jsonl 2>&1 &&
bash tools/gpu/prof_solo.sh
cat gpurun_out/interp.jsonl
