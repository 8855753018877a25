set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
export SHREWD_FI_LIB=$PWD/shrewd_amd/_lib/libshrewd_fi_prof.so
PROF_FLAGS=128 timeout -k 10 200 python -u tools/gpu/prof_trial.py intmix 0x5EED0003 1864 > gpurun_out/prof_trial.jsonl 2>&1 &&
PROF_FLAGS=128 timeout -k 10 200 python -u tools/gpu/prof_trial.py qsort 0x5EED0003 344 89586 56077 >> gpurun_out/prof_trial.jsonl 2>&1 &&
PROF_FLAGS=0 timeout -k 10 200 python -u tools/gpu/prof_trial.py qsort 0x5EED0003 344 >> gpurun_out/prof_trial.jsonl 2>&1
rc=$?; cat gpurun_out/prof_trial.jsonl; exit $rc
