set -o pipefail
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
for W in qsort intmix; do
timeout -k 10 300 python -u tools/diag.py $W --trials 100000 > gpurun_out/diag_$W.log 2>&1 || exit 1
cut -c1-1800 gpurun_out/diag_$W.log | grep -v amdgpu.ids
done
