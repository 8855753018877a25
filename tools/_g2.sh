set -o pipefail
mkdir -p gpurun_out
for w in crc32 qsort intmix hello; do
SHREWD_FI_LIB=shrewd_amd/_lib/libshrewd_fi_prof.so timeout -k 10 120 python -u tools/diag.py $w --trials 64 > gpurun_out/prof_$w.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/prof_$w.log
done
