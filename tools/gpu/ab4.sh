set -o pipefail
mkdir -p gpurun_out; export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
run() { l=$1; shift; timeout -k 10 100 python -u tools/gpu/ab_run.py $l crc32 qsort "$@" >> gpurun_out/ab_ep.log 2>&1; }
run e4 && run e5 --epochs 5 && run e6 --epochs 6 && run b2k_e5 --epochs 5 --epoch-iters 2048 &&
run b8k_e4 --epoch-iters 8192 && run b8k_e5 --epochs 5 --epoch-iters 8192; rc=$?
cat gpurun_out/ab_ep.log; exit $rc
