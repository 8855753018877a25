# A/B: translated blocks with / without the watched-register exits
set -o pipefail
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
for i in 1 2; do for V in "" 1; do for W in crc32 qsort; do
  SHREWD_FI_TX_NOWATCH=$V timeout -k 10 200 python -u bench.py --no-cpu-baseline --workload $W --steps 3 > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
  [ -z "$V" ] || unset SHREWD_FI_TX_NOWATCH
  python -c "import json;b=json.load(open('gpurun_out/ab.json'));print('nowatch=$V $W', round(b['value']), round(b['ms_per_step'],1))"
done; done; done
