#!/bin/bash
# Clean translated body variants (SHREWD_FI_TXV bits, fi_translate.cpp) per
# library: the crc32 bench line alone and crc32 trial 70460 on the
# translated solo path.  bash tools/gpu/txv_ab.sh TAG "LIB:TXV LIB:TXV ..."
set -o pipefail
mkdir -p gpurun_out
TAG=$1
O=gpurun_out/txv_$TAG.jsonl
: > $O
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
for v in $2; do
    lib=${v%%:*}; txv=${v#*:}
    export SHREWD_FI_LIB=$PWD/shrewd_amd/_lib/$lib SHREWD_FI_TXV=$txv
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --workloads "" --extra-parity 0 \
        > gpurun_out/txv_${TAG}_$lib_$txv.json 2> gpurun_out/txv_${TAG}.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/txv_${TAG}_$lib_$txv.json')); r=d['roofline']['per_kernel']; print(json.dumps({'lib': '$lib', 'txv': '$txv', 'value': round(d['value']), 'ms': round(d['ms_per_step'], 3), 'solo_ms': r['fi_trial_kernel_tx_solo']['avg_kernel_ms'], 'tx_ms': r['fi_trial_kernel_tx']['avg_kernel_ms']}))" >> $O
    SLOW_FLAGS=128 timeout -k 10 120 python -u tools/gpu/slow_trials.py crc32 0x5EED0002 regs_pc 70460 >> $O 2>&1 || exit $?
done
cat $O
