#!/bin/bash
# A/B of build variants (SHREWD_FI_LIB=shrewd_amd/_lib/libshrewd_fi_VARIANT.so):
# chosen tail trials alone, then bench lines, per variant.  Run via gpurun:
# bash tools/gpu/ab_lib.sh "default t8" "intmix:64617,53499 crc32:70460" "crc32 intmix"
set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
O=gpurun_out/ab.jsonl
: > $O
for v in $1; do
    if [ "$v" = default ]; then unset SHREWD_FI_LIB; else export SHREWD_FI_LIB=$PWD/shrewd_amd/_lib/libshrewd_fi_$v.so; fi
    for wt in $2; do
        w=${wt%%:*}; ids=${wt#*:}
        echo "{\"variant\": \"$v\", \"workload\": \"$w\"}" >> $O
        timeout -k 10 240 python -u tools/gpu/slow_trials.py $w 0x5EED0002 regs_pc ${ids//,/ } >> $O 2>&1 || { cat $O; exit 1; }
    done
    for w in $3; do
        timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/ab_${v}_$w.json 2> gpurun_out/ab_${v}_$w.err || { cat $O; exit 1; }
        python -c "import json; d=json.load(open('gpurun_out/ab_${v}_$w.json')); print(json.dumps({'variant': '$v', 'bench': '$w', 'value': round(d['value']), 'ms': d['ms_per_step'], 'parity': d['parity']}))" >> $O
    done
done
cat $O
