#!/bin/bash
# Build variants chosen by environment: the crc32 bench line (and WORKLOADS)
# per variant, in the order given (repeat one to see the noise).  A variant
# is a SHREWD_FI_TXV value (clean-body bits, fi_translate.cpp) or VAR=VAL[,VAR=VAL]
# (e.g. SHREWD_FI_TX_WPE=2, fi_jit.cpp).  bash tools/gpu/txv_bench.sh TAG "V V ..." [WORKLOADS]
set -o pipefail
mkdir -p gpurun_out
TAG=$1; W=${3:-}
O=gpurun_out/txv_$TAG.jsonl
: > $O
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
k=0
for txv in $2; do
    k=$((k + 1))
    unset SHREWD_FI_TXV SHREWD_FI_TX_WPE
    if [[ $txv == *=* ]]; then for a in ${txv//,/ }; do export "$a"; done; else export SHREWD_FI_TXV=$txv; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --workloads "$W" --extra-parity 0 \
        > gpurun_out/txv_${TAG}_$k.json 2> gpurun_out/txv_${TAG}.err || exit $?
    python - >> $O <<PY
import json
d = json.loads(open("gpurun_out/txv_${TAG}_$k.json").read().strip().splitlines()[-1])
r = d["roofline"]["per_kernel"]
o = {"txv": "$txv", "value": round(d["value"]), "ms": round(d["ms_per_step"], 3),
     "solo_ms": r["fi_trial_kernel_tx_solo"]["avg_kernel_ms"], "parity": (d.get("parity") or {}).get("mismatches")}
for w, x in d.get("workloads", {}).items():
    o[w] = round(x["value"]); o[w + "_ms"] = round(x["ms_per_step"], 2)
print(json.dumps(o))
PY
done
cat $O
