#!/bin/bash
# A/B of the solo interpreter alone (static kernels, SOLO_ALL | NO_TRANSLATE)
# on tail trials, per library: bash tools/gpu/ab_interp.sh TAG LIB [LIB ...]
# (libraries under shrewd_amd/_lib/, built with shrewd_amd.build.build(out=...)).
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
out=gpurun_out/ab_interp_$TAG.jsonl
: > $out
for lib in "$@"; do
    for t in "crc32 70460" "qsort 46948" "intmix 53499" "intmix 64617"; do
        set -- $t
        echo "{\"lib\": \"$lib\"}" >> $out
        SHREWD_FI_LIB=$PWD/shrewd_amd/_lib/$lib SLOW_FLAGS=132 timeout -k 10 120 \
            python -u tools/gpu/slow_trials.py $1 0x5EED0002 regs_pc $2 >> $out 2>&1 || exit $?
    done
done
python - <<PY
import json
lib = None
for line in open("$out"):
    d = json.loads(line)
    if "lib" in d: lib = d["lib"]; continue
    print(lib, d["trial"], d["cls"], d["executed"], d["kernel_ms"], d["ns_per_inst"])
PY
