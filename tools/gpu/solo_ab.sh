#!/bin/bash
# A/B of the solo translated kernel's register placement and occupancy
# (SHREWD_FI_SOLO_VREG, SHREWD_FI_SOLO_WAVES): bench.py per variant, then the
# resource notes of each variant's code object.  Run via gpurun.
set -o pipefail
mkdir -p gpurun_out/solo_ab
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/solo_ab/jit
W=${WORKLOAD:-crc32}
run() {   # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 240 python -u bench.py --cpu-seconds 3 --steps 5 --warmup 1 --workload $W \
        > gpurun_out/solo_ab/$name.json 2> gpurun_out/solo_ab/$name.err || return 1
    python - "$name" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/solo_ab/{sys.argv[1]}.json"))
print(sys.argv[1], round(d["value"]), "trials/s", round(d["ms_per_step"], 2), "ms/step", d.get("parity"))
PY
}
timeout -k 10 200 python tools/gpu/dump_golden.py crc32 qsort intmix > gpurun_out/solo_ab/dump.log 2>&1 &&
run base &&
run vreg SHREWD_FI_SOLO_VREG=1 &&
run w4 SHREWD_FI_SOLO_WAVES=4 &&
run vreg_w4 SHREWD_FI_SOLO_VREG=1 SHREWD_FI_SOLO_WAVES=4 &&
run vreg_w6 SHREWD_FI_SOLO_VREG=1 SHREWD_FI_SOLO_WAVES=6
rc=$?
for f in gpurun_out/solo_ab/jit/*.co; do
    echo "== $f"; /opt/rocm/lib/llvm/bin/llvm-readelf --notes $f | grep -E "\.name:|vgpr_count|sgpr_count|spill_count|private_segment_fixed" | grep -B1 -A5 "tx_solo" | head -8
done
exit $rc
