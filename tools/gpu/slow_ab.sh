#!/bin/bash
# Tail trials alone on the solo kernel under JIT A/B knobs (run via gpurun).
set -o pipefail
mkdir -p gpurun_out/slow_ab
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/slow_ab/jit
one() {   # name, env...
    local n=$1; shift
    env "$@" timeout -k 10 200 python -u tools/gpu/slow_trials.py qsort 0x5EED0003 regs_pc 69076 89586 56077 > gpurun_out/slow_ab/$n.jsonl 2>&1 &&
    env "$@" timeout -k 10 200 python -u tools/gpu/slow_trials.py intmix 0x5EED0003 regs_pc 1864 >> gpurun_out/slow_ab/$n.jsonl 2>&1 &&
    env "$@" timeout -k 10 200 python -u tools/gpu/slow_trials.py crc32 0x5EED0002 regs_pc 80709 85533 >> gpurun_out/slow_ab/$n.jsonl 2>&1 &&
    python - $n <<'PY'
import json, sys
n = sys.argv[1]
rows = [json.loads(l) for l in open(f"gpurun_out/slow_ab/{n}.jsonl") if l.startswith("{")]
print(n, [(r["trial"], r["ns_per_inst"]) for r in rows])
PY
}
one base && one cx0 SHREWD_FI_SOLO_CX=0 && one w1 SHREWD_FI_SOLO_WAVES=1 && one cx0w1 SHREWD_FI_SOLO_CX=0 SHREWD_FI_SOLO_WAVES=1
rc=$?
for f in gpurun_out/slow_ab/jit/*.co; do
    /opt/rocm/lib/llvm/bin/llvm-readelf --notes $f | grep -E "\.name:|vgpr_count|sgpr_spill_count|vgpr_spill_count|private_segment_fixed" | grep -A4 "tx_solo"
done
exit $rc
