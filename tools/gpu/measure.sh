#!/bin/bash
# Bench lines of the three campaign workloads (per-kernel roofline, parity)
# and the residency / slowest waves of each one's last dispatch (run via
# gpurun): tools/gpu/measure.sh TAG
set -o pipefail
TAG=${1:-r03}
O=gpurun_out/measure_$TAG
mkdir -p $O
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 300 python -u bench.py > $O/bench_crc32.json 2> $O/bench_crc32.err &&
timeout -k 10 300 python -u bench.py --workload qsort --cpu-seconds 5 --parity-trials 20000 > $O/bench_qsort.json 2> $O/bench_qsort.err &&
timeout -k 10 400 python -u bench.py --workload intmix --cpu-seconds 10 --parity-trials 20000 > $O/bench_intmix.json 2> $O/bench_intmix.err &&
timeout -k 10 200 python -u tools/gpu/occupancy.py crc32 0x5EED0002 > $O/occ_crc32.jsonl 2>&1 &&
timeout -k 10 200 python -u tools/gpu/occupancy.py qsort 0x5EED0002 > $O/occ_qsort.jsonl 2>&1 &&
timeout -k 10 300 python -u tools/gpu/occupancy.py intmix 0x5EED0002 > $O/occ_intmix.jsonl 2>&1
rc=$?
for w in crc32 qsort intmix; do
    python -c "import json,sys; d=json.load(open('$O/bench_$w.json')); r=d['roofline']; print('$w', round(d['value']), round(d['ms_per_step'],2), r['kernel'], {k: round(v['ms_per_step'],2) for k,v in r['per_kernel'].items()}, d['parity'])" 2>/dev/null
done
exit $rc
