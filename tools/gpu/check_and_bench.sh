#!/bin/bash
# GPU parity suite, then the default bench line and a qsort/intmix bench (run via gpurun).
set -o pipefail
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
# (intmix: a 15 s CPU sample, so that its parity leg checks >= 20k trials)
for w in qsort:3 intmix:15; do
    s=${w#*:}; w=${w%%:*}
    timeout -k 10 300 python -u bench.py --workload $w --cpu-seconds $s > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/bench_$w.json')); print('$w', round(d['value']), d['ms_per_step'], d['parity'])"
done
