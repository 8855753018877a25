#!/bin/bash
# crc32 bench under JIT A/B knobs: bench_ab.sh NAME=ENV[,ENV] ... (run via gpurun)
set -o pipefail
mkdir -p gpurun_out/bench_ab
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/bench_ab/jit
W=${WORKLOAD:-crc32}
for spec in "$@"; do
    name=${spec%%=*}; envs=${spec#*=}
    env $(echo $envs | tr ',' ' ') timeout -k 10 300 python -u bench.py --workload $W --no-cpu-baseline \
        > gpurun_out/bench_ab/$name.json 2> gpurun_out/bench_ab/$name.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/bench_ab/$name.json')); print('$name', round(d['value']), round(d['ms_per_step'], 2))"
done
