#!/bin/bash
# rocprofv3 passes of one bench workload on its own (run via gpurun):
# kernel trace + stats, FETCH_SIZE, WRITE_SIZE and the SQ issue counters,
# each in a separate pass with kernel tracing only, each time-limited and
# chained with &&.  Summarise with: python tools/pmc_summary.py TAG
#   bash tools/gpu/pmc_workload.sh r06q qsort 100000
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:?tag}
WL=${2:?workload}
T=${3:-100000}
mkdir -p $O
export TMPDIR=/tmp
export SHREWD_FI_JIT_CACHE=$O/jitcache
B="python $R/bench.py --workload $WL --trials $T --workloads "
cd /tmp
timeout -k 10 300 $B "" --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$TAG.json 2> $O/bench_$TAG.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_trace_$TAG -o trace --output-format csv -- \
    $B "" --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_trace_$TAG.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/prof_fetch_$TAG -o fetch --output-format csv -- \
    $B "" --steps 2 --warmup 0 --no-cpu-baseline > $O/prof_fetch_$TAG.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/prof_write_$TAG -o write --output-format csv -- \
    $B "" --steps 2 --warmup 0 --no-cpu-baseline > $O/prof_write_$TAG.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    -d $O/prof_sq_$TAG -o sq --output-format csv -- \
    $B "" --steps 2 --warmup 0 --no-cpu-baseline > $O/prof_sq_$TAG.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE \
    -d $O/prof_sqb_$TAG -o sqb --output-format csv -- \
    $B "" --steps 2 --warmup 0 --no-cpu-baseline > $O/prof_sqb_$TAG.log 2>&1
rc=$?
echo "pmc_workload $TAG $WL rc=$rc"
exit $rc
