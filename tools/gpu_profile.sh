#!/bin/bash
# Bench + rocprofv3 profile passes on the GPU box (run via gpurun).  Each GPU
# step is time-limited and chained with &&; counters are collected in
# separate --pmc passes with kernel tracing only (no sys/runtime traces).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-r01}
STEPS=${STEPS:-5}
mkdir -p $O
export TMPDIR=/tmp
export SHREWD_FI_JIT_CACHE=$O/jitcache
cd /tmp
timeout -k 10 400 python $R/bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_trace_$TAG -o trace --output-format csv -- \
    python $R/bench.py --steps $STEPS --warmup 1 --no-cpu-baseline --workloads "" > $O/prof_trace_$TAG.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/prof_fetch_$TAG -o fetch --output-format csv -- \
    python $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --workloads "" > $O/prof_fetch_$TAG.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/prof_write_$TAG -o write --output-format csv -- \
    python $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --workloads "" > $O/prof_write_$TAG.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    -d $O/prof_sq_$TAG -o sq --output-format csv -- \
    python $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --workloads "" > $O/prof_sq_$TAG.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE \
    -d $O/prof_sqb_$TAG -o sqb --output-format csv -- \
    python $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --workloads "" > $O/prof_sqb_$TAG.log 2>&1
rc=$?
echo "profile rc=$rc"
exit $rc
