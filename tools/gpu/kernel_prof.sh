#!/bin/bash
# rocprofv3 kernel trace + SQ counter passes of one bench configuration, per
# kernel (run via gpurun).  TAG WORKLOAD SEED.  Counter passes run with kernel
# tracing only, each in its own process with a hard time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-r02}; W=${2:-crc32}; S=${3:-0x5EED0002}
mkdir -p $O
export TMPDIR=/tmp
export SHREWD_FI_JIT_CACHE=$O/jitcache
cd /tmp
B="python $R/bench.py --no-cpu-baseline --workload $W --seed $S"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kp_trace_$TAG -o trace --output-format csv -- \
    $B --steps 3 --warmup 1 > $O/kp_trace_$TAG.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    -d $O/kp_a_$TAG -o a --output-format csv -- $B --steps 1 --warmup 0 > $O/kp_a_$TAG.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE \
    -d $O/kp_b_$TAG -o b --output-format csv -- $B --steps 1 --warmup 0 > $O/kp_b_$TAG.log 2>&1
rc=$?
echo "kernel_prof rc=$rc"
tail -3 $O/kp_b_$TAG.log
exit $rc
