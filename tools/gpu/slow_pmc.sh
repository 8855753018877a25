#!/bin/bash
# SQ counters of one tail trial run alone on the solo kernel (machine
# instructions per guest instruction, wait share).  Run via gpurun.
set -o pipefail
mkdir -p gpurun_out/slow_pmc
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache TMPDIR=/tmp
R=$PWD
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    -d $R/gpurun_out/slow_pmc/a -o a --output-format csv -- python3 $R/tools/gpu/slow_trials.py ${SLOW_ARGS:-qsort 0x5EED0002 regs_pc 46948} \
    > $R/gpurun_out/slow_pmc/a.log 2>&1
rc=$?
cat $R/gpurun_out/slow_pmc/a.log | grep trial
exit $rc
