# PMC passes over one converged wave (interpreter and translated)
set -o pipefail
O=$PWD/gpurun_out; export SHREWD_FI_JIT_CACHE=$O/jitcache TMPDIR=/tmp
timeout -k 10 120 python -u tools/conv.py crc32 --interp > $O/conv.log 2>&1 && timeout -k 10 120 python -u tools/conv.py crc32 >> $O/conv.log 2>&1 || exit 1
cat $O/conv.log
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
for M in "--interp" ""; do
  T=c$([ -n "$M" ] && echo i || echo t)
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS -d $O/pmc_${T}1 -o p --output-format csv -- python3 tools/conv.py crc32 $M > /dev/null 2>&1 || exit 2
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_IFETCH SQ_INSTS_FLAT SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM -d $O/pmc_${T}2 -o p --output-format csv -- python3 tools/conv.py crc32 $M > /dev/null 2>&1 || exit 3
done
