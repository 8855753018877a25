# instruction-cache and wait counters of the trial kernel on qsort (separate --pmc passes)
set -o pipefail
O=$PWD/gpurun_out; export SHREWD_FI_JIT_CACHE=$O/jitcache TMPDIR=/tmp
timeout -k 10 200 python -u bench.py --no-cpu-baseline --workload qsort --steps 1 --warmup 0 > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_HITS SQC_DCACHE_MISSES -d $O/pmc_ic -o p --output-format csv -- python3 bench.py --no-cpu-baseline --workload qsort --steps 1 --warmup 0 > $O/pmc_ic.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS -d $O/pmc_sq -o p --output-format csv -- python3 bench.py --no-cpu-baseline --workload qsort --steps 1 --warmup 0 > $O/pmc_sq.log 2>&1 || exit 3
