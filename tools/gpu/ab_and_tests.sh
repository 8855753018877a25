#!/bin/bash
# Round-4 A/B: the solo interpreter alone per library (tools/gpu/ab_interp.sh),
# the parity tests that run through it, then bench lines per library.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu/ab_interp.sh r04i libshrewd_fi_base.so libshrewd_fi.so || exit $?
bash tools/gpu/gpu_tests.sh r04i "rewritten or known_answer or execution_paths or odd_pc or resource_redo or checkpoint or trials_bit_exact" || exit $?
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
for lib in libshrewd_fi_base.so libshrewd_fi.so libshrewd_fi_vc.so; do
    SHREWD_FI_LIB=$PWD/shrewd_amd/_lib/$lib timeout -k 10 400 python -u bench.py --no-cpu-baseline \
        > gpurun_out/bench_r04i_$lib.json 2> gpurun_out/bench_r04i_$lib.err || exit $?
    echo "== $lib"; python tools/bench_summary.py gpurun_out/bench_r04i_$lib.json
done
