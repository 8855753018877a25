#!/bin/bash
# A/B of library builds: the solo interpreter alone per library
# (tools/gpu/ab_interp.sh), a parity-test selection on the default library,
# then bench lines per library.  Run via gpurun:
#   bash tools/gpu/ab_and_tests.sh TAG "LIB LIB ..." ["pytest -k expr" | none]
set -o pipefail
mkdir -p gpurun_out
TAG=$1; LIBS=$2; SEL=${3:-none}
bash tools/gpu/ab_interp.sh $TAG $LIBS || exit $?
if [ "$SEL" != none ]; then
    bash tools/gpu/gpu_tests.sh $TAG "$SEL" || exit $?
fi
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache
for lib in $LIBS; do
    SHREWD_FI_LIB=$PWD/shrewd_amd/_lib/$lib timeout -k 10 400 python -u bench.py --no-cpu-baseline \
        > gpurun_out/bench_${TAG}_$lib.json 2> gpurun_out/bench_${TAG}_$lib.err || exit $?
    echo "== $lib"; python tools/bench_summary.py gpurun_out/bench_${TAG}_$lib.json
done
