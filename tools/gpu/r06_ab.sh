#!/bin/bash
# Round 6 translator A/B: a parity selection on the default library, then
# alternating bench runs of the listed libraries on crc32 and qsort.
#   bash tools/gpu/r06_ab.sh TAG "pytest -k expr"|none ROUNDS LIB [LIB ...]
set -o pipefail
TAG=$1; SEL=$2; ROUNDS=$3; shift 3
mkdir -p gpurun_out
if [ "$SEL" != none ]; then bash tools/gpu/gpu_tests.sh $TAG "$SEL" || exit $?; fi
AB_ARGS="--workload crc32" bash tools/gpu/ab_bench.sh ${TAG}_crc32 $ROUNDS "$@" || exit $?
AB_ARGS="--workload qsort --steps 5" bash tools/gpu/ab_bench.sh ${TAG}_qsort 1 "$@" || exit $?
