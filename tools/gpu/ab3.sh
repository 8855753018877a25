#!/bin/bash
# headline + qsort + intmix A/B of library builds: bash tools/gpu/ab3.sh TAG ROUNDS LIB [LIB ...]
set -o pipefail
TAG=$1; R=$2; shift 2
bash tools/gpu/ab_bench.sh ${TAG}_crc $R "$@" &&
AB_ARGS="--workload qsort" bash tools/gpu/ab_bench.sh ${TAG}_qs $R "$@" &&
AB_ARGS="--workload intmix --trials 125000" bash tools/gpu/ab_bench.sh ${TAG}_im 1 "$@"
