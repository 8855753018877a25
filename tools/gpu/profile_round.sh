#!/bin/bash
# Round profile of the bench configuration: bench + rocprofv3 trace/stats +
# HBM counters + SQ counters (tools/gpu_profile.sh), then the per-kernel SQ
# breakdown (tools/gpu/kernel_prof.sh).  TAG.
set -o pipefail
TAG=${1:-r02}
bash tools/gpu_profile.sh $TAG && bash tools/gpu/kernel_prof.sh ${TAG}k crc32 0x5EED0002
