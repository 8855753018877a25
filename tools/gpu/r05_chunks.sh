#!/bin/bash
# Round-5 chunk pipelining check: the chunking / redo / M5 GPU tests, the 1M
# qsort campaign as one launch and as 10 x 100k (outcomes compared), and a
# kernel trace of the 10-chunk run (host gaps between chunks).
# bash tools/gpu/r05_chunks.sh TAG
set -o pipefail
TAG=${1:-r05}
mkdir -p gpurun_out
export SHREWD_FI_JIT_CACHE=$PWD/gpurun_out/jitcache LS_TOP=4
bash tools/gpu/gpu_tests.sh ${TAG}_chunks "chunking or resource_redo" &&
timeout -k 10 200 python -u tools/gpu/launch_size.py qsort 1000000 0x5EED0003 1000000 100000 > gpurun_out/${TAG}_ls.jsonl 2> gpurun_out/${TAG}_ls.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_trace -o run -- python3 -u $GRAFT_REPO_ROOT/tools/gpu/launch_size.py qsort 1000000 0x5EED0003 100000 > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_trace.log 2>&1
