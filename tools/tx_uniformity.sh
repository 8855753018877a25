#!/bin/bash
# Offline check that the translated region compiles as uniform control flow:
# splice a translation body into the kernel, emit LLVM IR, run the uniformity
# analysis and list divergent branches that touch the translated blocks.
# usage: tools/tx_uniformity.sh body.inc
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/shrewd_amd/csrc
python3 -c "
import sys
s=open('$C/hip/fi_trial.hip').read(); b=open('$1').read()
open('/tmp/txk.hip','w').write('#define FI_TX 1\n'+s.replace('/*@TX_BODY@*/',b))"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I$C -I$C/hip -I$ROOT/include --cuda-device-only \
    -emit-llvm -S -o /tmp/txk.ll /tmp/txk.hip 2>/dev/null
/opt/rocm/lib/llvm/bin/opt -mtriple=amdgcn-amd-amdhsa -mcpu=gfx950 -passes='print<uniformity>' -disable-output \
    /tmp/txk.ll 2>/tmp/txk_uni.txt
awk '/UniformityInfo for function .*fi_trial_kernel/{on=1} on' /tmp/txk_uni.txt > /tmp/txk_uni_k.txt
echo "divergent terminators: $(grep -c 'DIVERGENT:.*\(br i1\|switch\)' /tmp/txk_uni_k.txt)"
