// fi_device.h -- wave-level helpers shared by the CDNA4 kernels.
#pragma once
#include "fi_rtc.h"

namespace fi {

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, l);
    uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t uni32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    return ((uint64_t)uni32((uint32_t)(v >> 32)) << 32) | uni32((uint32_t)v);
}
// Wave minimum by DPP row shifts and row broadcasts (every lane active; the
// result is uniform).  A 64-bit minimum is the minimum high word, then the
// minimum low word among the lanes that hold it.
__device__ __forceinline__ uint32_t dpp_min32(uint32_t v) {
    uint32_t t;
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x111, 0xF, 0xF, false); v = t < v ? t : v;  // row_shr:1
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x112, 0xF, 0xF, false); v = t < v ? t : v;  // row_shr:2
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x114, 0xF, 0xF, false); v = t < v ? t : v;  // row_shr:4
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x118, 0xF, 0xF, false); v = t < v ? t : v;  // row_shr:8
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x142, 0xA, 0xF, false); v = t < v ? t : v;  // row_bcast:15
    t = (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)v, 0x143, 0xC, 0xF, false); v = t < v ? t : v;  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint64_t wave_min64(uint64_t v) {
    const uint32_t hi = dpp_min32((uint32_t)(v >> 32));
    const uint32_t lo = dpp_min32((uint32_t)(v >> 32) == hi ? (uint32_t)v : 0xFFFFFFFFu);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += (uint64_t)__shfl_xor((unsigned long long)v, off, 64);
    return v;
}
__device__ __forceinline__ uint64_t sx32(uint64_t v) { return (uint64_t)(int64_t)(int32_t)(uint32_t)v; }
__device__ __forceinline__ int64_t sext64(uint64_t v, int n) { return (int64_t)(v << (64 - n)) >> (64 - n); }

}  // namespace fi
