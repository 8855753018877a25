// latency.hip -- dependent-chain latencies of the primitives the interpreter's
// fast loop is built from, one wave alone on the chip (gfx950).
//   hipcc --offload-arch=gfx950 -O3 latency.hip -o latency && ./latency
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((address_space(4))) const uint32_t cu32;
#define N 4096

__global__ void k_sload(const uint32_t *tab, uint64_t *out) {     // s_load chain (K$ hit)
    uint32_t i = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; k++) i = __builtin_amdgcn_readfirstlane(((cu32 *)(uintptr_t)tab)[i]);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = i; }
}
__global__ void k_memtime(uint64_t *out) {                      // back-to-back s_memtime
    uint64_t acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; k++) acc += __builtin_amdgcn_s_memtime();
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = acc; }
}
__global__ void k_lds(uint64_t *out) {                          // ds_read chain
    __shared__ uint32_t L[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) L[i] = (i * 7 + 1) & 1023;
    __syncthreads();
    uint32_t i = threadIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; k++) i = L[i];
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = i; }
}
__global__ void k_ldsrw(uint64_t *out) {                        // write then dependent read (register-file pattern)
    __shared__ uint64_t R[33 * 64];
    for (int i = 0; i < 33; i++) R[i * 64 + threadIdx.x] = i;
    uint32_t r = 1;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; k++) {
        uint64_t v = R[r * 64 + threadIdx.x];
        R[((r + 5) & 31) * 64 + threadIdx.x] = v + 1;
        r = __builtin_amdgcn_readfirstlane((uint32_t)(v & 31));
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r; }
}
__global__ void k_gload(const uint32_t *tab, uint64_t *out) {    // global_load chain (L2/L1 hit)
    uint32_t i = threadIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; k++) i = tab[i];
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = i; }
}
__global__ void k_gstload(uint32_t *buf, uint64_t *out) {        // store then dependent load of another address
    uint32_t i = threadIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; k++) {
        buf[2048 + ((i * 13 + k) & 1023) * 64 + threadIdx.x] = i;
        i = buf[i & 1023];
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = i; }
}
__global__ void k_branchtree(const uint32_t *kinds, uint64_t *out) { // uniform switch dispatch
    uint64_t v = threadIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; k++) {
        const uint32_t kind = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 3) & 15) ^ kinds[0];
        switch (kind) {
        case 0: v += 3; break; case 1: v ^= 0x55; break; case 2: v <<= 1; break; case 3: v >>= 1; break;
        case 4: v -= 7; break; case 5: v |= 9; break; case 6: v &= 0xFFFF; break; case 7: v *= 3; break;
        case 8: v += 11; break; case 9: v ^= 0x33; break; case 10: v += 1; break; case 11: v -= 1; break;
        case 12: v += 5; break; case 13: v ^= 1; break; case 14: v += 2; break; default: v += 9; break;
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = v; }
}

int main() {
    uint32_t *tab, *buf; uint64_t *out;
    hipMalloc(&tab, 1 << 20); hipMalloc(&buf, 64 << 20); hipMalloc(&out, 64);
    uint32_t h[1024];
    for (int i = 0; i < 1024; i++) h[i] = (i * 37 + 11) & 1023;
    hipMemcpy(tab, h, sizeof h, hipMemcpyHostToDevice);
    hipMemset(buf, 0, 64 << 20);
    uint64_t r[2];
    auto run = [&](const char *name) {
        hipDeviceSynchronize();
        hipMemcpy(r, out, 16, hipMemcpyDeviceToHost);
        printf("%-12s %8.1f cycles/iter\n", name, (double)r[0] / N);
    };
    for (int rep = 0; rep < 2; rep++) {
        k_sload<<<1, 64>>>(tab, out); run("s_load");
        k_memtime<<<1, 64>>>(out); run("s_memtime");
        k_lds<<<1, 64>>>(out); run("ds_read");
        k_ldsrw<<<1, 64>>>(out); run("ds_wr+rd");
        k_gload<<<1, 64>>>(tab, out); run("global_ld");
        k_gstload<<<1, 64>>>(buf, out); run("st+ld");
        k_branchtree<<<1, 64>>>(tab, out); run("switch16");
    }
    return 0;
}
