// branch.hip -- cost of scalar control flow vs branch-free selection (gfx950),
// one wave alone.  hipcc --offload-arch=gfx950 -O3 branch.hip -o branch
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define N 4096

__global__ void k_nottaken(const uint32_t *p, uint64_t *out) {   // 8 not-taken uniform branches per iter
    uint32_t x = p[0], acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; k++) {
        asm volatile(
            "s_cmp_eq_u32 %1, 12345\n s_cbranch_scc1 1f\n"
            "s_cmp_eq_u32 %1, 12346\n s_cbranch_scc1 1f\n"
            "s_cmp_eq_u32 %1, 12347\n s_cbranch_scc1 1f\n"
            "s_cmp_eq_u32 %1, 12348\n s_cbranch_scc1 1f\n"
            "s_cmp_eq_u32 %1, 12349\n s_cbranch_scc1 1f\n"
            "s_cmp_eq_u32 %1, 12350\n s_cbranch_scc1 1f\n"
            "s_cmp_eq_u32 %1, 12351\n s_cbranch_scc1 1f\n"
            "s_cmp_eq_u32 %1, 12352\n s_cbranch_scc1 1f\n"
            "s_add_u32 %0, %0, 1\n"
            "1:\n" : "+s"(acc) : "s"(x) : "scc");
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = acc; }
}
__global__ void k_taken(uint64_t *out) {    // 8 taken unconditional branches per iter
    uint32_t acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; k++) {
        asm volatile(
            "s_branch 1f\n s_nop 0\n 1: s_branch 2f\n s_nop 0\n 2: s_branch 3f\n s_nop 0\n 3: s_branch 4f\n s_nop 0\n"
            "4: s_branch 5f\n s_nop 0\n 5: s_branch 6f\n s_nop 0\n 6: s_branch 7f\n s_nop 0\n 7: s_branch 8f\n s_nop 0\n"
            "8: s_add_u32 %0, %0, 1\n" : "+s"(acc) :: "scc");
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = acc; }
}
__global__ void k_setpc(uint64_t *out) {    // 8 indirect jumps (s_getpc / s_add / s_setpc) per iter
    uint32_t acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; k++) {
        asm volatile(
#define HOP(i) "s_getpc_b64 s[40:41]\n" "LA" i "_%=: s_add_u32 s40, s40, LB" i "_%=-LA" i "_%=\n s_addc_u32 s41, s41, 0\n s_setpc_b64 s[40:41]\n s_nop 0\n" "LB" i "_%=:\n"
            HOP("1") HOP("2") HOP("3") HOP("4") HOP("5") HOP("6") HOP("7") HOP("8")
            "s_add_u32 %0, %0, 1\n" : "+s"(acc) :: "scc", "s40", "s41");
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = acc; }
}
__global__ void k_valu64(uint64_t *out) {   // 16 dependent 64-bit VALU adds per iter
    uint64_t v = threadIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; k++) {
#pragma unroll
        for (int j = 0; j < 16; j++) { v += (uint64_t)j * 0x100000001ULL; asm volatile("" : "+v"(v)); }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = v; }
}
__global__ void k_select(const uint32_t *p, uint64_t *out) {   // branch-free 12-way ALU with v_cndmask selection
    uint64_t a = threadIdx.x + 5, b = 3;
    uint32_t kind = p[0];
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; k++) {
        kind = __builtin_amdgcn_readfirstlane((uint32_t)a & 7);
        uint64_t r = a + b;
        r = kind == 1 ? a - b : r;
        r = kind == 2 ? (a & b) : r;
        r = kind == 3 ? (a | b) : r;
        r = kind == 4 ? (a ^ b) : r;
        r = kind == 5 ? (uint64_t)((int64_t)a < (int64_t)b) : r;
        r = kind == 6 ? (uint64_t)(a < b) : r;
        r = kind == 7 ? a << (b & 63) : r;
        a = r;
        asm volatile("" : "+v"(a));
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = a; }
}
__global__ void k_empty(uint64_t *out) {   // loop overhead only
    uint32_t acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < N; k++) asm volatile("s_add_u32 %0, %0, 1" : "+s"(acc) :: "scc");
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = acc; }
}

int main() {
    uint32_t *p; uint64_t *out;
    (void)hipMalloc(&p, 64); (void)hipMalloc(&out, 64);
    (void)hipMemset(p, 0, 64);
    uint64_t r[2];
    auto run = [&](const char *name, double per) {
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(r, out, 16, hipMemcpyDeviceToHost);
        printf("%-12s %8.1f cycles/iter  %6.1f per op\n", name, (double)r[0] / N, (double)r[0] / N / per);
    };
    for (int rep = 0; rep < 2; rep++) {
        k_empty<<<1, 64>>>(out); run("empty", 1);
        k_nottaken<<<1, 64>>>(p, out); run("8 nottaken", 8);
        k_taken<<<1, 64>>>(out); run("8 taken", 8);
        k_setpc<<<1, 64>>>(out); run("8 setpc", 8);
        k_valu64<<<1, 64>>>(out); run("16 valu64", 16);
        k_select<<<1, 64>>>(p, out); run("select8", 1);
    }
    return 0;
}
