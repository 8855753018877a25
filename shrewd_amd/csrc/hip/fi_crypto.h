// fi_crypto.h -- RV64 scalar cryptography (Zbkb brev8, Zbkx xperm, Zknd/Zkne
// AES64, Zknh SHA-256/512, Zksed SM4, Zksh SM3) for the interpreter, written
// from the RISC-V scalar-crypto specification.  gem5 executes these through
// src/arch/riscv/rvk.hh (decoder.isa:1491-1531,1625-1630,2467-2613); the
// oracle links that header itself (oracle/rvk_ref.cc), and
// tests/test_crypto.py pins this port against it on the host and the device.
//
// Function numbers (the decoder's d.imm & 0xFF; RNUM / BS in d.imm >> 8):
//   0..3 sha256sum0/sum1/sig0/sig1   4..7 sha512sum0/sum1/sig0/sig1
//   8, 9 sm3p0/p1   10 aes64im   11 aes64ks1i   12 brev8   13 sm4ed   14 sm4ks
//   15..18 aes64es/esm/ds/dsm   19 aes64ks2   20 xperm4   21 xperm8
// 32-bit results (SHA-256, SM3, SM4) are sign-extended to 64 bits (Rd_sw).
#pragma once
#include "fi_rtc.h"

namespace fi {
namespace rvk {

// GF(2^8) tables built at compile time: the AES S-box (inverse modulo
// x^8+x^4+x^3+x+1, then the affine map b ^ rotl(b,1..4) ^ 0x63), its
// inverse, and the SM4 S-box (S(x) = A(I(A x + c)) + c with inversion modulo
// x^8+x^7+x^6+x^5+x^4+x^2+1, A the circulant of 0xA7, c = 0xD3).
struct Tables { uint8_t aes[256], aes_inv[256], sm4[256]; };

constexpr uint8_t gf_mul(uint8_t a, uint8_t b, uint32_t poly) {
    uint32_t r = 0, x = a;
    for (int i = 0; i < 8; i++) {
        if ((b >> i) & 1) r ^= x;
        x <<= 1;
        if (x & 0x100) x ^= poly;
    }
    return (uint8_t)r;
}
constexpr uint8_t gf_inv(uint8_t a, uint32_t poly) {
    // a^254 by square-and-multiply (0 -> 0)
    uint8_t r = 1, base = a;
    for (uint32_t e = 254; e; e >>= 1) {
        if (e & 1) r = gf_mul(r, base, poly);
        base = gf_mul(base, base, poly);
    }
    return a ? r : 0;
}
constexpr uint8_t rotl8(uint8_t x, int k) { return (uint8_t)((x << k) | (x >> ((8 - k) & 7))); }
constexpr uint8_t sm4_affine(uint8_t x) {
    uint8_t y = 0;
    for (int i = 0; i < 8; i++) {
        const uint8_t row = rotl8(0xA7, i);
        uint8_t p = (uint8_t)(row & x), par = 0;
        for (; p; p &= (uint8_t)(p - 1)) par ^= 1;
        y |= (uint8_t)(par << i);
    }
    return (uint8_t)(y ^ 0xD3);
}
constexpr Tables make_tables() {
    Tables t{};
    for (int x = 0; x < 256; x++) {
        const uint8_t b = gf_inv((uint8_t)x, 0x11B);
        const uint8_t s = (uint8_t)(b ^ rotl8(b, 1) ^ rotl8(b, 2) ^ rotl8(b, 3) ^ rotl8(b, 4) ^ 0x63);
        t.aes[x] = s;
        t.aes_inv[s] = (uint8_t)x;
        t.sm4[x] = sm4_affine(gf_inv(sm4_affine((uint8_t)x), 0x1F5));
    }
    return t;
}

#ifdef __HIP_DEVICE_COMPILE__
__constant__ const Tables kTab = make_tables();
#else
static const Tables kTab = make_tables();
#endif

__host__ __device__ inline uint32_t ror32(uint32_t x, int k) { return (x >> k) | (x << ((32 - k) & 31)); }
__host__ __device__ inline uint64_t ror64(uint64_t x, int k) { return (x >> k) | (x << ((64 - k) & 63)); }
__host__ __device__ inline uint64_t sx32(uint32_t x) { return (uint64_t)(int64_t)(int32_t)x; }
__host__ __device__ inline uint8_t byte_of(uint64_t x, int i) { return (uint8_t)(x >> (8 * i)); }

// xtime in AES's field
__host__ __device__ inline uint32_t xt(uint32_t b) { return ((b << 1) ^ ((b & 0x80) ? 0x1B : 0)) & 0xFF; }
// MixColumns / InvMixColumns of one 32-bit column (byte 0 = row 0)
__host__ __device__ inline uint32_t mix_col(uint32_t c, bool inv) {
    uint32_t b[4], r = 0;
    for (int i = 0; i < 4; i++) b[i] = (c >> (8 * i)) & 0xFF;
    for (int i = 0; i < 4; i++) {
        const uint32_t x0 = b[i], x1 = b[(i + 1) & 3], x2 = b[(i + 2) & 3], x3 = b[(i + 3) & 3];
        uint32_t v;
        if (!inv) {
            v = xt(x0) ^ (xt(x1) ^ x1) ^ x2 ^ x3;                                   // 2 3 1 1
        } else {
            auto m9 = [](uint32_t x) { return xt(xt(xt(x))) ^ x; };
            auto mb = [](uint32_t x) { return xt(xt(xt(x))) ^ xt(x) ^ x; };
            auto md = [](uint32_t x) { return xt(xt(xt(x))) ^ xt(xt(x)) ^ x; };
            auto me = [](uint32_t x) { return xt(xt(xt(x))) ^ xt(xt(x)) ^ xt(x); };
            v = me(x0) ^ mb(x1) ^ md(x2) ^ m9(x3);                                 // e b d 9
        }
        r |= (v & 0xFF) << (8 * i);
    }
    return r;
}
// The low 64 bits (columns 0, 1) of ShiftRows (or InvShiftRows) of the
// 128-bit state {rs2:rs1}, byte (row r, column c) at 4c + r, then SubBytes.
__host__ __device__ inline uint64_t aes64_round_lo(uint64_t rs1, uint64_t rs2, bool inv) {
    uint64_t r = 0;
    for (int c = 0; c < 2; c++)
        for (int row = 0; row < 4; row++) {
            const int src_c = (inv ? c - row + 4 : c + row) & 3;
            const int k = 4 * src_c + row;
            const uint8_t v = k < 8 ? byte_of(rs1, k) : byte_of(rs2, k - 8);
            r |= (uint64_t)(inv ? kTab.aes_inv[v] : kTab.aes[v]) << (8 * (4 * c + row));
        }
    return r;
}
__host__ __device__ inline uint64_t mix64(uint64_t x, bool inv) {
    return (uint64_t)mix_col((uint32_t)x, inv) | ((uint64_t)mix_col((uint32_t)(x >> 32), inv) << 32);
}
__host__ __device__ inline uint32_t sm4_sbox_rot(uint64_t rs2, int bs, bool ks) {
    const uint32_t sh = 8u * (uint32_t)(bs & 3);
    const uint32_t s = kTab.sm4[(rs2 >> sh) & 0xFF];
    const uint32_t x = ks ? s ^ ((s & 0x07) << 29) ^ ((s & 0xFE) << 7) ^ ((s & 1) << 23) ^ ((s & 0xF8) << 13)
                          : s ^ (s << 8) ^ (s << 2) ^ (s << 18) ^ ((s & 0x3F) << 26) ^ ((s & 0xC0) << 10);
    return sh ? (x << sh) | (x >> (32 - sh)) : x;
}
__host__ __device__ inline uint64_t xperm(uint64_t rs1, uint64_t rs2, int lg) {
    const int w = 1 << lg;
    const uint64_t mask = (1ULL << w) - 1;
    uint64_t r = 0;
    for (int i = 0; i < 64; i += w) {
        const uint64_t pos = ((rs2 >> i) & mask) << lg;
        if (pos < 64) r |= ((rs1 >> pos) & mask) << i;
    }
    return r;
}

__host__ __device__ inline uint64_t exec(int fn, uint64_t a, uint64_t b) {
    const uint32_t w = (uint32_t)a;
    const int sub = fn >> 8;
    switch (fn & 0xFF) {
    case 0: return sx32(ror32(w, 2) ^ ror32(w, 13) ^ ror32(w, 22));
    case 1: return sx32(ror32(w, 6) ^ ror32(w, 11) ^ ror32(w, 25));
    case 2: return sx32(ror32(w, 7) ^ ror32(w, 18) ^ (w >> 3));
    case 3: return sx32(ror32(w, 17) ^ ror32(w, 19) ^ (w >> 10));
    case 4: return ror64(a, 28) ^ ror64(a, 34) ^ ror64(a, 39);
    case 5: return ror64(a, 14) ^ ror64(a, 18) ^ ror64(a, 41);
    case 6: return ror64(a, 1) ^ ror64(a, 8) ^ (a >> 7);
    case 7: return ror64(a, 19) ^ ror64(a, 61) ^ (a >> 6);
    case 8: return sx32(w ^ ror32(w, 23) ^ ror32(w, 15));    // x ^ rol 9 ^ rol 17
    case 9: return sx32(w ^ ror32(w, 17) ^ ror32(w, 9));     // x ^ rol 15 ^ rol 23
    case 10: return mix64(a, true);
    case 11: {   // key schedule: SubWord(RotWord(hi word)) ^ rcon; RNUM > 9 skips rotate and rcon
        uint32_t t = (uint32_t)(a >> 32), rc = 0;
        if (sub < 10) {
            t = ror32(t, 8);
            rc = sub < 8 ? (1u << sub) : (sub == 8 ? 0x1Bu : 0x36u);
        }
        t = (uint32_t)kTab.aes[t & 0xFF] | ((uint32_t)kTab.aes[(t >> 8) & 0xFF] << 8) |
            ((uint32_t)kTab.aes[(t >> 16) & 0xFF] << 16) | ((uint32_t)kTab.aes[t >> 24] << 24);
        t ^= rc;
        return (uint64_t)t | ((uint64_t)t << 32);
    }
    case 12: {   // reverse the bits of every byte
        uint64_t x = a;
        x = ((x & 0x5555555555555555ULL) << 1) | ((x >> 1) & 0x5555555555555555ULL);
        x = ((x & 0x3333333333333333ULL) << 2) | ((x >> 2) & 0x3333333333333333ULL);
        return ((x & 0x0F0F0F0F0F0F0F0FULL) << 4) | ((x >> 4) & 0x0F0F0F0F0F0F0F0FULL);
    }
    case 13: return sx32(w ^ sm4_sbox_rot(b, sub, false));
    case 14: return sx32(w ^ sm4_sbox_rot(b, sub, true));
    case 15: return aes64_round_lo(a, b, false);
    case 16: return mix64(aes64_round_lo(a, b, false), false);
    case 17: return aes64_round_lo(a, b, true);
    case 18: return mix64(aes64_round_lo(a, b, true), true);
    case 19: {
        const uint32_t t = (uint32_t)(a >> 32) ^ (uint32_t)b;
        return (uint64_t)t ^ ((uint64_t)t << 32) ^ (b & 0xFFFFFFFF00000000ULL);
    }
    case 20: return xperm(a, b, 2);
    default: return xperm(a, b, 3);
    }
}

}  // namespace rvk
}  // namespace fi
