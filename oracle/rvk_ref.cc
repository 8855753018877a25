// rvk_ref.cc -- TEST INFRASTRUCTURE ONLY.
//
// A C entry point over the reference's scalar-cryptography helpers
// (src/arch/riscv/rvk.hh, included from /root/reference at build time by
// oracle/rvk_ref.mk; nothing of the header is copied here), so the oracle's
// Zkn/Zks instructions run the reference's own arithmetic.  The operand and
// result conversions are those of the generated execute() bodies
// (decoder.isa:1491-1531,1625-1630,2467-2529,2570-2613): `_sw` operands are
// the low 32 bits as int32_t and `Rd_sw` results are sign-extended, `_sd`
// operands and results are the full 64 bits.
#include <cstdint>

#include "arch/riscv/rvk.hh"

extern "C" uint64_t or_rvk_ref(int fn, uint64_t a, uint64_t b) {
    using namespace gem5::RiscvISA;
    const int64_t x = (int64_t)a, y = (int64_t)b;
    const int32_t xw = (int32_t)(uint32_t)a, yw = (int32_t)(uint32_t)b;
    const int sub = fn >> 8;
    int64_t r = 0;
    switch (fn & 0xFF) {
    case 0: r = _rvk_emu_sha256sum0(xw); break;
    case 1: r = _rvk_emu_sha256sum1(xw); break;
    case 2: r = _rvk_emu_sha256sig0(xw); break;
    case 3: r = _rvk_emu_sha256sig1(xw); break;
    case 4: r = _rvk_emu_sha512sum0(x); break;
    case 5: r = _rvk_emu_sha512sum1(x); break;
    case 6: r = _rvk_emu_sha512sig0(x); break;
    case 7: r = _rvk_emu_sha512sig1(x); break;
    case 8: r = _rvk_emu_sm3p0(xw); break;
    case 9: r = _rvk_emu_sm3p1(xw); break;
    case 10: r = _rvk_emu_aes64im(x); break;
    case 11: r = _rvk_emu_aes64ks1i(x, sub); break;
    case 12: r = _rvk_emu_brev8_64(x); break;
    case 13: r = _rvk_emu_sm4ed(xw, yw, (uint8_t)sub); break;
    case 14: r = _rvk_emu_sm4ks(xw, yw, (uint8_t)sub); break;
    case 15: r = _rvk_emu_aes64es(x, y); break;
    case 16: r = _rvk_emu_aes64esm(x, y); break;
    case 17: r = _rvk_emu_aes64ds(x, y); break;
    case 18: r = _rvk_emu_aes64dsm(x, y); break;
    case 19: r = _rvk_emu_aes64ks2(x, y); break;
    case 20: r = _rvk_emu_xperm4_64(x, y); break;
    case 21: r = _rvk_emu_xperm8_64(x, y); break;
    default: break;
    }
    return (uint64_t)r;
}
