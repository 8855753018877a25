// rv64_isa.h -- RV64 decode for the CDNA4 interpreter.
//
// Decode follows the decode tree of gem5's src/arch/riscv/isa/decoder.isa for
// rv_type = RV64 and enable_zcd = 1 (src/arch/riscv/RiscvISA.py:95,121-127);
// bitfields from isa/bitfields.isa:36-130.  Encodings gem5 decodes to an
// instruction this engine does not model (FP, vector, AMO, crypto, privileged
// SYSTEM, cbo, M5 ops, hypervisor loads) map to ESC_* ops and end the trial as
// an explicit ESCAPE outcome; encodings gem5 decodes to Unknown map to UNKNOWN.
// The function is evaluated on wave-uniform (scalar) operands by the
// pre-decode kernel and on the slow fetch path.
#pragma once
#include "fi_rtc.h"
#include "gem5_decode_table.h"

#define FI_OPS(X) \
    X(UNKNOWN) X(ESC_FP) X(ESC_VEC) X(ESC_AMO) X(ESC_SYS) X(ESC_CRYPTO) X(ESC_CBO) X(ESC_CMP) X(ESC_M5) X(ESC_HYP) \
    X(c_addi4spn) X(c_lw) X(c_ld) X(c_lbu) X(c_lhu) X(c_lh) X(c_sb) X(c_sh) X(c_sw) X(c_sd) \
    X(c_addi) X(c_addiw) X(c_li) X(c_addi16sp) X(c_lui) X(c_srli) X(c_srai) X(c_andi) \
    X(c_sub) X(c_xor) X(c_or) X(c_and) X(c_subw) X(c_addw) X(c_mul) \
    X(c_zext_b) X(c_sext_b) X(c_zext_h) X(c_sext_h) X(c_zext_w) X(c_not) \
    X(c_j) X(c_beqz) X(c_bnez) X(c_slli) X(c_lwsp) X(c_ldsp) X(c_jr) X(c_mv) X(c_ebreak) X(c_jalr) X(c_add) \
    X(c_swsp) X(c_sdsp) \
    X(lb) X(lh) X(lw) X(ld) X(lbu) X(lhu) X(lwu) X(fence) X(fence_i) \
    X(slli) X(bseti) X(bclri) X(binvi) X(clz) X(ctz) X(cpop) X(sext_b) X(sext_h) \
    X(addi) X(slti) X(sltiu) X(xori) X(srli) X(orc_b) X(srai) X(bexti) X(rori) X(rev8) \
    X(prefetch_i) X(prefetch_r) X(prefetch_w) X(ori_hint) X(ori) X(andi) X(auipc) \
    X(addiw) X(slliw) X(slli_uw) X(clzw) X(ctzw) X(cpopw) X(srliw) X(sraiw) X(roriw) \
    X(sb) X(sh) X(sw) X(sd) \
    X(add) X(sub) X(mul) X(sll) X(mulh) X(clmul) X(bset) X(bclr) X(rol) X(binv) \
    X(slt) X(mulhsu) X(clmulr) X(sh1add) X(sltu) X(mulhu) X(clmulh) \
    X(xor_) X(div_) X(pack) X(min_) X(sh2add) X(xnor) \
    X(srl) X(divu) X(czero_eqz) X(sra) X(minu) X(bext) X(ror) \
    X(or_) X(rem) X(max_) X(sh3add) X(orn) \
    X(and_) X(remu) X(packh) X(maxu) X(czero_nez) X(andn) \
    X(lui) X(addw) X(mulw) X(add_uw) X(subw) X(sllw) X(rolw) X(sh1add_uw) \
    X(divw) X(packw) X(sh2add_uw) X(srlw) X(divuw) X(sraw) X(rorw) X(remw) X(sh3add_uw) X(remuw) \
    X(beq) X(bne) X(blt) X(bge) X(bltu) X(bgeu) X(jalr) X(jal) \
    X(ecall) X(ebreak) X(csr) \
    X(flh) X(flw) X(fld) X(fsh) X(fsw) X(fsd) X(c_fld) X(c_fsd) X(c_fldsp) X(c_fsdsp) \
    X(fmv_x_w) X(fmv_x_d) X(fmv_x_h) X(fmv_w_x) X(fmv_d_x) X(fmv_h_x) \
    X(fsgnj_s) X(fsgnjn_s) X(fsgnjx_s) X(fsgnj_d) X(fsgnjn_d) X(fsgnjx_d) X(fsgnj_h) X(fsgnjn_h) X(fsgnjx_h) \
    X(fclass_s) X(fclass_d) X(fclass_h) \
    X(amoadd_w) X(amoswap_w) X(amoxor_w) X(amoor_w) X(amoand_w) X(amomin_w) X(amomax_w) X(amominu_w) X(amomaxu_w) \
    X(amoadd_d) X(amoswap_d) X(amoxor_d) X(amoor_d) X(amoand_d) X(amomin_d) X(amomax_d) X(amominu_d) X(amomaxu_d) \
    X(lr_w) X(sc_w) X(lr_d) X(sc_d) \
    X(fadd) X(fsub) X(fmul) X(fdiv) X(fsqrt) X(fmin) X(fmax) X(fmadd) X(fmsub) X(fnmsub) X(fnmadd) \
    X(feq) X(flt) X(fle) X(fcvt_f2i) X(fcvt_i2f) X(fcvt_f2f) \
    X(priv) X(cbo) X(m5op) X(crypto) X(fli) X(fround) X(fcvtmod) X(vec) X(vset)

namespace fi {

enum Op : uint8_t {
#define FI_X(n) OP_##n,
    FI_OPS(FI_X)
#undef FI_X
    OP_COUNT
};

struct Dec {
    uint32_t raw;
    int32_t imm;
    uint8_t op, rd, rs1, rs2, len, flags;  // flags: kPreRs1|kPreRs2|kPreRd
    uint16_t aux;
};

__host__ __device__ inline uint32_t fbits(uint32_t v, int hi, int lo) {
    return (v >> lo) & ((1u << (hi - lo + 1)) - 1u);
}
__host__ __device__ inline int32_t fsext(uint32_t v, int n) { return (int32_t)(v << (32 - n)) >> (32 - n); }

#define D_RD(r) (d.rd = (uint8_t)(r), d.flags |= 16)
#define D_RS1(r) (d.rs1 = (uint8_t)(r), d.flags |= 4)
#define D_RS2(r) (d.rs2 = (uint8_t)(r), d.flags |= 8)

__device__ inline Dec rv_decode_tree(uint32_t raw) {
    Dec d;
    d.raw = raw; d.imm = 0; d.op = OP_UNKNOWN; d.rd = d.rs1 = d.rs2 = 0; d.flags = 0; d.aux = 0;
    const uint32_t q = raw & 3;
    if (q != 3) {  // compressed, decoder.isa:43-536
        raw &= 0xFFFF; d.raw = raw; d.len = 2;
        const uint32_t cop = fbits(raw, 15, 13);
        const uint32_t rp1 = 8 + fbits(raw, 9, 7), rp2 = 8 + fbits(raw, 4, 2);
        const uint32_t rc1 = fbits(raw, 11, 7), rc2 = fbits(raw, 6, 2);
        const uint32_t cimm5 = fbits(raw, 6, 2), cimm1 = fbits(raw, 12, 12), cimm3 = fbits(raw, 12, 10);
        const uint32_t cimm2 = fbits(raw, 6, 5), cimm6 = fbits(raw, 12, 7), cimm8 = fbits(raw, 12, 5);
        if (q == 0) {
            switch (cop) {
            case 0: d.op = OP_c_addi4spn; D_RD(rp2); D_RS1(2);
                d.imm = (fbits(cimm8, 1, 1) << 2) | (fbits(cimm8, 0, 0) << 3) | (fbits(cimm8, 7, 6) << 4) |
                        (fbits(cimm8, 5, 2) << 6);
                return d;
            case 1: d.op = OP_c_fld; d.rd = (uint8_t)rp2; D_RS1(rp1); d.imm = (cimm3 << 3) | (cimm2 << 6); return d;
            case 2: d.op = OP_c_lw; D_RD(rp2); D_RS1(rp1);
                d.imm = (fbits(cimm2, 1, 1) << 2) | (cimm3 << 3) | (fbits(cimm2, 0, 0) << 6); return d;
            case 3: d.op = OP_c_ld; D_RD(rp2); D_RS1(rp1); d.imm = (cimm3 << 3) | (cimm2 << 6); return d;
            case 4:
                switch (fbits(raw, 12, 10)) {
                case 0: d.op = OP_c_lbu; D_RD(rp2); D_RS1(rp1); d.imm = (fbits(cimm2, 0, 0) << 1) | fbits(cimm2, 1, 1); return d;
                case 1: d.op = fbits(raw, 6, 6) ? OP_c_lh : OP_c_lhu; D_RD(rp2); D_RS1(rp1); d.imm = fbits(cimm2, 0, 0) << 1; return d;
                case 2: d.op = OP_c_sb; D_RS1(rp1); D_RS2(rp2); d.imm = (fbits(cimm2, 0, 0) << 1) | fbits(cimm2, 1, 1); return d;
                case 3: d.op = OP_c_sh; D_RS1(rp1); D_RS2(rp2); d.imm = fbits(cimm2, 0, 0) << 1; return d;
                default: return d;
                }
            case 5: d.op = OP_c_fsd; d.rs2 = (uint8_t)rp2; D_RS1(rp1); d.imm = (cimm3 << 3) | (cimm2 << 6); return d;
            case 6: d.op = OP_c_sw; D_RS1(rp1); D_RS2(rp2);
                d.imm = (fbits(cimm2, 1, 1) << 2) | (cimm3 << 3) | (fbits(cimm2, 0, 0) << 6); return d;
            default: d.op = OP_c_sd; D_RS1(rp1); D_RS2(rp2); d.imm = (cimm3 << 3) | (cimm2 << 6); return d;
            }
        }
        if (q == 1) {
            switch (cop) {
            case 0: d.op = OP_c_addi; D_RD(rc1); D_RS1(rc1); d.imm = fsext(cimm5 | (cimm1 << 5), 6); return d;
            case 1: d.op = OP_c_addiw; D_RD(rc1); D_RS1(rc1); d.imm = fsext(cimm5 | (cimm1 << 5), 6); return d;
            case 2: d.op = OP_c_li; D_RD(rc1); d.imm = fsext(cimm5 | (cimm1 << 5), 6); return d;
            case 3:
                if (rc1 == 2) {
                    d.op = OP_c_addi16sp; D_RD(2); D_RS1(2);
                    d.imm = fsext((fbits(cimm5, 4, 4) << 4) | (fbits(cimm5, 0, 0) << 5) | (fbits(cimm5, 3, 3) << 6) |
                                  (fbits(cimm5, 2, 1) << 7) | (cimm1 << 9), 10);
                } else {
                    d.op = OP_c_lui; D_RD(rc1); d.imm = fsext(cimm5 | (cimm1 << 5), 6) * 4096;
                }
                return d;
            case 4:
                switch (fbits(raw, 11, 10)) {
                case 0: d.op = OP_c_srli; D_RD(rp1); D_RS1(rp1); d.imm = cimm5 | (cimm1 << 5); return d;
                case 1: d.op = OP_c_srai; D_RD(rp1); D_RS1(rp1); d.imm = cimm5 | (cimm1 << 5); return d;
                case 2: d.op = OP_c_andi; D_RD(rp1); D_RS1(rp1); d.imm = fsext(cimm5 | (cimm1 << 5), 6); return d;
                default: {
                    const uint32_t f2 = fbits(raw, 6, 5);
                    // (no local lookup arrays: they would live in scratch memory)
                    if (!cimm1) { d.op = (uint8_t)(OP_c_sub + f2); D_RD(rp1); D_RS1(rp1); D_RS2(rp2); return d; }
                    if (f2 < 3) { d.op = (uint8_t)(OP_c_subw + f2); D_RD(rp1); D_RS1(rp1); D_RS2(rp2); return d; }
                    const uint32_t sel = fbits(raw, 4, 2);
                    if (sel > 5) return d;
                    d.op = (uint8_t)(OP_c_zext_b + sel); D_RD(rp1); D_RS1(rp1); return d;
                }
                }
            case 5:
                d.op = OP_c_j;
                d.imm = fsext((fbits(raw, 5, 3) << 1) | (fbits(raw, 11, 11) << 4) | (fbits(raw, 2, 2) << 5) |
                              (fbits(raw, 7, 7) << 6) | (fbits(raw, 6, 6) << 7) | (fbits(raw, 10, 9) << 8) |
                              (fbits(raw, 8, 8) << 10) | (fbits(raw, 12, 12) << 11), 12);
                return d;
            default:
                d.op = cop == 6 ? OP_c_beqz : OP_c_bnez; D_RS1(rp1);
                d.imm = fsext((fbits(cimm5, 2, 1) << 1) | (fbits(cimm3, 1, 0) << 3) | (fbits(cimm5, 0, 0) << 5) |
                              (fbits(cimm5, 4, 3) << 6) | (fbits(cimm3, 2, 2) << 8), 9);
                return d;
            }
        }
        switch (cop) {  // q == 2
        case 0: d.op = OP_c_slli; D_RD(rc1); D_RS1(rc1); d.imm = cimm5 | (cimm1 << 5); return d;
        case 1: d.op = OP_c_fldsp; d.rd = (uint8_t)rc1; D_RS1(2);
            d.imm = (fbits(cimm5, 4, 3) << 3) | (cimm1 << 5) | (fbits(cimm5, 2, 0) << 6); return d;
        case 2: d.op = OP_c_lwsp; D_RD(rc1); D_RS1(2);
            d.imm = (fbits(cimm5, 4, 2) << 2) | (cimm1 << 5) | (fbits(cimm5, 1, 0) << 6); return d;
        case 3: d.op = OP_c_ldsp; D_RD(rc1); D_RS1(2);
            d.imm = (fbits(cimm5, 4, 3) << 3) | (cimm1 << 5) | (fbits(cimm5, 2, 0) << 6); return d;
        case 4:
            if (!cimm1) {
                if (rc2 == 0) { d.op = OP_c_jr; D_RS1(rc1); }
                else { d.op = OP_c_mv; D_RD(rc1); D_RS2(rc2); }
            } else if (rc2 == 0) {
                if (rc1 == 0) d.op = OP_c_ebreak;
                else { d.op = OP_c_jalr; D_RD(1); D_RS1(rc1); }
            } else { d.op = OP_c_add; D_RD(rc1); D_RS1(rc1); D_RS2(rc2); }
            return d;
        case 5: d.op = OP_c_fsdsp; d.rs2 = (uint8_t)rc2; D_RS1(2);
            d.imm = (fbits(cimm6, 5, 3) << 3) | (fbits(cimm6, 2, 0) << 6); return d;
        case 6: d.op = OP_c_swsp; D_RS1(2); D_RS2(rc2); d.imm = (fbits(cimm6, 5, 2) << 2) | (fbits(cimm6, 1, 0) << 6); return d;
        default: d.op = OP_c_sdsp; D_RS1(2); D_RS2(rc2); d.imm = (fbits(cimm6, 5, 3) << 3) | (fbits(cimm6, 2, 0) << 6); return d;
        }
    }
    // 32-bit, decoder.isa:537-6365
    d.len = 4;
    const uint32_t opc = fbits(raw, 6, 2), f3 = fbits(raw, 14, 12), f7 = fbits(raw, 31, 25);
    const uint32_t rd = fbits(raw, 11, 7), rs1 = fbits(raw, 19, 15), rs2 = fbits(raw, 24, 20);
    const uint32_t fs3 = fbits(raw, 31, 27);
    const int32_t imm_i = fsext(fbits(raw, 31, 20), 12);
    const int32_t imm_s = fsext((fbits(raw, 31, 25) << 5) | fbits(raw, 11, 7), 12);
    const int32_t imm_b = fsext((fbits(raw, 31, 31) << 12) | (fbits(raw, 7, 7) << 11) | (fbits(raw, 30, 25) << 5) |
                                (fbits(raw, 11, 8) << 1), 13);
    const int32_t imm_j = fsext((fbits(raw, 31, 31) << 20) | (fbits(raw, 19, 12) << 12) | (fbits(raw, 20, 20) << 11) |
                                (fbits(raw, 30, 21) << 1), 21);
    const int32_t imm_u = (int32_t)(raw & 0xFFFFF000u);
    const uint32_t sh6 = fbits(raw, 25, 20), sh5 = fbits(raw, 24, 20);
    d.aux = (uint16_t)f3;
#define RI(o, im) do { d.op = (o); D_RD(rd); D_RS1(rs1); d.imm = (im); return d; } while (0)
#define RR(o) do { d.op = (o); D_RD(rd); D_RS1(rs1); D_RS2(rs2); return d; } while (0)
    switch (opc) {
    case 0x00: {  // LOAD :538-566
        if (f3 == 7) return d;
        RI((uint8_t)(OP_lb + f3), imm_i);
    }
    case 0x01: d.op = OP_ESC_FP; return d;
    case 0x03:  // MISC-MEM :1336-1433
        if (f3 == 0) { d.op = OP_fence; return d; }
        if (f3 == 1) { d.op = OP_fence_i; return d; }
        if (f3 == 2 && rd == 0) {
            const uint32_t f12 = fbits(raw, 31, 20);
            if (f12 == 0 || f12 == 1 || f12 == 2 || f12 == 4) d.op = OP_ESC_CBO;
        }
        return d;
    case 0x04:  // OP-IMM :1435-1670
        switch (f3) {
        case 0: RI(OP_addi, imm_i);
        case 1:
            if (fs3 == 0x00) RI(OP_slli, sh6);
            if (fs3 == 0x02 && rs2 <= 9) { d.op = OP_ESC_CRYPTO; return d; }
            if (fs3 == 0x05) RI(OP_bseti, sh6);
            if (fs3 == 0x06) { d.op = OP_ESC_CRYPTO; return d; }
            if (fs3 == 0x09) RI(OP_bclri, sh6);
            if (fs3 == 0x0d) RI(OP_binvi, sh6);
            if (fs3 == 0x0c) {
                if (rs2 == 0) RI(OP_clz, 0);
                if (rs2 == 1) RI(OP_ctz, 0);
                if (rs2 == 2) RI(OP_cpop, 0);
                if (rs2 == 4) RI(OP_sext_b, 0);
                if (rs2 == 5) RI(OP_sext_h, 0);
            }
            return d;
        case 2: RI(OP_slti, imm_i);
        case 3: RI(OP_sltiu, imm_i);
        case 4: RI(OP_xori, imm_i);
        case 5:
            if (fs3 == 0x0) RI(OP_srli, sh6);
            if (fs3 == 0x5) RI(OP_orc_b, sh6);
            if (fs3 == 0x8) RI(OP_srai, sh6);
            if (fs3 == 0x9) RI(OP_bexti, sh6);
            if (fs3 == 0xc) RI(OP_rori, sh6);
            if (fs3 == 0xd && rs2 == 0x18) RI(OP_rev8, 0);
            if (fs3 == 0xd && rs2 == 0x07) { d.op = OP_ESC_CRYPTO; return d; }
            return d;
        case 6:
            if (rd == 0) {
                if (rs2 == 0 || rs2 == 1 || rs2 == 3) {
                    d.op = rs2 == 0 ? OP_prefetch_i : rs2 == 1 ? OP_prefetch_r : OP_prefetch_w;
                    D_RS1(rs1); d.imm = (int32_t)(fbits(raw, 31, 25) << 5);
                    return d;
                }
                RI(OP_ori_hint, imm_i);
            }
            RI(OP_ori, imm_i);
        default: RI(OP_andi, imm_i);
        }
    case 0x05: d.op = OP_auipc; D_RD(rd); d.imm = imm_u; return d;
    case 0x06:  // OP-IMM-32 :1676-1720
        if (f3 == 0) RI(OP_addiw, imm_i);
        if (f3 == 1) {
            if (fs3 == 0x0) RI(OP_slliw, sh5);
            if (fs3 == 0x1) RI(OP_slli_uw, sh6);
            if (fs3 == 0xc && rs2 == 0) RI(OP_clzw, 0);
            if (fs3 == 0xc && rs2 == 1) RI(OP_ctzw, 0);
            if (fs3 == 0xc && rs2 == 2) RI(OP_cpopw, 0);
        }
        if (f3 == 5) {
            if (fs3 == 0x0) RI(OP_srliw, sh5);
            if (fs3 == 0x8) RI(OP_sraiw, sh5);
            if (fs3 == 0xc) RI(OP_roriw, sh5);
        }
        return d;
    case 0x08: {  // STORE :1722-1739
        if (f3 > 3) return d;
        d.op = (uint8_t)(OP_sb + f3); D_RS1(rs1); D_RS2(rs2); d.imm = imm_s; return d;
    }
    case 0x09: d.op = OP_ESC_FP; return d;
    case 0x0b: d.op = OP_ESC_AMO; return d;
    case 0x0c: {  // OP :2285-2613
        const uint32_t kf5 = fbits(raw, 29, 25), bs = fbits(raw, 31, 30);
        switch (f3) {
        case 0:
            if (kf5 == 0x00 && bs == 0) RR(OP_add);
            if (kf5 == 0x00 && bs == 1) RR(OP_sub);
            if (kf5 == 0x01 && bs == 0) RR(OP_mul);
            if (kf5 == 0x18 || kf5 == 0x1a) { d.op = OP_ESC_CRYPTO; return d; }
            if ((kf5 == 0x19 || kf5 == 0x1b || kf5 == 0x1d) && bs == 0) { d.op = OP_ESC_CRYPTO; return d; }
            if (kf5 == 0x1f && bs <= 1) { d.op = OP_ESC_CRYPTO; return d; }
            return d;
        case 1:
            switch (f7) {
            case 0x00: RR(OP_sll); case 0x01: RR(OP_mulh); case 0x05: RR(OP_clmul); case 0x14: RR(OP_bset);
            case 0x24: RR(OP_bclr); case 0x30: RR(OP_rol); case 0x34: RR(OP_binv);
            }
            return d;
        case 2:
            switch (f7) {
            case 0x00: RR(OP_slt); case 0x01: RR(OP_mulhsu); case 0x05: RR(OP_clmulr); case 0x10: RR(OP_sh1add);
            case 0x14: d.op = OP_ESC_CRYPTO; return d;
            }
            return d;
        case 3:
            switch (f7) { case 0x00: RR(OP_sltu); case 0x01: RR(OP_mulhu); case 0x05: RR(OP_clmulh); }
            return d;
        case 4:
            switch (f7) {
            case 0x00: RR(OP_xor_); case 0x01: RR(OP_div_); case 0x04: RR(OP_pack); case 0x05: RR(OP_min_);
            case 0x10: RR(OP_sh2add); case 0x14: d.op = OP_ESC_CRYPTO; return d; case 0x20: RR(OP_xnor);
            }
            return d;
        case 5:
            switch (f7) {
            case 0x00: RR(OP_srl); case 0x01: RR(OP_divu); case 0x07: RR(OP_czero_eqz); case 0x20: RR(OP_sra);
            case 0x05: RR(OP_minu); case 0x24: RR(OP_bext); case 0x30: RR(OP_ror);
            }
            return d;
        case 6:
            switch (f7) {
            case 0x00: RR(OP_or_); case 0x01: RR(OP_rem); case 0x05: RR(OP_max_); case 0x10: RR(OP_sh3add);
            case 0x20: RR(OP_orn);
            }
            return d;
        default:
            switch (f7) {
            case 0x00: RR(OP_and_); case 0x01: RR(OP_remu); case 0x04: RR(OP_packh); case 0x05: RR(OP_maxu);
            case 0x07: RR(OP_czero_nez); case 0x20: RR(OP_andn);
            }
            return d;
        }
    }
    case 0x0d: d.op = OP_lui; D_RD(rd); d.imm = imm_u; return d;
    case 0x0e:  // OP-32 :2620-2692
        switch (f3) {
        case 0: switch (f7) { case 0x00: RR(OP_addw); case 0x01: RR(OP_mulw); case 0x04: RR(OP_add_uw); case 0x20: RR(OP_subw); } return d;
        case 1: switch (f7) { case 0x00: RR(OP_sllw); case 0x30: RR(OP_rolw); } return d;
        case 2: if (f7 == 0x10) RR(OP_sh1add_uw); return d;
        case 4: switch (f7) { case 0x01: RR(OP_divw); case 0x04: RR(OP_packw); case 0x10: RR(OP_sh2add_uw); } return d;
        case 5: switch (f7) { case 0x00: RR(OP_srlw); case 0x01: RR(OP_divuw); case 0x20: RR(OP_sraw); case 0x30: RR(OP_rorw); } return d;
        case 6: switch (f7) { case 0x01: RR(OP_remw); case 0x10: RR(OP_sh3add_uw); } return d;
        case 7: RR(OP_remuw);   // decoded on FUNCT3 alone (:2687-2689)
        default: return d;
        }
    case 0x10: case 0x11: case 0x12: case 0x13: case 0x14: d.op = OP_ESC_FP; return d;
    case 0x15: d.op = OP_ESC_VEC; return d;
    case 0x18: {  // BRANCH :5891-5936
        if (f3 == 2 || f3 == 3) return d;
        d.op = (uint8_t)(OP_beq + (f3 < 4 ? f3 : f3 - 2)); D_RS1(rs1); D_RS2(rs2); d.imm = imm_b; return d;
    }
    case 0x19: if (f3 == 0) RI(OP_jalr, imm_i); return d;   // :5938-5943
    case 0x1b: d.op = OP_jal; D_RD(rd); d.imm = imm_j; return d;
    case 0x1c:  // SYSTEM :5950-6300
        if (f3 == 0) {
            if (f7 == 0) {
                if (rs2 == 0) d.op = OP_ecall;
                else if (rs2 == 1) d.op = OP_ebreak;
                return d;
            }
            d.op = OP_ESC_SYS; return d;
        }
        if (f3 == 4) { d.op = OP_ESC_HYP; return d; }
        d.op = OP_csr; D_RD(rd);
        if (f3 < 5) D_RS1(rs1);
        d.imm = (int32_t)rs1; d.aux = (uint16_t)fbits(raw, 31, 20);
        return d;
    case 0x1e: d.op = OP_ESC_M5; return d;
    default: return d;
    }
#undef RI
#undef RR
}

// gem5's known-vs-Unknown split for the opcode groups the engine does not
// execute; rows generated from decoder.isa (../gem5_decode_table.h).
struct DecRow { uint32_t mask, match, known; };
#define FI_ROW(m, v, k) {m, v, k},
__constant__ const DecRow kGem5Rows[FI_GEM5_DEC_ROWS] = { FI_GEM5_DEC_TABLE(FI_ROW) };
#undef FI_ROW

// 0 Unknown, 1 known; RVV classes: their action before any vset* (2 no-op,
// 3 no-op of two ticks, 4 IllegalInst, 5 undefined in gem5, 6 needs vector
// state; oracle/rv64se.c VEC_*)
__device__ inline uint32_t gem5_known(uint32_t raw) {
    const uint32_t op5 = (raw >> 2) & 31;
    int first = -1, cnt = 0;
#define FI_IDX(o, f, c) if (op5 == (o)) { first = (f); cnt = (c); }
    FI_GEM5_DEC_INDEX(FI_IDX)
#undef FI_IDX
    if (first < 0) return 1;
    for (int i = first; i < first + cnt; i++)
        if ((raw & kGem5Rows[i].mask) == kGem5Rows[i].match) return kGem5Rows[i].known;
    return 0;
}

// F/D/Zfh arithmetic (decoder.isa:2694-2810, 2811-3440), as in
// oracle/rv64se.c:refine_fp_arith: one op per operation, imm = rm | fmt << 3 |
// sub << 5 | rs3 << 8 (fmt 0 binary16, 1 binary32, 2 binary64).  FP register
// fields plain, integer ones with their flags.  Returns false if the encoding
// is not one of them (fli / fround / froundnx / fcvtmod stay escapes).
__device__ inline int fp_fmt_code(uint32_t f) { return f == 0 ? 1 : f == 1 ? 2 : f == 2 ? 0 : -1; }
__device__ inline bool rv_refine_fp_arith(uint32_t raw, Dec &d) {
    const uint32_t opc = fbits(raw, 6, 2), f3 = fbits(raw, 14, 12), f7 = fbits(raw, 31, 25);
    const uint32_t rd = fbits(raw, 11, 7), rs1 = fbits(raw, 19, 15), rs2 = fbits(raw, 24, 20);
    if (opc >= 0x10 && opc <= 0x13) {
        const int fmt = fp_fmt_code(fbits(raw, 26, 25));
        if (fmt < 0) return false;
        d.op = (uint8_t)(OP_fmadd + (opc - 0x10));
        d.rd = (uint8_t)rd; d.rs1 = (uint8_t)rs1; d.rs2 = (uint8_t)rs2;
        d.imm = (int32_t)(f3 | ((uint32_t)fmt << 3) | (fbits(raw, 31, 27) << 8));
        return true;
    }
    const int fmt = fp_fmt_code(f7 & 3);
    if (opc != 0x14 || fmt < 0) return false;
    int op = -1;
    uint32_t sub = 0;
    switch (f7 >> 2) {
    case 0x00: op = OP_fadd; break;
    case 0x01: op = OP_fsub; break;
    case 0x02: op = OP_fmul; break;
    case 0x03: op = OP_fdiv; break;
    case 0x0b: op = OP_fsqrt; break;
    case 0x05:   // fmin / fmax / fminm / fmaxm (binary16: fminm at 3, fmaxm at 4)
        if (f3 == 0) op = OP_fmin;
        else if (f3 == 1) op = OP_fmax;
        else if (f3 == (fmt == 0 ? 3u : 2u)) { op = OP_fmin; sub = 1; }
        else if (f3 == (fmt == 0 ? 4u : 3u)) { op = OP_fmax; sub = 1; }
        else return false;
        break;
    case 0x14:
        if (f3 == 0) op = OP_fle;
        else if (f3 == 1) op = OP_flt;
        else if (f3 == 2) op = OP_feq;
        else if (f3 == 4) { op = OP_fle; sub = 1; }
        else if (f3 == 5) { op = OP_flt; sub = 1; }
        else return false;
        d.op = (uint8_t)op; D_RD(rd); d.rs1 = (uint8_t)rs1; d.rs2 = (uint8_t)rs2;
        d.imm = (int32_t)(f3 | ((uint32_t)fmt << 3) | (sub << 5));
        return true;
    case 0x18:
        if (rs2 == 8 && fmt == 2) {   // Zfa fcvtmod.w.d
            d.op = OP_fcvtmod; D_RD(rd); d.rs1 = (uint8_t)rs1; d.imm = (int32_t)(f3 | (2u << 3));
            return true;
        }
        if (rs2 > 3) return false;
        d.op = OP_fcvt_f2i; D_RD(rd); d.rs1 = (uint8_t)rs1;
        d.imm = (int32_t)(f3 | ((uint32_t)fmt << 3) | (rs2 << 5));
        return true;
    case 0x1a:
        if (rs2 > 3) return false;
        d.op = OP_fcvt_i2f; d.rd = (uint8_t)rd; D_RS1(rs1);
        d.imm = (int32_t)(f3 | ((uint32_t)fmt << 3) | (rs2 << 5));
        return true;
    case 0x08: {
        if (rs2 == 4 || rs2 == 5) {   // Zfa fround / froundnx
            d.op = OP_fround; d.rd = (uint8_t)rd; d.rs1 = (uint8_t)rs1;
            d.imm = (int32_t)(f3 | ((uint32_t)fmt << 3) | ((uint32_t)(rs2 == 5) << 5));
            return true;
        }
        const int src = fp_fmt_code(rs2);
        if (rs2 > 2 || src < 0 || src == fmt) return false;
        d.op = OP_fcvt_f2f; d.rd = (uint8_t)rd; d.rs1 = (uint8_t)rs1;
        d.imm = (int32_t)(f3 | ((uint32_t)fmt << 3) | ((uint32_t)src << 5));
        return true;
    }
    default: return false;
    }
    d.op = (uint8_t)op; d.rd = (uint8_t)rd; d.rs1 = (uint8_t)rs1; d.rs2 = (uint8_t)rs2;
    d.imm = (int32_t)(f3 | ((uint32_t)fmt << 3) | (sub << 5));
    return true;
}

// The executed members of the LOAD-FP / STORE-FP / OP-FP / AMO groups among
// the encodings gem5 knows (decoder.isa:567-591, :1741-1763, :2067-2283,
// :2896-2942, :3500-3548, :3593-3598, :3648-3652).  FP register indices sit in
// rd / rs1 / rs2 WITHOUT the integer-register flags (liveness and the replica
// watch only see integer operands).
__device__ inline void rv_refine_fp_amo(uint32_t raw, Dec &d) {
    const uint32_t opc = fbits(raw, 6, 2), f3 = fbits(raw, 14, 12), f7 = fbits(raw, 31, 25);
    const uint32_t rd = fbits(raw, 11, 7), rs1 = fbits(raw, 19, 15), rs2 = fbits(raw, 24, 20);
    if (opc == 0x01 && f3 >= 1 && f3 <= 3) {
        d.op = (uint8_t)(OP_flh + f3 - 1); d.rd = (uint8_t)rd; D_RS1(rs1); d.imm = fsext(fbits(raw, 31, 20), 12);
        return;
    }
    if (opc == 0x09 && f3 >= 1 && f3 <= 3) {
        d.op = (uint8_t)(OP_fsh + f3 - 1); d.rs2 = (uint8_t)rs2; D_RS1(rs1);
        d.imm = fsext((fbits(raw, 31, 25) << 5) | fbits(raw, 11, 7), 12);
        return;
    }
    if (opc == 0x0b && (f3 == 2 || f3 == 3)) {
        int o;
        switch (fbits(raw, 31, 27)) {
        case 0x00: o = OP_amoadd_w; break;  case 0x01: o = OP_amoswap_w; break; case 0x04: o = OP_amoxor_w; break;
        case 0x08: o = OP_amoor_w; break;   case 0x0c: o = OP_amoand_w; break;  case 0x10: o = OP_amomin_w; break;
        case 0x14: o = OP_amomax_w; break;  case 0x18: o = OP_amominu_w; break; case 0x1c: o = OP_amomaxu_w; break;
        case 0x02: case 0x03:   // lr / sc (decoder.isa:2069-2075, 2175-2181)
            d.op = (uint8_t)(fbits(raw, 31, 27) == 0x02 ? (f3 == 2 ? OP_lr_w : OP_lr_d) : (f3 == 2 ? OP_sc_w : OP_sc_d));
            D_RD(rd); D_RS1(rs1);
            if (fbits(raw, 31, 27) == 0x03) D_RS2(rs2);
            d.imm = 0;
            return;
        default: return;
        }
        d.op = (uint8_t)(f3 == 2 ? o : o + (OP_amoadd_d - OP_amoadd_w));
        D_RD(rd); D_RS1(rs1); D_RS2(rs2); d.imm = 0;
        return;
    }
    if (rv_refine_fp_arith(raw, d)) return;
    if (opc != 0x14) return;
    if ((f7 == 0x10 || f7 == 0x11 || f7 == 0x12) && f3 <= 2) {
        d.op = (uint8_t)((f7 == 0x10 ? OP_fsgnj_s : f7 == 0x11 ? OP_fsgnj_d : OP_fsgnj_h) + f3);
        d.rd = (uint8_t)rd; d.rs1 = (uint8_t)rs1; d.rs2 = (uint8_t)rs2;
        return;
    }
    if (f7 == 0x70 && f3 <= 1) { d.op = f3 ? OP_fclass_s : OP_fmv_x_w; D_RD(rd); d.rs1 = (uint8_t)rs1; return; }
    if (f7 == 0x71 && f3 == 1) { d.op = OP_fclass_d; D_RD(rd); d.rs1 = (uint8_t)rs1; return; }
    if (f7 == 0x71 && f3 == 0 && rs2 == 0) { d.op = OP_fmv_x_d; D_RD(rd); d.rs1 = (uint8_t)rs1; return; }
    if (f7 == 0x72 && f3 <= 1) { d.op = f3 ? OP_fclass_h : OP_fmv_x_h; D_RD(rd); d.rs1 = (uint8_t)rs1; return; }
    if (f7 == 0x78 && f3 == 0 && rs2 == 0) { d.op = OP_fmv_w_x; d.rd = (uint8_t)rd; D_RS1(rs1); return; }
    if ((f7 == 0x78 && f3 == 0 && rs2 == 1) || ((f7 == 0x79 || f7 == 0x7a) && rs2 == 1)) {   // Zfa fli: rs1 = index
        d.op = OP_fli; d.rd = (uint8_t)rd;
        d.imm = (int32_t)((rs1 << 8) | ((uint32_t)(f7 == 0x78 ? 1 : f7 == 0x79 ? 2 : 0) << 3));
        return;
    }
    if (f7 == 0x79 && rs2 == 0) { d.op = OP_fmv_d_x; d.rd = (uint8_t)rd; D_RS1(rs1); return; }
    if (f7 == 0x7a && rs2 == 0) { d.op = OP_fmv_h_x; d.rd = (uint8_t)rd; D_RS1(rs1); return; }
}

// The gem5-known members of the privileged SYSTEM, hypervisor load/store,
// cache-block, M5 pseudo-op and scalar-crypto groups (oracle/rv64se.c:
// refine_misc, which cites the reference): priv imm 0 = IllegalInst in PRV_U,
// 1 = warn-only no-op; cbo imm = FUNCT12; m5op imm = M5FUNC, rd = a0;
// crypto imm = function | RNUM / BS << 8 (fi_crypto.h).
__device__ inline void rv_refine_misc(uint32_t raw, Dec &d) {
    const uint32_t f3 = fbits(raw, 14, 12), f7 = fbits(raw, 31, 25);
    const uint32_t rd = fbits(raw, 11, 7), rs1 = fbits(raw, 19, 15), rs2 = fbits(raw, 24, 20);
    switch (d.op) {
    case OP_ESC_SYS:
        d.op = OP_priv;
        d.imm = (f7 == 0x0b || f7 == 0x0c || f7 == 0x13 || f7 == 0x33) ? 1 : 0;
        if (f7 == 0x09 || f7 == 0x11 || f7 == 0x31) { D_RS1(rs1); D_RS2(rs2); }
        return;
    case OP_ESC_HYP:
        d.op = OP_priv; d.imm = 0; D_RS1(rs1);
        if (f7 & 1) D_RS2(rs2);
        return;
    case OP_ESC_CBO: d.op = OP_cbo; D_RS1(rs1); d.imm = (int32_t)fbits(raw, 31, 20); return;
    case OP_ESC_M5: d.op = OP_m5op; D_RD(10); d.imm = (int32_t)f7; return;
    case OP_ESC_CRYPTO: {
        const uint32_t opc = fbits(raw, 6, 2), kf5 = fbits(raw, 29, 25), bs = fbits(raw, 31, 30);
        int fn = -1;
        if (opc == 0x04 && f3 == 1) {
            if (fbits(raw, 31, 27) == 0x02) fn = (int)rs2;
            else fn = fbits(raw, 24, 24) ? (int)(11 | (fbits(raw, 23, 20) << 8)) : 10;
        } else if (opc == 0x04) {
            fn = 12;
        } else if (opc == 0x0c && f3 == 0) {
            if (kf5 == 0x18) fn = (int)(13 | (bs << 8));
            else if (kf5 == 0x1a) fn = (int)(14 | (bs << 8));
            else if (kf5 == 0x19) fn = 15;
            else if (kf5 == 0x1b) fn = 16;
            else if (kf5 == 0x1d) fn = 17;
            else if (kf5 == 0x1f) fn = bs ? 19 : 18;
        } else if (opc == 0x0c) {
            fn = f3 == 2 ? 20 : 21;
        }
        if (fn < 0) return;
        d.op = OP_crypto; d.imm = fn; D_RD(rd); D_RS1(rs1);
        if ((fn & 0xFF) >= 13) D_RS2(rs2);
        return;
    }
    default: return;
    }
}

__device__ inline Dec rv_decode(uint32_t raw) {
    Dec d = rv_decode_tree(raw);
    if ((raw & 3) == 3 && (d.op == OP_ESC_FP || d.op == OP_ESC_VEC || d.op == OP_ESC_AMO ||
                           d.op == OP_ESC_SYS || d.op == OP_ESC_HYP)) {
        const uint32_t k = gem5_known(raw);
        if (!k) d.op = OP_UNKNOWN;
        else if (k >= 2) { d.op = OP_vec; d.imm = (int32_t)k; }
    }
    if ((raw & 3) == 3 && (d.op == OP_ESC_FP || d.op == OP_ESC_AMO)) rv_refine_fp_amo(raw, d);
    if ((raw & 3) == 3) rv_refine_misc(raw, d);
    // vsetvli / vsetvl / vsetivli out of the vector-state class (oracle/rv64se.c
    // decode, decoder.isa:5838-5886): imm = the requested vtype's immediate |
    // form << 16 (0 vsetvli, 1 vsetvl: vtype from Rs2, 2 vsetivli: its uimm << 20)
    if (d.op == OP_vec && d.imm == 6 && (raw & 0x7F) == 0x57 && fbits(raw, 14, 12) == 7) {
        const uint32_t form = fbits(raw, 31, 31) ? (fbits(raw, 30, 30) ? 2u : 1u) : 0u;
        d.op = OP_vset;
        D_RD(fbits(raw, 11, 7));
        if (form != 2) D_RS1(fbits(raw, 19, 15));
        if (form == 1) D_RS2(fbits(raw, 24, 20));
        d.imm = (int32_t)((form == 0 ? fbits(raw, 30, 20) : form == 2 ? fbits(raw, 29, 20) : 0u) | (form << 16) |
                          (form == 2 ? fbits(raw, 19, 15) << 20 : 0u));
    }
    return d;
}
#undef D_RD
#undef D_RS1
#undef D_RS2

// ---------------------------------------------------------------- micro-ops
// The fast path executes a normalised micro-op instead of the 170 gem5 ops:
// aux = kind | U_* flags | log2(size) << 12.  Every op whose semantics are not a
// plain ALU/load/store/branch/jump (M-extension beyond mul, bitmanip, system,
// unknown, escapes, and the encodings that raise IllegalInst at execute) is
// K_SLOW and goes through the full per-op switch of the general path.
enum Kind : uint8_t {
    K_SLOW = 0, K_ADD, K_SUB, K_AND, K_OR, K_XOR, K_SLT, K_SLTU, K_SLL, K_SRL, K_SRA, K_MUL,
    K_LOAD, K_STORE, K_BEQ, K_BNE, K_BLT, K_BGE, K_BLTU, K_BGEU, K_JAL, K_JALR, K_NOP,
    K_MULH, K_MULHU, K_MULHSU, K_DIV, K_DIVU, K_REM, K_REMU
};
constexpr uint16_t U_BIMM = 1u << 8, U_APC = 1u << 9, U_W32 = 1u << 10, U_SEXT = 1u << 11;

__host__ __device__ inline uint16_t uop_of(Dec &d) {
    auto ls = [](uint8_t k, int lg, bool sx) -> uint16_t {
        return (uint16_t)(k | (lg << 12) | (sx ? U_SEXT : 0));
    };
    switch (d.op) {
    case OP_c_addi4spn: return d.imm ? (uint16_t)(K_ADD | U_BIMM) : K_SLOW;
    case OP_c_lwsp: if (d.rd == 0) return K_SLOW; return ls(K_LOAD, 2, true);
    case OP_c_lw: case OP_lw: return ls(K_LOAD, 2, true);
    case OP_c_ldsp: if (d.rd == 0) return K_SLOW; return ls(K_LOAD, 3, false);
    case OP_c_ld: case OP_ld: return ls(K_LOAD, 3, false);
    case OP_c_lbu: case OP_lbu: return ls(K_LOAD, 0, false);
    case OP_c_lhu: case OP_lhu: return ls(K_LOAD, 1, false);
    case OP_c_lh: case OP_lh: return ls(K_LOAD, 1, true);
    case OP_lb: return ls(K_LOAD, 0, true);
    case OP_lwu: return ls(K_LOAD, 2, false);
    case OP_c_sb: case OP_sb: return ls(K_STORE, 0, false);
    case OP_c_sh: case OP_sh: return ls(K_STORE, 1, false);
    case OP_c_sw: case OP_sw: case OP_c_swsp: return ls(K_STORE, 2, false);
    case OP_c_sd: case OP_sd: case OP_c_sdsp: return ls(K_STORE, 3, false);
    case OP_c_addi: case OP_addi: case OP_c_li: case OP_lui: return K_ADD | U_BIMM;
    case OP_c_addiw: if (d.rd == 0) return K_SLOW; return K_ADD | U_BIMM | U_W32;
    case OP_addiw: return K_ADD | U_BIMM | U_W32;
    case OP_c_addi16sp: case OP_c_lui: return d.imm ? (uint16_t)(K_ADD | U_BIMM) : K_SLOW;
    case OP_c_srli: case OP_srli: return K_SRL | U_BIMM;
    case OP_c_srai: case OP_srai: return K_SRA | U_BIMM;
    case OP_c_slli: case OP_slli: return K_SLL | U_BIMM;
    case OP_c_andi: case OP_andi: return K_AND | U_BIMM;
    case OP_xori: return K_XOR | U_BIMM;
    case OP_ori: case OP_ori_hint: return K_OR | U_BIMM;
    case OP_slti: return K_SLT | U_BIMM;
    case OP_sltiu: return K_SLTU | U_BIMM;
    case OP_c_sub: case OP_sub: return K_SUB;
    case OP_c_xor: case OP_xor_: return K_XOR;
    case OP_c_or: case OP_or_: return K_OR;
    case OP_c_and: case OP_and_: return K_AND;
    case OP_c_subw: case OP_subw: return K_SUB | U_W32;
    case OP_c_addw: case OP_addw: return K_ADD | U_W32;
    case OP_c_mul: case OP_mul: return K_MUL;
    case OP_mulh: return K_MULH;
    case OP_mulhu: return K_MULHU;
    case OP_mulhsu: return K_MULHSU;
    case OP_div_: return K_DIV;
    case OP_divu: return K_DIVU;
    case OP_rem: return K_REM;
    case OP_remu: return K_REMU;
    case OP_divw: return K_DIV | U_W32;
    case OP_divuw: return K_DIVU | U_W32;
    case OP_remw: return K_REM | U_W32;
    case OP_remuw: return K_REMU | U_W32;
    case OP_mulw: return K_MUL | U_W32;
    case OP_c_zext_b: d.imm = 0xFF; return K_AND | U_BIMM;
    case OP_c_zext_h: d.imm = 0xFFFF; return K_AND | U_BIMM;
    case OP_c_not: d.imm = -1; return K_XOR | U_BIMM;
    case OP_c_j: case OP_jal: return K_JAL;
    case OP_c_beqz: case OP_beq: return K_BEQ;
    case OP_c_bnez: case OP_bne: return K_BNE;
    case OP_blt: return K_BLT;
    case OP_bge: return K_BGE;
    case OP_bltu: return K_BLTU;
    case OP_bgeu: return K_BGEU;
    case OP_c_jr: return d.rs1 ? (uint16_t)K_JALR : K_SLOW;
    case OP_c_jalr: case OP_jalr: return K_JALR;
    case OP_c_mv: case OP_c_add: case OP_add: return K_ADD;
    case OP_sll: return K_SLL;
    case OP_srl: return K_SRL;
    case OP_sra: return K_SRA;
    case OP_slt: return K_SLT;
    case OP_sltu: return K_SLTU;
    case OP_sllw: return K_SLL | U_W32;
    case OP_srlw: return K_SRL | U_W32;
    case OP_sraw: return K_SRA | U_W32;
    case OP_slliw: return K_SLL | U_BIMM | U_W32;
    case OP_srliw: return K_SRL | U_BIMM | U_W32;
    case OP_sraiw: return K_SRA | U_BIMM | U_W32;
    case OP_auipc: return K_ADD | U_BIMM | U_APC;
    case OP_fence: case OP_fence_i: case OP_prefetch_i: case OP_prefetch_r: case OP_prefetch_w: return K_NOP;
    default: return K_SLOW;
    }
}

}  // namespace fi
