"""Known-answer vectors for the oracle's M-extension, shift, bit-manipulation and Zicond semantics (CPU).

Expected values are computed here straight from the reference's definitions:
- div/divu/rem/remu edge cases: `src/arch/riscv/utility.hh:191-231`
  (x/0 -> -1 or all-ones, rem x/0 -> x, INT_MIN/-1 -> INT_MIN with rem 0);
- mulh/mulhsu/mulhu through a double-width product: `utility.hh:171-189`;
- the W forms: `src/arch/riscv/isa/decoder.isa:2627-2689` (operands
  truncated to 32 bits, result sign-extended from 32 bits, also for the
  unsigned divuw/remuw);
- shift amounts: 6 bits for sll/srl/sra (`decoder.isa:2404-2551`), 5 bits
  for sllw/srlw/sraw (`:2638-2672`).
Each instruction runs through `or_probe` (one instruction in a scratch
machine), the same entry the GPU parity tests use.
"""
import itertools
import json
import os
import random
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools", "rvasm"))
from rvasm import enc_i, enc_r  # noqa: E402

M64 = (1 << 64) - 1
M32 = (1 << 32) - 1


def s64(v):
    v &= M64
    return v - (1 << 64) if v >> 63 else v


def s32(v):
    v &= M32
    return v - (1 << 32) if v >> 31 else v


def tdiv(a, b):   # C++ truncating division
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def div(a, b, bits):
    lo = -(1 << (bits - 1))
    if b == 0:
        return -1
    if a == lo and b == -1:
        return lo
    return tdiv(a, b)


def rem(a, b, bits):
    lo = -(1 << (bits - 1))
    if b == 0:
        return a
    if a == lo and b == -1:
        return 0
    return a - tdiv(a, b) * b


def divu(a, b, bits):
    return (1 << bits) - 1 if b == 0 else a // b


def remu(a, b):
    return a if b == 0 else a % b


# (name, opcode, funct3, funct7, model(a, b) -> value as a Python int)
OPS = [
    ("mul", 0x33, 0, 1, lambda a, b: a * b),
    ("mulh", 0x33, 1, 1, lambda a, b: (s64(a) * s64(b)) >> 64),
    ("mulhsu", 0x33, 2, 1, lambda a, b: (s64(a) * b) >> 64),
    ("mulhu", 0x33, 3, 1, lambda a, b: (a * b) >> 64),
    ("div", 0x33, 4, 1, lambda a, b: div(s64(a), s64(b), 64)),
    ("divu", 0x33, 5, 1, lambda a, b: divu(a, b, 64)),
    ("rem", 0x33, 6, 1, lambda a, b: rem(s64(a), s64(b), 64)),
    ("remu", 0x33, 7, 1, lambda a, b: remu(a, b)),
    ("mulw", 0x3B, 0, 1, lambda a, b: s32(s32(a) * s32(b))),
    ("divw", 0x3B, 4, 1, lambda a, b: s32(div(s32(a), s32(b), 32))),
    ("divuw", 0x3B, 5, 1, lambda a, b: s32(divu(a & M32, b & M32, 32))),
    ("remw", 0x3B, 6, 1, lambda a, b: s32(rem(s32(a), s32(b), 32))),
    ("remuw", 0x3B, 7, 1, lambda a, b: s32(remu(a & M32, b & M32))),
    ("sll", 0x33, 1, 0, lambda a, b: a << (b & 63)),
    ("srl", 0x33, 5, 0, lambda a, b: a >> (b & 63)),
    ("sra", 0x33, 5, 0x20, lambda a, b: s64(a) >> (b & 63)),
    ("sllw", 0x3B, 1, 0, lambda a, b: s32(a << (b & 31))),
    ("srlw", 0x3B, 5, 0, lambda a, b: s32((a & M32) >> (b & 31))),
    ("sraw", 0x3B, 5, 0x20, lambda a, b: s32(a) >> (b & 31)),
]

EDGE = [0, 1, 2, 3, 7, M64, M64 - 1, 1 << 63, (1 << 63) - 1, 1 << 31, (1 << 31) - 1, M32, 1 << 32,
        0xFFFFFFFF80000000, 0x8000000000000001, 0x123456789ABCDEF0, 63, 64, 31, 32]


def vectors():
    rng = random.Random(0x5EED)
    pairs = list(itertools.product(EDGE, EDGE))
    pairs += [(rng.getrandbits(64), rng.getrandbits(64)) for _ in range(200)]
    pairs += [(rng.getrandbits(64), rng.choice([0, 1, M64, rng.getrandbits(8)])) for _ in range(100)]
    return pairs


@pytest.mark.parametrize("name,opc,f3,f7,model", OPS, ids=[o[0] for o in OPS])
def test_m_extension_and_shifts(oracle_mod, name, opc, f3, f7, model):
    inst = enc_r(opc, f3, f7, 10, 11, 12)   # name a0, a1, a2
    bad = []
    for a, b in vectors():
        regs = [0] * 32
        regs[11], regs[12] = a, b
        p = oracle_mod.probe(inst, 0x10000, regs)
        want = model(a, b) & M64
        assert p.fault == 0 and p.rd == 10 and p.len == 4 and p.npc == 0x10004
        if p.rd_value != want:
            bad.append((hex(a), hex(b), hex(p.rd_value), hex(want)))
    assert not bad, f"{name}: {len(bad)} mismatches, first {bad[:3]}"


def test_x0_destination_is_dropped(oracle_mod):
    """Writes to x0 are discarded (`regs/int.hh:65-79`, x0 = InvalidRegClass)."""
    inst = enc_r(0x33, 0, 1, 0, 11, 12)      # mul x0, a1, a2
    regs = [0] * 32
    regs[11], regs[12] = 3, 5
    p = oracle_mod.probe(inst, 0x10000, regs)
    assert p.fault == 0 and p.rd_value == 0


def clmul128(a, b):
    r = 0
    for i in range(64):
        if (b >> i) & 1:
            r ^= a << i
    return r


# Zba/Zbb/Zbc/Zbs/Zicond register-register forms (OP, opcode 0x33):
# `decoder.isa:2414-2612`.  XLEN = 64, so rvSext/rvZext are identities.
BITMANIP = [
    ("clmul", 1, 0x05, lambda a, b: clmul128(a, b)),
    ("clmulr", 2, 0x05, lambda a, b: clmul128(a, b) >> 63),
    ("clmulh", 3, 0x05, lambda a, b: clmul128(a, b) >> 64),
    ("bset", 1, 0x14, lambda a, b: a | (1 << (b & 63))),
    ("bclr", 1, 0x24, lambda a, b: a & ~(1 << (b & 63))),
    ("binv", 1, 0x34, lambda a, b: a ^ (1 << (b & 63))),
    ("bext", 5, 0x24, lambda a, b: (a >> (b & 63)) & 1),
    ("rol", 1, 0x30, lambda a, b: (a << (b & 63)) | (a >> ((64 - (b & 63)) & 63))),
    ("ror", 5, 0x30, lambda a, b: (a >> (b & 63)) | (a << ((64 - (b & 63)) & 63))),
    ("sh1add", 2, 0x10, lambda a, b: (a << 1) + b),
    ("sh2add", 4, 0x10, lambda a, b: (a << 2) + b),
    ("sh3add", 6, 0x10, lambda a, b: (a << 3) + b),
    ("xnor", 4, 0x20, lambda a, b: ~(a ^ b)),
    ("orn", 6, 0x20, lambda a, b: a | ~b),
    ("andn", 7, 0x20, lambda a, b: a & ~b),
    ("min", 4, 0x05, lambda a, b: min(s64(a), s64(b))),
    ("minu", 5, 0x05, lambda a, b: min(a, b)),
    ("max", 6, 0x05, lambda a, b: max(s64(a), s64(b))),
    ("maxu", 7, 0x05, lambda a, b: max(a, b)),
    ("czero_eqz", 5, 0x07, lambda a, b: 0 if b == 0 else a),
    ("czero_nez", 7, 0x07, lambda a, b: 0 if b != 0 else a),
]


@pytest.mark.parametrize("name,f3,f7,model", BITMANIP, ids=[o[0] for o in BITMANIP])
def test_bitmanip_and_zicond(oracle_mod, name, f3, f7, model):
    inst = enc_r(0x33, f3, f7, 10, 11, 12)
    assert oracle_mod.mnemonic(inst).replace(".", "_") == name
    bad = []
    for a, b in vectors():
        regs = [0] * 32
        regs[11], regs[12] = a, b
        p = oracle_mod.probe(inst, 0x10000, regs)
        want = model(a, b) & M64
        assert p.fault == 0 and p.rd == 10
        if p.rd_value != want:
            bad.append((hex(a), hex(b), hex(p.rd_value), hex(want)))
    assert not bad, f"{name}: {len(bad)} mismatches, first {bad[:3]}"


def rot(v, n, w):
    m = (1 << w) - 1
    v &= m
    n %= w
    return ((v >> n) | (v << (w - n))) & m


def sx(v, bits):
    v &= (1 << bits) - 1
    return v - (1 << bits) if v >> (bits - 1) else v


def orc_b(a):
    return sum(0xFF << (8 * i) for i in range(8) if (a >> (8 * i)) & 0xFF)


# Immediate, unary and W forms, as (name, instruction word, model(a, b)):
# `decoder.isa:1490-1716` (OP-IMM / OP-IMM-32) and `:2630-2686` (OP-32).
# rd = a0, rs1 = a1, rs2 = a2 where the format has one.
UNARY = [
    ("clz", enc_i(0x13, 1, 10, 11, 0x600), lambda a, b: 64 - a.bit_length()),
    ("ctz", enc_i(0x13, 1, 10, 11, 0x601), lambda a, b: 64 if a == 0 else (a & -a).bit_length() - 1),
    ("cpop", enc_i(0x13, 1, 10, 11, 0x602), lambda a, b: bin(a).count("1")),
    ("sext_b", enc_i(0x13, 1, 10, 11, 0x604), lambda a, b: sx(a, 8)),
    ("sext_h", enc_i(0x13, 1, 10, 11, 0x605), lambda a, b: sx(a, 16)),
    # zext.h is packw with rs2 = x0 on RV64 (gem5 decodes it as packw, `decoder.isa:2656`)
    ("packw", enc_r(0x3B, 4, 0x04, 10, 11, 12), lambda a, b: sx(((b & 0xFFFF) << 16) | (a & 0xFFFF), 32)),
    ("rev8", enc_i(0x13, 5, 10, 11, 0x6B8), lambda a, b: int.from_bytes(a.to_bytes(8, "little"), "big")),
    ("orc_b", enc_i(0x13, 5, 10, 11, 0x287), lambda a, b: orc_b(a)),
    ("rori", enc_i(0x13, 5, 10, 11, 0x600 | 13), lambda a, b: rot(a, 13, 64)),
    ("bexti", enc_i(0x13, 5, 10, 11, 0x480 | 40), lambda a, b: (a >> 40) & 1),
    ("bseti", enc_i(0x13, 1, 10, 11, 0x280 | 63), lambda a, b: a | (1 << 63)),
    ("bclri", enc_i(0x13, 1, 10, 11, 0x480 | 5), lambda a, b: a & ~(1 << 5)),
    ("binvi", enc_i(0x13, 1, 10, 11, 0x680 | 33), lambda a, b: a ^ (1 << 33)),
    ("addiw", enc_i(0x1B, 0, 10, 11, -1), lambda a, b: sx(a - 1, 32)),
    ("slli_uw", enc_i(0x1B, 1, 10, 11, 0x080 | 33), lambda a, b: (a & M32) << 33),
    ("clzw", enc_i(0x1B, 1, 10, 11, 0x600), lambda a, b: 32 - (a & M32).bit_length()),
    ("ctzw", enc_i(0x1B, 1, 10, 11, 0x601),
     lambda a, b: 32 if a & M32 == 0 else ((a & M32) & -(a & M32)).bit_length() - 1),
    ("cpopw", enc_i(0x1B, 1, 10, 11, 0x602), lambda a, b: bin(a & M32).count("1")),
    ("roriw", enc_i(0x1B, 5, 10, 11, 0x600 | 7), lambda a, b: sx(rot(a, 7, 32), 32)),
    ("addw", enc_r(0x3B, 0, 0x00, 10, 11, 12), lambda a, b: sx(a + b, 32)),
    ("subw", enc_r(0x3B, 0, 0x20, 10, 11, 12), lambda a, b: sx(a - b, 32)),
    ("add_uw", enc_r(0x3B, 0, 0x04, 10, 11, 12), lambda a, b: (a & M32) + b),
    ("sh1add_uw", enc_r(0x3B, 2, 0x10, 10, 11, 12), lambda a, b: ((a & M32) << 1) + b),
    ("sh2add_uw", enc_r(0x3B, 4, 0x10, 10, 11, 12), lambda a, b: ((a & M32) << 2) + b),
    ("sh3add_uw", enc_r(0x3B, 6, 0x10, 10, 11, 12), lambda a, b: ((a & M32) << 3) + b),
    ("rolw", enc_r(0x3B, 1, 0x30, 10, 11, 12), lambda a, b: sx(rot(a, 32 - (b & 31), 32), 32)),
    ("rorw", enc_r(0x3B, 5, 0x30, 10, 11, 12), lambda a, b: sx(rot(a, b & 31, 32), 32)),
]


@pytest.mark.parametrize("name,word,model", UNARY, ids=[o[0] for o in UNARY])
def test_immediate_unary_and_w_forms(oracle_mod, name, word, model):
    assert oracle_mod.mnemonic(word).replace(".", "_") == name
    bad = []
    for a, b in vectors():
        regs = [0] * 32
        regs[11], regs[12] = a, b
        p = oracle_mod.probe(word, 0x10000, regs)
        want = model(a, b) & M64
        assert p.fault == 0 and p.rd == 10
        if p.rd_value != want:
            bad.append((hex(a), hex(b), hex(p.rd_value), hex(want)))
    assert not bad, f"{name}: {len(bad)} mismatches, first {bad[:3]}"


# ---- the same vectors as a guest program (device known-answer workload) ----
# Every R-type op above runs on every (a, b) pair inside one RV64 process that
# writes the results to stdout, 8 bytes each, pair-major.  The GPU test checks
# the device's golden stdout against the models and runs no-fault trials
# through the pre-decoded and translated paths (tests/test_gpu_parity.py).
ALL_OPS = [(n, enc_r(opc, f3, f7, 10, 11, 12), m) for (n, opc, f3, f7, m) in OPS] + \
          [(n, enc_r(0x33, f3, f7, 10, 11, 12), m) for (n, f3, f7, m) in BITMANIP] + UNARY


def program_pairs():
    rng = random.Random(0x15A)
    edge = EDGE[:14]
    pairs = list(itertools.product(edge, edge))
    pairs += [(rng.getrandbits(64), rng.getrandbits(64)) for _ in range(40)]
    pairs += [(rng.getrandbits(64), rng.choice([0, 1, M64, rng.getrandbits(8)])) for _ in range(20)]
    return pairs


def program_source() -> str:
    pairs = program_pairs()
    body = []
    for k, (_, word, _m) in enumerate(ALL_OPS):
        body.append(f"    .word {word:#010x}")
        body.append(f"    sd    a0, {8 * k}(s2)")
    n_out = 8 * len(ALL_OPS) * len(pairs)
    data = "\n".join(f"    .dword {a:#x}, {b:#x}" for a, b in pairs)
    return f"""    .text
_start:
    la    s0, vec
    li    s1, {len(pairs)}
    la    s2, out
loop:
    ld    a1, 0(s0)
    ld    a2, 8(s0)
{chr(10).join(body)}
    addi  s0, s0, 16
    addi  s2, s2, {8 * len(ALL_OPS)}
    addi  s1, s1, -1
    bnez  s1, loop
    li    a0, 1
    la    a1, out
    li    a2, {n_out}
    li    a7, 64
    ecall
    li    a0, 0
    li    a7, 94
    ecall
    .data
    .balign 8
vec:
{data}
    .bss
    .balign 8
out:
    .zero {n_out}
"""


def program_elf() -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(program_source())


def program_expected() -> bytes:
    out = bytearray()
    for a, b in program_pairs():
        for (_, _, m) in ALL_OPS:
            out += ((m(a, b)) & M64).to_bytes(8, "little")
    return bytes(out)


def test_alu_program_on_oracle(oracle_mod):
    """The guest program's stdout on the oracle equals the models."""
    o = oracle_mod.Oracle(program_elf(), "alu")
    g = o.run_golden()
    assert g.exit_code == 0
    assert o.golden_stdout() == program_expected()


# ---- misaligned and line/page-crossing loads and stores (guest program) ----
# SE mode has no alignment check and no read-only pages; an access is split at
# 64-byte lines (`atomic.cc:331-545`, `tlb.cc:573-604`), little-endian.  Each
# case stores one value with sb/sh/sw/sd at buf+off, then loads it back with
# all seven load forms; the 8-byte results go to stdout.  buf is two pages.
MEM_OFFS = [0, 1, 2, 3, 5, 7, 30, 57, 59, 61, 62, 63, 4033, 4039, 4089, 4091, 4093, 4094, 4095]
STORES = [("sb", 1), ("sh", 2), ("sw", 4), ("sd", 8)]
LOADS = [("lb", 1, True), ("lbu", 1, False), ("lh", 2, True), ("lhu", 2, False),
         ("lw", 4, True), ("lwu", 4, False), ("ld", 8, False)]


def mem_cases():
    rng = random.Random(0x3E3)
    return [(off, st, rng.getrandbits(64) | (1 << 63 if k % 2 else 0))
            for k, (st, off) in enumerate(itertools.product(STORES, MEM_OFFS))]


def mem_program_source() -> str:
    # one loop per store width over MEM_OFFS (short code: the translated
    # blocks stay small)
    cases = mem_cases()
    lines = []
    for st, _ in STORES:
        lines += [f"    li    s1, {len(MEM_OFFS)}", f"loop_{st}:", "    ld    t2, 0(s3)", "    addi  s3, s3, 8",
                  "    ld    t0, 0(s4)", "    addi  s4, s4, 8", "    add   t1, s0, t0", f"    {st:<5} t2, 0(t1)"]
        for k, (ld, _, _) in enumerate(LOADS):
            lines += [f"    {ld:<5} a0, 0(t1)", f"    sd    a0, {8 * k}(s2)"]
        lines += [f"    addi  s2, s2, {8 * len(LOADS)}", "    addi  s1, s1, -1", f"    bnez  s1, loop_{st}"]
    n_out = 8 * len(LOADS) * len(cases)
    vals = "\n".join(f"    .dword {v:#x}" for _, _, v in cases)
    offs = "\n".join(f"    .dword {o}" for o, _, _ in cases)
    return f"""    .text
_start:
    la    s0, buf
    la    s2, out
    la    s3, vals
    la    s4, offs
{chr(10).join(lines)}
    li    a0, 1
    la    a1, out
    li    a2, {n_out}
    li    a7, 64
    ecall
    li    a0, 0
    li    a7, 94
    ecall
    .data
    .balign 8
vals:
{vals}
offs:
{offs}
    .bss
    .balign 4096
buf:
    .zero 8192
out:
    .zero {n_out}
"""


def mem_program_elf() -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(mem_program_source())


def mem_program_expected() -> bytes:
    mem = bytearray(8192 + 8)
    out = bytearray()
    for off, (_, w), v in mem_cases():
        mem[off:off + w] = (v & ((1 << (8 * w)) - 1)).to_bytes(w, "little")
        for _, lw, signed in LOADS:
            x = int.from_bytes(mem[off:off + lw], "little")
            if signed:
                x = sx(x, 8 * lw)
            out += (x & M64).to_bytes(8, "little")
    return bytes(out)


def test_mem_program_on_oracle(oracle_mod):
    """Misaligned, line-crossing and page-crossing accesses on the oracle."""
    o = oracle_mod.Oracle(mem_program_elf(), "mem")
    g = o.run_golden()
    assert g.exit_code == 0
    assert o.golden_stdout() == mem_program_expected()


# ---- compares and branches (guest program + single-instruction probes) ----
# slt/sltu/slti/sltiu (`decoder.isa:1555-1560,2476-2500`) and the six
# conditional branches (`:5891-5936`): a branch case stores 0 if taken, 1 if
# not.  jalr clears bit 0 of the target (`:5938-5943`).
CMP_OPS = [
    ("slt", enc_r(0x33, 2, 0, 10, 11, 12), lambda a, b: int(s64(a) < s64(b))),
    ("sltu", enc_r(0x33, 3, 0, 10, 11, 12), lambda a, b: int(a < b)),
    ("slti", enc_i(0x13, 2, 10, 11, -1), lambda a, b: int(s64(a) < -1)),
    ("sltiu", enc_i(0x13, 3, 10, 11, -1), lambda a, b: int(a < M64)),
    ("slti", enc_i(0x13, 2, 10, 11, 5), lambda a, b: int(s64(a) < 5)),
    ("sltiu", enc_i(0x13, 3, 10, 11, 5), lambda a, b: int(a < 5)),
]
BRANCHES = [
    ("beq", lambda a, b: a == b), ("bne", lambda a, b: a != b),
    ("blt", lambda a, b: s64(a) < s64(b)), ("bge", lambda a, b: s64(a) >= s64(b)),
    ("bltu", lambda a, b: a < b), ("bgeu", lambda a, b: a >= b),
]


@pytest.mark.parametrize("name,word,model", CMP_OPS, ids=[f"{o[0]}{i}" for i, o in enumerate(CMP_OPS)])
def test_compare_forms(oracle_mod, name, word, model):
    assert oracle_mod.mnemonic(word).replace(".", "_") == name
    for a, b in vectors():
        regs = [0] * 32
        regs[11], regs[12] = a, b
        p = oracle_mod.probe(word, 0x10000, regs)
        assert p.rd_value == model(a, b), (name, hex(a), hex(b))


def test_jalr_clears_bit0_and_links(oracle_mod):
    for base, imm in ((0x20001, 0), (0x20000, 3), (0x20000, -1), (M64, 2)):
        word = enc_i(0x67, 0, 1, 11, imm)             # jalr ra, imm(a1)
        regs = [0] * 32
        regs[11] = base
        p = oracle_mod.probe(word, 0x10000, regs)
        assert p.fault == 0 and p.rd == 1 and p.rd_value == 0x10004
        assert p.npc == ((base + imm) & M64) & ~1


def cmp_program_source() -> str:
    pairs = program_pairs()
    body = []
    k = 0
    for _, word, _ in CMP_OPS:
        body += [f"    .word {word:#010x}", f"    sd    a0, {8 * k}(s2)"]
        k += 1
    for j, (br, _) in enumerate(BRANCHES):
        body += ["    li    a0, 0", f"    {br:<5} a1, a2, br_{j}", "    li    a0, 1", f"br_{j}:",
                 f"    sd    a0, {8 * k}(s2)"]
        k += 1
    n_out = 8 * k * len(pairs)
    data = "\n".join(f"    .dword {a:#x}, {b:#x}" for a, b in pairs)
    return f"""    .text
_start:
    la    s0, vec
    li    s1, {len(pairs)}
    la    s2, out
loop:
    ld    a1, 0(s0)
    ld    a2, 8(s0)
{chr(10).join(body)}
    addi  s0, s0, 16
    addi  s2, s2, {8 * k}
    addi  s1, s1, -1
    bnez  s1, loop
    li    a0, 1
    la    a1, out
    li    a2, {n_out}
    li    a7, 64
    ecall
    li    a0, 0
    li    a7, 94
    ecall
    .data
    .balign 8
vec:
{data}
    .bss
    .balign 8
out:
    .zero {n_out}
"""


def cmp_program_elf() -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(cmp_program_source())


def cmp_program_expected() -> bytes:
    out = bytearray()
    for a, b in program_pairs():
        for _, _, m in CMP_OPS:
            out += m(a, b).to_bytes(8, "little")
        for _, c in BRANCHES:
            out += (0 if c(a, b) else 1).to_bytes(8, "little")
    return bytes(out)


def test_cmp_program_on_oracle(oracle_mod):
    o = oracle_mod.Oracle(cmp_program_elf(), "cmp")
    g = o.run_golden()
    assert g.exit_code == 0
    assert o.golden_stdout() == cmp_program_expected()


# ---- compressed (RVC + Zcb) register forms, single-instruction probes ----
# `decoder.isa:43-536`.  rd = rd' = a0 (x10, also the first source), rs2' = a1.
def _c(f3, b12, b11_7, b6_2, op):
    return (f3 << 13) | (b12 << 12) | (b11_7 << 7) | (b6_2 << 2) | op


def _ca(f6, rdp, f2, rs2p):
    return (f6 << 10) | (rdp << 7) | (f2 << 5) | (rs2p << 2) | 1


def _cb(f2, sh):   # c.srli / c.srai / c.andi on a0 (rd' = 2)
    return (0b100 << 13) | (((sh >> 5) & 1) << 12) | (f2 << 10) | (2 << 7) | ((sh & 31) << 2) | 1


COMPRESSED = [
    ("c_addi", _c(0, 1, 10, 0b11001, 1), lambda a, b: a - 7),
    ("c_addiw", _c(1, 1, 10, 0b11001, 1), lambda a, b: sx(a - 7, 32)),
    ("c_li", _c(2, 1, 10, 0b11001, 1), lambda a, b: -7),
    ("c_lui", _c(3, 1, 10, 0b00001, 1), lambda a, b: sx(0x21 << 12, 18)),
    ("c_srli", _cb(0, 33), lambda a, b: a >> 33),
    ("c_srai", _cb(1, 33), lambda a, b: s64(a) >> 33),
    ("c_andi", _cb(2, 0x39), lambda a, b: a & -7),
    ("c_sub", _ca(0b100011, 2, 0, 3), lambda a, b: a - b),
    ("c_xor", _ca(0b100011, 2, 1, 3), lambda a, b: a ^ b),
    ("c_or", _ca(0b100011, 2, 2, 3), lambda a, b: a | b),
    ("c_and", _ca(0b100011, 2, 3, 3), lambda a, b: a & b),
    ("c_subw", _ca(0b100111, 2, 0, 3), lambda a, b: sx(a - b, 32)),
    ("c_addw", _ca(0b100111, 2, 1, 3), lambda a, b: sx(a + b, 32)),
    ("c_mul", _ca(0b100111, 2, 2, 3), lambda a, b: a * b),
    ("c_zext_b", _ca(0b100111, 2, 3, 0), lambda a, b: a & 0xFF),
    ("c_sext_b", _ca(0b100111, 2, 3, 1), lambda a, b: sx(a, 8)),
    ("c_zext_h", _ca(0b100111, 2, 3, 2), lambda a, b: a & 0xFFFF),
    ("c_sext_h", _ca(0b100111, 2, 3, 3), lambda a, b: sx(a, 16)),
    ("c_zext_w", _ca(0b100111, 2, 3, 4), lambda a, b: a & M32),
    ("c_not", _ca(0b100111, 2, 3, 5), lambda a, b: ~a),
    ("c_slli", _c(0, 1, 10, 1, 2), lambda a, b: a << 33),
    ("c_mv", _c(4, 0, 10, 11, 2), lambda a, b: b),
    ("c_add", _c(4, 1, 10, 11, 2), lambda a, b: a + b),
]


@pytest.mark.parametrize("name,word,model", COMPRESSED, ids=[o[0] for o in COMPRESSED])
def test_compressed_forms(oracle_mod, name, word, model):
    assert oracle_mod.mnemonic(word).replace(".", "_") == name
    bad = []
    for a, b in vectors():
        regs = [0] * 32
        regs[10], regs[11] = a, b
        p = oracle_mod.probe(word, 0x10000, regs)
        assert p.fault == 0 and p.rd == 10 and p.len == 2 and p.npc == 0x10002
        want = model(a, b) & M64
        if p.rd_value != want:
            bad.append((hex(a), hex(b), hex(p.rd_value), hex(want)))
    assert not bad, f"{name}: {len(bad)} mismatches, first {bad[:3]}"


def rvc_program_source() -> str:
    pairs = program_pairs()
    body = []
    for k, (_, word, _) in enumerate(COMPRESSED):
        body += ["    ld    a0, 0(s0)", f"    .half {word:#06x}", f"    sd    a0, {8 * k}(s2)"]
    n_out = 8 * len(COMPRESSED) * len(pairs)
    data = "\n".join(f"    .dword {a:#x}, {b:#x}" for a, b in pairs)
    return f"""    .text
_start:
    la    s0, vec
    li    s1, {len(pairs)}
    la    s2, out
loop:
    ld    a1, 8(s0)
{chr(10).join(body)}
    addi  s0, s0, 16
    addi  s2, s2, {8 * len(COMPRESSED)}
    addi  s1, s1, -1
    bnez  s1, loop
    li    a0, 1
    la    a1, out
    li    a2, {n_out}
    li    a7, 64
    ecall
    li    a0, 0
    li    a7, 94
    ecall
    .data
    .balign 8
vec:
{data}
    .bss
    .balign 8
out:
    .zero {n_out}
"""


def rvc_program_elf() -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(rvc_program_source())


def rvc_program_expected() -> bytes:
    out = bytearray()
    for a, b in program_pairs():
        for _, _, m in COMPRESSED:
            out += (m(a, b) & M64).to_bytes(8, "little")
    return bytes(out)


def test_rvc_program_on_oracle(oracle_mod):
    o = oracle_mod.Oracle(rvc_program_elf(), "rvc")
    g = o.run_golden()
    assert g.exit_code == 0
    assert o.golden_stdout() == rvc_program_expected()


# ---- modelled syscalls (guest program) ----
# get*id return the Process params (`sim/Process.py:61-67`: pid 100, ppid 0,
# uid/euid/gid/egid 100; gettid -> pid), write to fd > 2 returns -EBADF,
# write of 0 bytes returns 0, write(2) goes to stderr, an ignoreFunc syscall
# returns 0 (`syscall_emul.cc:84-104`), exit status is `& 0xff`
# (`syscall_emul.cc:120-248`).
SYS_STDERR = b"err!\n?"
SYS_EXPECTED_VALUES = [100, 0, 100, 100, 100, 100, 100, -9, 0, len(SYS_STDERR), 0]


def sys_program_source() -> str:
    ids = "\n".join(f"    li    a7, {n}\n    ecall\n    sd    a0, {8 * k}(s2)" for k, n in enumerate(range(172, 179)))
    n_out = 8 * len(SYS_EXPECTED_VALUES)
    msg = ", ".join(str(c) for c in SYS_STDERR)
    return f"""    .text
_start:
    la    s2, out
{ids}
    li    a0, 5
    mv    a1, s2
    li    a2, 8
    li    a7, 64
    ecall
    sd    a0, 56(s2)
    li    a0, 1
    mv    a1, s2
    li    a2, 0
    li    a7, 64
    ecall
    sd    a0, 64(s2)
    li    a0, 2
    la    a1, msg
    li    a2, {len(SYS_STDERR)}
    li    a7, 64
    ecall
    sd    a0, 72(s2)
    li    a0, 12345
    li    a7, 99
    ecall
    sd    a0, 80(s2)
    li    a0, 1
    mv    a1, s2
    li    a2, {n_out}
    li    a7, 64
    ecall
    li    a0, 300
    li    a7, 93
    ecall
    .data
msg:
    .byte {msg}
    .bss
    .balign 8
out:
    .zero {n_out}
"""


def sys_program_elf() -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(sys_program_source())


def sys_program_expected() -> bytes:
    return b"".join((v & M64).to_bytes(8, "little") for v in SYS_EXPECTED_VALUES)


def test_sys_program_on_oracle(oracle_mod):
    o = oracle_mod.Oracle(sys_program_elf(), "sys")
    g = o.run_golden()
    assert g.exit_code == 300 & 0xFF
    assert g.stderr_len == len(SYS_STDERR)
    assert o.golden_stdout() == sys_program_expected()
    assert o.golden_stderr() == SYS_STDERR


# ---------------------------------------------------------------- LR / SC
# Known answers for LR/SC as gem5's atomic CPU with the reference's SE memory
# (NoCache: the data port reaches AbstractMemory) gives them: the ISA
# reservation (src/arch/riscv/isa.cc:1006-1064: set by each LR fragment,
# cleared by every SC, SC fails when it is empty or in another 64-byte line),
# and this context's lock record in memory (src/mem/abstract_mem.cc:258-345:
# granule = paddr & ~0xf, replaced by each LR, erased by any store to its
# granule -- the SC's own included -- kept by a failed SC; AMOs and proxy
# writes leave it).  rd = 0 on success, 1 on failure (formats/amo.isa).
LRSC_EXPECTED = [
    0x1111,      # 1. lr.d A
    0,           #    sc.d A succeeds (A = 0x2222)
    1,           # 2. sc.d with no reservation fails
    1,           # 3. lr.d A; sd to A's granule erases the lock; sc.d fails
    0,           # 4. lr.d A; sd to another granule of the line; sc.d succeeds (A = 0x3333)
    1,           # 5. lr.d A; sc.d to the next line fails (ISA) and clears the reservation
    1,           #    sc.d A fails: reservation empty
    1,           # 6. lr.d A; lr.d B (same line): record -> B; sc.d A passes the ISA, memory refuses
    0,           #    lr.w B; sc.w B succeeds
    (-5) & M64,  #    lw B: -5
    0,           # 7. lr.d A; amoadd.d A leaves the record; sc.d.aqrl A succeeds
    0x5555,      #    ld A
    (-2**31) & M64,   # 8. lr.w sign-extends
    0,           # 9. lr.d across a line (last fragment holds the reservation); sc.d there succeeds
    0x6666,      #    ld at the second fragment
]


def lrsc_program_source() -> str:
    return f"""    .text
_start:
    la    s0, buf
    la    s2, out
    li    t0, 0x1111
    sd    t0, 0(s0)
    sd    t0, 16(s0)
    sd    t0, 64(s0)
    lr.d  t1, (s0)
    li    t2, 0x2222
    sc.d  t3, t2, (s0)
    sd    t1, 0(s2)
    sd    t3, 8(s2)
    li    t2, 0x3333
    sc.d  t3, t2, (s0)
    sd    t3, 16(s2)
    lr.d  t1, (s0)
    sd    zero, 8(s0)
    sc.d  t3, t2, (s0)
    sd    t3, 24(s2)
    lr.d  t1, (s0)
    sd    zero, 16(s0)
    sc.d  t3, t2, (s0)
    sd    t3, 32(s2)
    lr.d  t1, (s0)
    addi  t4, s0, 64
    sc.d  t3, t2, (t4)
    sd    t3, 40(s2)
    sc.d  t3, t2, (s0)
    sd    t3, 48(s2)
    lr.d  t1, (s0)
    addi  t4, s0, 16
    lr.d  t1, (t4)
    li    t2, 0x4444
    sc.d  t3, t2, (s0)
    sd    t3, 56(s2)
    lr.w  t1, (t4)
    li    t2, -5
    sc.w  t3, t2, (t4)
    sd    t3, 64(s2)
    lw    t5, 0(t4)
    sd    t5, 72(s2)
    lr.d  t1, (s0)
    li    t2, 1
    amoadd.d t6, t2, (s0)
    li    t2, 0x5555
    sc.d.aqrl t3, t2, (s0)
    sd    t3, 80(s2)
    ld    t5, 0(s0)
    sd    t5, 88(s2)
    addi  t4, s0, 128
    li    t2, 0x80000000
    sw    t2, 0(t4)
    lr.w.aq t5, (t4)
    sd    t5, 96(s2)
    addi  t4, s0, 188
    lr.d  t1, (t4)
    addi  t4, s0, 192
    li    t2, 0x6666
    sc.d.rl t3, t2, (t4)
    sd    t3, 104(s2)
    ld    t5, 0(t4)
    sd    t5, 112(s2)
    li    a0, 1
    la    a1, out
    li    a2, {8 * len(LRSC_EXPECTED)}
    li    a7, 64
    ecall
    li    a0, 0
    li    a7, 94
    ecall
    .bss
    .balign 4096
buf:
    .zero 4096
out:
    .zero {8 * len(LRSC_EXPECTED)}
"""


def lrsc_program_elf() -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(lrsc_program_source())


def lrsc_program_expected() -> bytes:
    return b"".join((v & M64).to_bytes(8, "little") for v in LRSC_EXPECTED)


def test_lrsc_program_on_oracle(oracle_mod):
    o = oracle_mod.Oracle(lrsc_program_elf(), "lrsc")
    g = o.run_golden()
    assert g.exit_code == 0
    assert o.golden_stdout() == lrsc_program_expected()


def test_lrsc_decode(oracle_mod):
    # lr.w / sc.d / lr.d.aqrl decode to the executed ops (no longer escapes)
    for raw, name in ((0x1005272F, "lr_w"), (0x18B5362F, "sc_d"), (0x1605352F, "lr_d")):
        assert oracle_mod.mnemonic(raw) == name, hex(raw)


# SE memory map and the remaining deterministic handlers (oracle/rv64se.c
# do_syscall; gem5 MemState, src/sim/mem_state.cc): brk grows, shrinks (the
# pages leave the map and come back zero) and regrows; anonymous mmap grows
# down from mmap_end = 0x4000000000000000 (RiscvProcess64, process.cc:79), a
# free hint is honoured, MAP_FIXED replaces; munmap; set_tid_address; ioctl;
# getrlimit / prlimit64; uname; writev; close of stderr then write(2) ->
# -EBADF; exit clears *childClearTID.
VM_MMAP0 = 0x4000000000000000 - 0x2000
VM_EXPECTED_TAIL = [0x2800, 0x1234, 8, 0x2000, 0, VM_MMAP0, 0x77, 0, 0x1000, 0, 0x1000, 0, 0, -22, -9, -22, 100,
                    -25, -25, 0, 8 << 20, 0, 256 << 20, -1, -22, 0, 1, 0, 13, 5, 0, -9, -9, -9, 0, 0x2000]
VM_STDOUT_HEAD = b"Linuxriscv64\n"
VM_STDERR = b"Linux"


def vm_program_source() -> str:
    n_out = 8 * (1 + len(VM_EXPECTED_TAIL))
    def mmap(a0, a1, a3, a4=-1, a2=3):
        return (f"    {a0}\n    li    a1, {a1}\n    li    a2, {a2}\n    li    a3, {a3}\n    li    a4, {a4}\n"
                f"    li    a5, 0\n    li    a7, 222\n    ecall\n")
    return f"""    .text
_start:
    la    s2, out
    li    a0, 0
    li    a7, 214
    ecall
    mv    s0, a0
    sd    a0, 0(s2)
    li    t0, 0x2800
    add   a0, s0, t0
    li    a7, 214
    ecall
    sub   t1, a0, s0
    sd    t1, 8(s2)
    li    t0, 0x1000
    add   t3, s0, t0
    li    t1, 0x1234
    sd    t1, 0(t3)
    ld    t1, 0(t3)
    sd    t1, 16(s2)
    addi  a0, s0, 8
    li    a7, 214
    ecall
    sub   t1, a0, s0
    sd    t1, 24(s2)
    li    t0, 0x2000
    add   a0, s0, t0
    li    a7, 214
    ecall
    sub   t1, a0, s0
    sd    t1, 32(s2)
    ld    t1, 0(t3)
    sd    t1, 40(s2)
{mmap("li    a0, 0", 0x2000, 0x22)}    mv    s1, a0
    sd    a0, 48(s2)
    li    t0, 0x1008
    add   t3, s1, t0
    li    t1, 0x77
    sd    t1, 0(t3)
    ld    t1, 0(t3)
    sd    t1, 56(s2)
    li    t0, 0x1000
    add   a0, s1, t0
    li    a1, 0x1000
    li    a7, 215
    ecall
    sd    a0, 64(s2)
    li    t0, 0x1000
{mmap("add   a0, s1, t0", 0x1000, 0x22)}    sub   t1, a0, s1
    sd    t1, 72(s2)
    ld    t1, 0(t3)
    sd    t1, 80(s2)
{mmap("li    a0, 0", 0x1000, 0x22)}    sub   t1, s1, a0
    sd    t1, 88(s2)
    li    t1, 0x55
    sd    t1, 0(s1)
{mmap("mv    a0, s1", 0x1000, 0x32)}    sub   t1, a0, s1
    sd    t1, 96(s2)
    ld    t1, 0(s1)
    sd    t1, 104(s2)
{mmap("li    a0, 0", 0x1000, 0x20)}    sd    a0, 112(s2)
{mmap("li    a0, 0", 0x1000, 0x2, a4=3, a2=1)}    sd    a0, 120(s2)
    addi  a0, s1, 1
    li    a1, 0x1000
    li    a7, 215
    ecall
    sd    a0, 128(s2)
    la    a0, tid
    li    a7, 96
    ecall
    sd    a0, 136(s2)
    li    a0, 1
    li    a1, 0x5401
    li    a2, 0
    li    a7, 29
    ecall
    sd    a0, 144(s2)
    li    a0, 7
    li    a1, 0x1234
    li    a2, 0
    li    a7, 29
    ecall
    sd    a0, 152(s2)
    la    s3, rl
    li    a0, 3
    mv    a1, s3
    li    a7, 163
    ecall
    sd    a0, 160(s2)
    ld    t1, 0(s3)
    sd    t1, 168(s2)
    li    a0, 0
    li    a1, 2
    li    a2, 0
    mv    a3, s3
    li    a7, 261
    ecall
    sd    a0, 176(s2)
    ld    t1, 8(s3)
    sd    t1, 184(s2)
    li    a0, 1
    li    a1, 2
    li    a2, 0
    mv    a3, s3
    li    a7, 261
    ecall
    sd    a0, 192(s2)
    li    a0, 7
    mv    a1, s3
    li    a7, 163
    ecall
    sd    a0, 200(s2)
    li    a0, 6
    mv    a1, s3
    li    a7, 163
    ecall
    sd    a0, 208(s2)
    ld    t1, 0(s3)
    sd    t1, 216(s2)
    la    a0, uts
    li    a7, 160
    ecall
    sd    a0, 224(s2)
    la    t0, iov
    la    t1, uts
    sd    t1, 0(t0)
    li    t2, 5
    sd    t2, 8(t0)
    addi  t1, t1, 260
    sd    t1, 16(t0)
    li    t2, 7
    sd    t2, 24(t0)
    la    t1, nl
    sd    t1, 32(t0)
    li    t2, 1
    sd    t2, 40(t0)
    li    a0, 1
    la    a1, iov
    li    a2, 3
    li    a7, 66
    ecall
    sd    a0, 232(s2)
    li    a0, 2
    la    a1, iov
    li    a2, 1
    li    a7, 66
    ecall
    sd    a0, 240(s2)
    li    a0, 2
    li    a7, 57
    ecall
    sd    a0, 248(s2)
    li    a0, 2
    la    a1, nl
    li    a2, 1
    li    a7, 64
    ecall
    sd    a0, 256(s2)
    li    a0, 2
    la    a1, iov
    li    a2, 1
    li    a7, 66
    ecall
    sd    a0, 264(s2)
    li    a0, -1
    li    a7, 57
    ecall
    sd    a0, 272(s2)
    li    a0, 9
    li    a7, 57
    ecall
    sd    a0, 280(s2)
    li    a0, 0
    li    a7, 214
    ecall
    sub   t1, a0, s0
    sd    t1, 288(s2)
    li    a0, 1
    mv    a1, s2
    li    a2, {n_out}
    li    a7, 64
    ecall
    li    a0, 0
    li    a7, 93
    ecall
    .data
nl:
    .byte 10
    .bss
    .balign 8
out:
    .zero {n_out}
rl:
    .zero 16
iov:
    .zero 48
tid:
    .zero 8
uts:
    .zero 328
"""


def vm_program_elf() -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(vm_program_source())


def elf_brk0(elf: bytes) -> int:
    """roundUp(max p_vaddr + p_memsz of the PT_LOAD segments, page)."""
    import struct
    phoff, = struct.unpack_from("<Q", elf, 0x20)
    phentsize, phnum = struct.unpack_from("<HH", elf, 0x36)
    top = 0
    for i in range(phnum):
        p_type, _, _, vaddr, paddr, _, memsz = struct.unpack_from("<IIQQQQQ", elf, phoff + i * phentsize)
        if p_type == 1:
            top = max(top, paddr + memsz)
    return (top + 4095) & ~4095


def vm_program_expected() -> bytes:
    vals = [elf_brk0(vm_program_elf())] + VM_EXPECTED_TAIL
    return VM_STDOUT_HEAD + b"".join((v & M64).to_bytes(8, "little") for v in vals)


def test_vm_program_on_oracle(oracle_mod):
    o = oracle_mod.Oracle(vm_program_elf(), "vm")
    g = o.run_golden()
    assert g.exit_code == 0
    got = o.golden_stdout()
    exp = vm_program_expected()
    assert len(got) == len(exp)
    vals = [int.from_bytes(got[13 + 8 * k:21 + 8 * k], "little") for k in range((len(got) - 13) // 8)]
    evals = [int.from_bytes(exp[13 + 8 * k:21 + 8 * k], "little") for k in range((len(exp) - 13) // 8)]
    assert [hex(v) for v in vals] == [hex(v) for v in evals]
    assert got == exp
    assert o.golden_stderr() == VM_STDERR


# F/D/Zfh arithmetic known answers.  Each case loads NaN-boxed operand bits
# into f1..f3, runs one instruction with an explicit rounding mode (or the
# dynamic one after csrrwi frm), stores the destination's raw 64 bits and the
# fflags it raised (read-and-clear through csrrw fflags).  The expected values
# come from the reference's own SoftFloat (oracle/_ref) through the same
# operation codes the engine's port uses, with gem5's instruction-level rules
# (NaN-boxing, sign injection of fmsub/fnmadd, w/wu sign extension).
FP_BOX = {"h": 0xFFFFFFFFFFFF0000, "s": 0xFFFFFFFF00000000, "d": 0}
FP_SIGN = {"h": 0x8000, "s": 0x80000000, "d": 1 << 63}
FP_FMTC = {"h": 0, "s": 1, "d": 2}
RMS = {"rne": 0, "rtz": 1, "rdn": 2, "rup": 3, "rmm": 4}


def fp_cases():
    one = {"h": 0x3C00, "s": 0x3F800000, "d": 0x3FF0000000000000}
    three = {"h": 0x4200, "s": 0x40400000, "d": 0x4008000000000000}
    tenth = {"h": 0x2E66, "s": 0x3DCCCCCD, "d": 0x3FB999999999999A}
    big = {"h": 0x7BFF, "s": 0x7F7FFFFF, "d": 0x7FEFFFFFFFFFFFFF}
    tiny = {"h": 0x0001, "s": 0x00000001, "d": 0x0000000000000001}
    qnan = {"h": 0x7E00, "s": 0x7FC00000, "d": 0x7FF8000000000000}
    snan = {"h": 0x7C01, "s": 0x7F800001, "d": 0x7FF0000000000001}
    inf = {"h": 0x7C00, "s": 0x7F800000, "d": 0x7FF0000000000000}
    c = []
    for f in ("d", "s", "h"):
        n = lambda k: k[f] | FP_SIGN[f]   # noqa: E731
        for rm in ("rne", "rtz", "rdn", "rup", "rmm"):
            c.append(("fdiv", f, rm, one[f], three[f], 0))
            c.append(("fadd", f, rm, tenth[f], three[f], 0))
        c += [("fadd", f, "rne", big[f], big[f], 0), ("fsub", f, "rdn", three[f], three[f], 0),
              ("fmul", f, "rne", tiny[f], tenth[f], 0), ("fmul", f, "rup", tiny[f], tenth[f], 0),
              ("fmul", f, "rne", inf[f], 0, 0), ("fdiv", f, "rne", one[f], 0, 0), ("fdiv", f, "rne", 0, 0, 0),
              ("fsqrt", f, "rne", three[f], 0, 0), ("fsqrt", f, "rne", n(one), 0, 0),
              ("fsqrt", f, "rtz", tenth[f], 0, 0), ("fadd", f, "rne", snan[f], one[f], 0),
              ("fmadd", f, "rne", three[f], tenth[f], one[f]), ("fmsub", f, "rtz", three[f], tenth[f], one[f]),
              ("fnmsub", f, "rdn", three[f], tenth[f], one[f]), ("fnmadd", f, "rup", three[f], tenth[f], one[f]),
              ("fmadd", f, "rne", inf[f], 0, qnan[f]),
              ("fmin", f, None, 0, n({f: 0}), 0), ("fmax", f, None, 0, n({f: 0}), 0),
              ("fmin", f, None, qnan[f], one[f], 0), ("fmax", f, None, snan[f], one[f], 0),
              ("fminm", f, None, qnan[f], one[f], 0), ("fmaxm", f, None, three[f], one[f], 0),
              ("feq", f, None, qnan[f], one[f], 0), ("feq", f, None, snan[f], one[f], 0),
              ("flt", f, None, qnan[f], one[f], 0), ("fltq", f, None, qnan[f], one[f], 0),
              ("fle", f, None, one[f], one[f], 0), ("fleq", f, None, n(one), one[f], 0),
              ("fcvt.w", f, "rtz", n(three), 0, 0), ("fcvt.wu", f, "rne", n(three), 0, 0),
              ("fcvt.wu", f, "rne", three[f], 0, 0), ("fcvt.l", f, "rmm", tenth[f], 0, 0),
              ("fcvt.lu", f, "rup", tenth[f], 0, 0), ("fcvt.w", f, "rne", big[f], 0, 0),
              ("fcvt.w", f, "rne", qnan[f], 0, 0),
              ("fcvt.from.w", f, "rne", 0xFFFFFFFF80000001, 0, 0), ("fcvt.from.wu", f, "rtz", 0xFFFFFFFF, 0, 0),
              ("fcvt.from.l", f, "rdn", 0x7FFFFFFFFFFFFFFF, 0, 0), ("fcvt.from.lu", f, "rup", 0x1FFFFFFFFFFFFF, 0, 0)]
        for g in ("d", "s", "h"):
            if g != f:
                c += [(f"fcvt.to.{g}", f, "rne", tenth[f], 0, 0), (f"fcvt.to.{g}", f, "rtz", big[f], 0, 0),
                      (f"fcvt.to.{g}", f, "rne", snan[f], 0, 0)]
    return c


def fp_expected(case):
    """(destination register bits, fflags) per the reference SoftFloat."""
    from oracle.pyoracle import sf_ref
    op, f, rm, a, b, cc = case
    fc, r = FP_FMTC[f], RMS.get(rm, 0)

    def ref(code, x, y=0, z=0, fmt=fc, rmode=r):
        v, fl = sf_ref(code, fmt, rmode, [x], [y], [z])
        return int(v[0]), int(fl[0])
    box = lambda v: (v | FP_BOX[f]) & 0xFFFFFFFFFFFFFFFF   # noqa: E731
    s = FP_SIGN[f]
    ex = {"h": 0x7C00, "s": 0x7F800000, "d": 0x7FF0000000000000}[f]
    isnan = lambda v: (v & ~s) > ex   # noqa: E731
    codes = {"fadd": 0, "fsub": 1, "fmul": 2, "fdiv": 3, "fsqrt": 4}
    if op in codes:
        v, fl = ref(codes[op], a, b)
        return box(v), fl
    if op in ("fmadd", "fmsub", "fnmsub", "fnmadd"):
        x = a ^ (s if op in ("fnmsub", "fnmadd") else 0)
        z = cc ^ (s if op in ("fmsub", "fnmadd") else 0)
        v, fl = ref(5, x, b, z)
        return box(v), fl
    if op in ("fmin", "fmax", "fminm", "fmaxm"):
        p, q = (b, a) if op.startswith("fmax") else (a, b)
        pick, fl = ref(9, p, q)
        if not pick:
            e, fl2 = ref(6, p, q)
            pick = e and bool(p & s)
            fl |= fl2
        qn = {"h": 0x7E00, "s": 0x7FC00000, "d": 0x7FF8000000000000}[f]
        if op.endswith("m"):
            return (box(qn) if isnan(a) or isnan(b) else (a if pick else b)), fl
        return box(qn if isnan(a) and isnan(b) else (a if pick or isnan(b) else b)), fl
    if op in ("feq", "flt", "fltq", "fle", "fleq"):
        return ref({"feq": 6, "flt": 7, "fle": 8, "fltq": 9, "fleq": 10}[op], a, b)
    if op.startswith("fcvt.from."):
        k = {"w": 15, "wu": 16, "l": 17, "lu": 18}[op.split(".")[2]]
        v, fl = ref(k, a)
        return box(v), fl
    if op.startswith("fcvt.to."):
        g = op.split(".")[2]
        v, fl = ref(19 + FP_FMTC[g], a)
        return (v | FP_BOX[g]) & 0xFFFFFFFFFFFFFFFF, fl
    k = {"fcvt.w": 11, "fcvt.wu": 12, "fcvt.l": 13, "fcvt.lu": 14}[op]
    v, fl = ref(k, a)
    if k <= 12:
        v = (v & 0xFFFFFFFF) | (0xFFFFFFFF00000000 if v & 0x80000000 else 0)
    return v & 0xFFFFFFFFFFFFFFFF, fl


def fp_program_source():
    lines = ["    .text", "_start:", "    la    s2, out", "    mv    s3, s2"]
    for k, (op, f, rm, a, b, cc) in enumerate(fp_cases()):
        for reg_, val in (("f1", a), ("f2", b), ("f3", cc)):
            lines += [f"    li    t0, {(val | FP_BOX[f]) & 0xFFFFFFFFFFFFFFFF if not op.startswith('fcvt.from') else 0}",
                      f"    fmv.d.x {reg_}, t0"]
        rms = f", {rm}" if rm else ""
        if op.startswith("fcvt.from."):
            lines += [f"    li    t1, {a}", f"    fcvt.{f}.{op.split('.')[2]} f0, t1{rms}", "    fmv.x.d t1, f0"]
        elif op.startswith("fcvt.to."):
            lines += [f"    fcvt.{op.split('.')[2]}.{f} f0, f1{rms}", "    fmv.x.d t1, f0"]
        elif op.startswith("fcvt."):
            lines += [f"    {op}.{f} t1, f1{rms}"]
        elif op in ("feq", "flt", "fltq", "fle", "fleq"):
            lines += [f"    {op}.{f} t1, f1, f2"]
        elif op in ("fmadd", "fmsub", "fnmsub", "fnmadd"):
            lines += [f"    {op}.{f} f0, f1, f2, f3{rms}", "    fmv.x.d t1, f0"]
        elif op == "fsqrt":
            lines += [f"    fsqrt.{f} f0, f1{rms}", "    fmv.x.d t1, f0"]
        else:
            lines += [f"    {op}.{f} f0, f1, f2{rms}", "    fmv.x.d t1, f0"]
        lines += ["    sd    t1, 0(s2)", "    csrrw t2, 1, zero", "    sd    t2, 8(s2)", "    addi  s2, s2, 16"]
    n = len(fp_cases())
    # the dynamic rounding mode: frm = rtz, 1/3 in binary64, then fcsr read back
    lines += ["    csrrwi zero, 2, 1", "    li    t0, 4607182418800017408", "    fmv.d.x f1, t0",
              "    li    t0, 4613937818241073152", "    fmv.d.x f2, t0", "    fdiv.d f0, f1, f2",
              "    fmv.x.d t1, f0", "    sd    t1, 0(s2)", "    csrrs t2, 3, zero",
              "    sd    t2, 8(s2)",
              "    li    a0, 1", "    mv    a1, s3", f"    li    a2, {16 * (n + 1)}", "    li    a7, 64", "    ecall",
              "    li    a0, 0", "    li    a7, 93", "    ecall", "    .bss", "    .balign 8", "out:",
              f"    .zero {16 * (n + 1)}"]
    return "\n".join(lines) + "\n"


def fp_program_elf() -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(fp_program_source())


def fp_program_expected() -> bytes:
    from oracle.pyoracle import sf_ref
    vals = []
    for case in fp_cases():
        vals += list(fp_expected(case))
    v, fl = sf_ref(3, 2, 1, [0x3FF0000000000000], [0x4008000000000000])   # 1/3 rounded toward zero
    vals += [int(v[0]), int(fl[0]) | (1 << 5)]                               # fcsr = fflags | rtz << 5
    return b"".join((x & M64).to_bytes(8, "little") for x in vals)


def test_fp_program_on_oracle(oracle_mod):
    from oracle.pyoracle import has_softfloat
    if not has_softfloat():
        pytest.skip("oracle without the reference SoftFloat")
    o = oracle_mod.Oracle(fp_program_elf(), "fp")
    g = o.run_golden()
    assert g.exit_code == 0, g
    got, exp = o.golden_stdout(), fp_program_expected()
    assert len(got) == len(exp)
    cases = fp_cases() + [("dyn", "d", "frm", 0, 0, 0)]
    for k, case in enumerate(cases):
        gv, gf = (int.from_bytes(got[16 * k + 8 * j:16 * k + 8 * j + 8], "little") for j in (0, 1))
        ev, ef = (int.from_bytes(exp[16 * k + 8 * j:16 * k + 8 * j + 8], "little") for j in (0, 1))
        assert (gv, gf) == (ev, ef), (k, case, hex(gv), gf, hex(ev), ef)


def test_fp_known_values():
    """A few binary64 answers that need no SoftFloat: numpy's IEEE RNE arithmetic."""
    import numpy as np
    from oracle.pyoracle import has_softfloat, sf_ref
    if not has_softfloat():
        pytest.skip("oracle without the reference SoftFloat")
    rng = np.random.default_rng(5)
    x = rng.standard_normal(1000) * 10.0 ** rng.integers(-30, 30, 1000)
    y = rng.standard_normal(1000) * 10.0 ** rng.integers(-30, 30, 1000)
    xb, yb = x.view(np.uint64), y.view(np.uint64)
    for code, npop in ((0, np.add), (1, np.subtract), (2, np.multiply), (3, np.divide)):
        v, _ = sf_ref(code, 2, 0, xb, yb)
        assert (v == npop(x, y).view(np.uint64)).all()
    v, _ = sf_ref(4, 2, 0, np.abs(x).view(np.uint64))
    assert (v == np.sqrt(np.abs(x)).view(np.uint64)).all()


# getrandom and clock_gettime (oracle/rv64se.c; syscall_emul.hh:3222-3236 and
# 2266-2278): the bytes are gem5's Random(5489) stream (std::mt19937_64)
# % 255 -- the first 12 draws below from the C++ standard library's
# std::mt19937_64(5489u); clock_gettime reports curTick in ns + 1e9 s, so two
# calls K uncompressed instructions (K ticks) apart differ by K x 500 / 1000 ns
# at the default 2 GHz.
RND_BYTES = bytes([175, 33, 200, 247, 86])
CLK_GAP = 40


def rnd_program_source() -> str:
    gap = "\n".join(["    addi  t3, t3, 1"] * (CLK_GAP - 2))
    return f"""    .text
_start:
    la    s2, out
    mv    a0, s2
    li    a1, 5
    li    a2, 0
    li    a7, 278
    ecall
    sd    a0, 8(s2)
    li    a0, 0
    addi  a1, s2, 16
    li    a7, 113
    ecall
{gap}
    addi  a1, s2, 32
    ecall
    li    a0, 1
    mv    a1, s2
    li    a2, 48
    li    a7, 64
    ecall
    li    a0, 0
    li    a7, 93
    ecall
    .bss
    .balign 8
out:
    .zero 48
"""


def rnd_program_elf() -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(rnd_program_source(), compress=False)


def rnd_check(out: bytes):
    assert out[:5] == RND_BYTES and out[5:8] == bytes(3)
    assert int.from_bytes(out[8:16], "little") == 5
    s1, n1, s2, n2 = (int.from_bytes(out[k:k + 8], "little") for k in (16, 24, 32, 40))
    assert s1 == s2 == 10**9
    assert n2 - n1 == CLK_GAP * 500 // 1000


def test_rnd_program_on_oracle(oracle_mod):
    o = oracle_mod.Oracle(rnd_program_elf(), "rnd")
    g = o.run_golden()
    assert g.exit_code == 0
    rnd_check(o.golden_stdout())


def rnd_program_expected() -> bytes:
    """The oracle's output for the rnd program, itself checked by rnd_check."""
    from oracle import pyoracle
    o = pyoracle.Oracle(rnd_program_elf(), "rnd")
    o.run_golden()
    out = o.golden_stdout()
    rnd_check(out)
    return out


# ---------------------------------------------------------------- stdin program
# Process.input as a file (src/sim/Process.py:44, fd_array.cc:69-75) and
# readFunc (syscall_emul.hh:2798-2822): read(0) takes min(n, left) bytes at
# the file offset and the zero-filled BufferArg copies all n bytes out when the
# read returned any (syscall_emul_buf.hh:55-85); at EOF nothing is copied (a
# null buffer is fine); write / writev to the O_RDONLY fd 0 give -EBADF.
STDIN_DATA = b"abcdefghij0123456789XYZ"
STDIN_CALLS = [(0, 8), (8, 4), (16, 32), (48, 8), (None, 8)]   # (buffer offset | None = null, n)


def stdin_program_source() -> str:
    body = []
    for k, (off, n) in enumerate(STDIN_CALLS):
        buf = "    li    a1, 0" if off is None else f"    addi  a1, s2, {off}"
        body += ["    li    a0, 0", buf, f"    li    a2, {n}", "    li    a7, 63", "    ecall",
                 f"    sd    a0, {8 * k}(s3)"]
    k = len(STDIN_CALLS)
    body += ["    li    a0, 0", "    mv    a1, s2", "    li    a2, 4", "    li    a7, 64", "    ecall",
             f"    sd    a0, {8 * k}(s3)"]
    body += ["    sd    s2, 0(s4)", "    li    t0, 4", "    sd    t0, 8(s4)",
             "    li    a0, 0", "    mv    a1, s4", "    li    a2, 1", "    li    a7, 66", "    ecall",
             f"    sd    a0, {8 * (k + 1)}(s3)"]
    body = "\n".join(body)
    return f"""    .text
_start:
    la    s2, buf
    la    s3, res
    la    s4, iov
{body}
    li    a0, 1
    mv    a1, s2
    li    a2, 56
    li    a7, 64
    ecall
    li    a0, 1
    mv    a1, s3
    li    a2, {8 * (len(STDIN_CALLS) + 2)}
    li    a7, 64
    ecall
    li    a0, 0
    li    a7, 93
    ecall
    .data
    .balign 8
buf:
""" + "\n".join(["    .dword 0xaaaaaaaaaaaaaaaa"] * 7) + f"""
res:
    .zero {8 * (len(STDIN_CALLS) + 2)}
iov:
    .zero 16
"""


def stdin_program_elf() -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(stdin_program_source(), compress=False)


def stdin_program_expected() -> bytes:
    """Model: the buffer after the reads, then each call's return value."""
    buf = bytearray(b"\xaa" * 56)
    pos, rets = 0, []
    for off, n in STDIN_CALLS:
        k = min(n, len(STDIN_DATA) - pos)
        if k and off is not None:
            buf[off:off + n] = STDIN_DATA[pos:pos + k] + bytes(n - k)
        pos += k
        rets.append(k)
    rets += [-9, -9]
    return bytes(buf) + b"".join((r & (2**64 - 1)).to_bytes(8, "little") for r in rets)


def test_stdin_program_on_oracle(oracle_mod):
    o = oracle_mod.Oracle(stdin_program_elf(), "stdin")
    o.set_stdin(STDIN_DATA)
    g = o.run_golden()
    assert g.exit_code == 0
    assert o.golden_stdout() == stdin_program_expected()


def test_stdin_cin_escapes_on_oracle(oracle_mod):
    """Process.input = "cin" (the default): the read of the host's stdin is not
    reproducible -- the golden run itself ends as escape/host."""
    o = oracle_mod.Oracle(stdin_program_elf(), "stdin")
    with pytest.raises(RuntimeError):
        o.run_golden()
    out, _ = o.run_one()
    assert (out["cls"], out["sub"]) == (5, 4)


# ---------------------------------------------------------------- clk program
# A branch on s3 whose two arms commit the same instructions but take
# different numbers of ticks: the taken arm (s3 != 0, a fault) adds CLK_ECALLS
# ignored-syscall ecalls, each one tick that does not count as an instruction
# (SyscallFault: atomic.cc:688-700 counts numInst only on NoFault).  Both arms
# leave a0 = 0, a7 = 99, and s3 is rewritten after the merge, so a trial that
# took the slow arm reaches every later snapshot with the golden registers,
# memory, pc and numInst -- only curTick differs.  The program then reads
# clock_gettime (curTick in ns, syscall_emul.hh:2266-2278) and prints it: the
# trial prints CLK_ECALLS * 500 / 1000 ns more than the golden run (SDC).
CLK_PRE = 300      # instructions before the branch (fault sites)
CLK_POST = 700     # instructions between the merge and the clock read (snapshot boundaries)
CLK_ECALLS = 16


def clk_program_source() -> str:
    pre = "\n".join(["    addi  t3, t3, 1"] * CLK_PRE)
    post = "\n".join(["    addi  t4, t4, 3"] * CLK_POST)
    ecalls = "\n".join(["    ecall"] * CLK_ECALLS)
    return f"""    .text
_start:
    la    s2, out
    li    s3, 0
{pre}
    bnez  s3, slow
    li    a0, 0
    li    a7, 99
    j     merge
slow:
    li    a7, 99
{ecalls}
    li    a0, 0
    j     merge
merge:
    li    s3, 0
{post}
    li    a0, 0
    mv    a1, s2
    li    a7, 113
    ecall
    li    a0, 1
    mv    a1, s2
    li    a2, 16
    li    a7, 64
    ecall
    li    a0, 0
    li    a7, 93
    ecall
    .bss
    .balign 8
out:
    .zero 16
"""


def clk_program_elf() -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(clk_program_source(), compress=False)


def clk_branch_sites(n=64):
    """Faults on s3 (x19) before the branch: every bit sends the trial down the slow arm."""
    import numpy as np
    from oracle.pyoracle import SITE_DT
    s = np.zeros(n, SITE_DT)
    s["inst"] = 3 + np.arange(n) * (CLK_PRE // n)
    s["mask"] = np.uint64(1) << (np.arange(n) % 64).astype(np.uint64)
    s["target"] = 19
    s["trial"] = np.arange(n)
    return s


def clk_program_expected() -> bytes:
    from oracle import pyoracle
    o = pyoracle.Oracle(clk_program_elf(), "clk")
    o.run_golden()
    return o.golden_stdout()


def test_clk_program_on_oracle(oracle_mod):
    """The oracle's golden run prints curTick at the clock read; a branch-register
    fault (slow arm) ends SDC, its output later by exactly the extra ticks."""
    o = oracle_mod.Oracle(clk_program_elf(), "clk")
    g = o.run_golden()
    assert g.exit_code == 0
    out = o.golden_stdout()
    sec, nsec = int.from_bytes(out[:8], "little"), int.from_bytes(out[8:16], "little")
    assert sec == 10**9
    assert 0 < nsec < g.ncycles * 500 // 1000
    sites = clk_branch_sites(8)
    res = o.run_trials(sites, protect_mask=0)
    assert (res["cls"] == 1).all()              # SDC: the printed time differs
    assert (res["ninst"] == g.ninst).all()      # ... with the golden instruction count
    _, t = o.run_one(sites[0], protect_mask=0)
    t_ns = int.from_bytes(t[8:16], "little")
    assert t_ns - nsec == CLK_ECALLS * 500 // 1000


# ---------------------------------------------------------------- xop program
# The instruction groups gem5 executes outside the base ISA (oracle/rv64se.c
# refine_misc, the Zfa ops): scalar crypto on operand pairs (answers from the
# reference's rvk.hh through oracle/_ref), Zfa fli (the reference decoder's
# tables, tests/golden/fli_rv64.json), fround / froundnx (the reference
# SoftFloat's roundToInt) and fcvtmod.w.d (a model of decoder.isa:3320-3384),
# M5 pseudo-ops under SE defaults (rpns = curTick() in ns, m5sum, initparam
# keys, functions without an architectural effect; a1 = 0 after each), the
# warn-only privileged no-ops, and cbo.zero / cbo.clean / cbo.flush /
# cbo.inval on a 64-byte line.
XOP_PAIRS = [(0x0123456789ABCDEF, 0xFEDCBA9876543210), (0, 0xFFFFFFFFFFFFFFFF), (0x8000000080000000, 0x7F),
             (0xDEADBEEFCAFEBABE, 0x0F1E2D3C4B5A6978)]
XOP_CRYPTO = [*range(0, 11), 11 | (0 << 8), 11 | (9 << 8), 11 | (0xA << 8), 11 | (0xF << 8), 12,
              *[13 | (bs << 8) for bs in range(4)], *[14 | (bs << 8) for bs in range(4)], *range(15, 22)]
XOP_FROUND = [0x3FF8000000000000, 0xC004000000000000, 0x4330000000000001, 0x3FE0000000000000,
              0xBFE8000000000000, 0x7FF0000000000000, 0x7FF4000000000000, 0x0000000000000001]
XOP_FCVTMOD = [0x41E0000000000000, 0xC1E0000000200000, 0x4340000000000001, 0x4540000000000005,
               0x3FF8000000000000, 0xBFF0000000000000, 0x7FF8000000000000, 0x0000000000000003,
               0x45B0000000000000, 0xC3F0000000012345]
XOP_M5_NOEFFECT = [0x00, 0x09, 0x0D, 0x10, 0x11, 0x20, 0x31, 0x40, 0x41, 0x42, 0x43, 0x50, 0x52, 0x55, 0x59, 0x7F]
XOP_RPNS_GAP = 40
XOP_PRIV_NOPS = [0x16000073, 0x18000073, 0x18100073, 0x26000073, 0x66000073]
# RVV before any vset* (vl = 0): no-ops of one micro-op tick (vadd.vv, vle8.v,
# vse32.v, vmerge.vvm, vslideup.vx, vrgather.vv, vlse64.v, vluxei8.v,
# vlseg2e8.v) and of two (vle8ff.v: + the vl trim; vsaddu.vv: + vxsat)
XOP_VNOPS = [0x02218057, 0x02050087, 0x0205e0a7, 0x5c2180d7, 0x3a2540d7, 0x322180d7, 0x0a2570d7 & ~0x70 | 0x07,
             0x06250087, 0x22050087, 0x03050087, 0x822180d7]


def _crypto_word(fn, rd=7, rs1=5, rs2=6):
    f, sub = fn & 0xFF, fn >> 8
    if f <= 9:
        return (0x08 << 25) | (f << 20) | (rs1 << 15) | (1 << 12) | (rd << 7) | 0x13
    if f == 10:
        return (0x18 << 25) | (rs1 << 15) | (1 << 12) | (rd << 7) | 0x13
    if f == 11:
        return (0x18 << 25) | (1 << 24) | (sub << 20) | (rs1 << 15) | (1 << 12) | (rd << 7) | 0x13
    if f == 12:
        return (0x34 << 25) | (7 << 20) | (rs1 << 15) | (5 << 12) | (rd << 7) | 0x13
    f7 = {13: (sub << 5) | 0x18, 14: (sub << 5) | 0x1A, 15: 0x19, 16: 0x1B, 17: 0x1D, 18: 0x1F, 19: 0x3F,
          20: 0x14, 21: 0x14}[f]
    f3 = {20: 2, 21: 4}.get(f, 0)
    return (f7 << 25) | (rs2 << 20) | (rs1 << 15) | (f3 << 12) | (rd << 7) | 0x33


def _fcvtmod_model(a):
    sign, ex, frac = a >> 63, (a >> 52) & 0x7FF, a & ((1 << 52) - 1)
    inexact = invalid = False
    if ex == 0:
        inexact, frac = frac != 0, 0
    elif ex == 0x7FF:
        invalid, frac = True, 0
    else:
        te = ex - 1023
        m = frac | (1 << 52)
        sh = te - 52
        if sh >= 0:
            v = (m << sh) if sh < 64 else 0
            v &= (1 << 64) - 1
        else:
            inexact = (m & ((1 << -sh) - 1)) != 0 if -sh < 64 else True
            v = m >> -sh if -sh < 64 else 0
        if te > 31 or v > (0x80000000 if sign else 0x7FFFFFFF):
            invalid, inexact = True, False
        frac = (-v) & ((1 << 64) - 1) if sign else v
    r = frac & 0xFFFFFFFF
    r = r | 0xFFFFFFFF00000000 if r & 0x80000000 else r
    return r, (1 if inexact else 0) | (16 if invalid else 0)


def xop_program_source() -> str:
    L = ["    .text", "_start:", "    .word 0x0E00007B", "    mv    s4, a0"]      # rpns at tick 0
    L += ["    addi  t3, t3, 1"] * (XOP_RPNS_GAP - 2)
    L += ["    .word 0x0E00007B", "    mv    s5, a0"]
    L += [f"    .word {w:#x}" for w in XOP_VNOPS]
    L += ["    .word 0x0E00007B", "    mv    s6, a0", "    la    s2, out", "    mv    s3, s2",
          "    sd    s4, 0(s2)", "    sd    s5, 8(s2)", "    sd    s6, 16(s2)", "    addi  s2, s2, 24"]
    # m5sum, initparam keys, functions without an effect (a0 / a1 after each)
    L += [f"    li    a{k}, {0x1111 * (k + 1) + (1 << (60 - k))}" for k in range(6)]
    L += ["    .word 0x4600007B", "    sd    a0, 0(s2)", "    sd    a1, 8(s2)", "    addi  s2, s2, 16"]
    for k0, k1 in ((0, 0x55), (int.from_bytes(b"dist-ran", "little"), ord("k")),
                   (int.from_bytes(b"dist-siz", "little"), ord("e"))):
        L += [f"    li    a0, {k0}", f"    li    a1, {k1}", "    .word 0x6000007B", "    sd    a0, 0(s2)",
              "    sd    a1, 8(s2)", "    addi  s2, s2, 16"]
    for fn in XOP_M5_NOEFFECT:
        L += ["    li    a0, -1", "    li    a1, -2", f"    .word {(fn << 25) | 0x7B:#x}", "    sd    a0, 0(s2)",
              "    sd    a1, 8(s2)", "    addi  s2, s2, 16"]
    L += [f"    .word {w:#x}" for w in XOP_PRIV_NOPS]
    # scalar crypto
    for a, b in XOP_PAIRS:
        L += [f"    li    t0, {a}", f"    li    t1, {b}"]
        for fn in XOP_CRYPTO:
            L += [f"    .word {_crypto_word(fn):#x}", "    sd    t2, 0(s2)", "    addi  s2, s2, 8"]
    # Zfa: fli in all three formats
    for f7 in (0x78, 0x79, 0x7A):
        for i in range(32):
            L += [f"    .word {(f7 << 25) | (1 << 20) | (i << 15) | (0 << 7) | 0x53:#x}", "    fmv.x.d t2, f0",
                  "    sd    t2, 0(s2)", "    addi  s2, s2, 8"]
    # fround / froundnx (binary64, every static rounding mode), flags read and cleared
    for x in XOP_FROUND:
        L += [f"    li    t0, {x}", "    fmv.d.x f1, t0"]
        for nx in (0, 1):
            for rm in range(5):
                L += [f"    .word {(0x21 << 25) | ((4 + nx) << 20) | (1 << 15) | (rm << 12) | 0x53:#x}",
                      "    fmv.x.d t2, f0", "    csrrw t3, 1, zero", "    sd    t2, 0(s2)", "    sd    t3, 8(s2)",
                      "    addi  s2, s2, 16"]
    for x in XOP_FCVTMOD:
        L += [f"    li    t0, {x}", "    fmv.d.x f1, t0",
              f"    .word {(0x61 << 25) | (8 << 20) | (1 << 15) | (1 << 12) | (7 << 7) | 0x53:#x}",
              "    csrrw t3, 1, zero", "    sd    t2, 0(s2)", "    sd    t3, 8(s2)", "    addi  s2, s2, 16"]
    # cache-block ops on two 0xFF lines: zero the first (through an unaligned
    # pointer), clean / flush / inval the second; then print both lines
    L += ["    la    t0, lines", "    li    t1, -1", "    li    t4, 16"]
    L += ["fill:", "    sd    t1, 0(t0)", "    addi  t0, t0, 8", "    addi  t4, t4, -1", "    bnez  t4, fill"]
    L += ["    la    t0, lines", "    addi  t0, t0, 37", f"    .word {(4 << 20) | (5 << 15) | (2 << 12) | 0x0F:#x}",
          "    addi  t0, t0, 64"]
    L += [f"    .word {(k << 20) | (5 << 15) | (2 << 12) | 0x0F:#x}" for k in (0, 1, 2)]
    L += ["    la    t0, lines", "    li    t4, 16"]
    L += ["dump:", "    ld    t1, 0(t0)", "    sd    t1, 0(s2)", "    addi  s2, s2, 8", "    addi  t0, t0, 8",
          "    addi  t4, t4, -1", "    bnez  t4, dump"]
    L += ["    li    a0, 1", "    mv    a1, s3", "    sub   a2, s2, s3", "    li    a7, 64", "    ecall",
          "    li    a0, 0", "    li    a7, 93", "    ecall",
          "    .data", "    .balign 64", "lines:", "    .zero 128",
          "    .bss", "    .balign 8", "out:", "    .zero 8192"]
    return "\n".join(L) + "\n"


def xop_program_elf() -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(xop_program_source(), compress=False)


def xop_program_expected() -> bytes:
    from oracle.pyoracle import rvk_ref, sf_ref
    from oracle.pyoracle import mnemonic
    M = (1 << 64) - 1
    acts = [mnemonic(w) for w in XOP_VNOPS]
    assert set(acts) == {"vector:2", "vector:3"}, acts
    ticks = XOP_RPNS_GAP + 2 + sum(1 if a == "vector:2" else 2 for a in acts)
    vals = [0, XOP_RPNS_GAP * 500 // 1000, ticks * 500 // 1000]
    sargs = [0x1111 * (k + 1) + (1 << (60 - k)) for k in range(6)]
    vals += [sum(sargs) & M, 0]
    vals += [0, 0, 0, 0, 1, 0]
    for _ in XOP_M5_NOEFFECT:
        vals += [0, 0]
    for a, b in XOP_PAIRS:
        for fn in XOP_CRYPTO:
            vals.append(int(rvk_ref(fn, [a], [b])[0]))
    fli = json.load(open(os.path.join(ROOT, "tests", "golden", "fli_rv64.json")))
    for f, box in (("s", 0xFFFFFFFF00000000), ("d", 0), ("h", 0xFFFFFFFFFFFF0000)):
        vals += [v | box for v in fli[f]]
    for x in XOP_FROUND:
        for nx in (0, 1):
            for rm in range(5):
                v, fl = sf_ref(22 + nx, 2, rm, [x])
                vals += [int(v[0]), int(fl[0])]
    for x in XOP_FCVTMOD:
        vals += list(_fcvtmod_model(x))
    lines = [0] * 8 + [M] * 8
    vals += lines
    return b"".join((v & M).to_bytes(8, "little") for v in vals)


def test_xop_program_on_oracle(oracle_mod):
    from oracle.pyoracle import has_rvk, has_softfloat
    if not (has_softfloat() and has_rvk()):
        pytest.skip("oracle without the reference SoftFloat / rvk.hh")
    o = oracle_mod.Oracle(xop_program_elf(), "xop")
    g = o.run_golden()
    assert g.exit_code == 0, g
    got, exp = o.golden_stdout(), xop_program_expected()
    assert len(got) == len(exp)
    for k in range(0, len(exp), 8):
        assert got[k:k + 8] == exp[k:k + 8], (k // 8, got[k:k + 8].hex(), exp[k:k + 8].hex())


def test_fli_probe_matches_reference_table(oracle_mod):
    fli = json.load(open(os.path.join(ROOT, "tests", "golden", "fli_rv64.json")))
    for f7, f, box in ((0x78, "s", 0xFFFFFFFF00000000), (0x79, "d", 0), (0x7A, "h", 0xFFFFFFFFFFFF0000)):
        for i in range(32):
            p = oracle_mod.probe((f7 << 25) | (1 << 20) | (i << 15) | (3 << 7) | 0x53, 0x1000, [0] * 32)
            assert p.fault == 0 and p.rd == 35 and p.rd_value == fli[f][i] | box, (f, i, hex(p.rd_value))


def test_vector_actions_before_vset(oracle_mod):
    """RVV before any vset* (gen_vector_actions.py): vill-checking classes raise
    IllegalInst, floating-point classes reach GEM5_UNREACHABLE at SEW = 8
    (escape), whole-register moves need vector state (escape); a legal vset*
    executes (rd = VLMAX here)."""
    P = oracle_mod.probe
    regs = [0] * 32
    cases = {0x622180d7: ("vector:4", 3),    # vmseq.vv: the first micro-op checks vill
             0x422020d7: ("vector:4", 3),    # vmv.x.s x1, v2 (non-split)
             0x02219057: ("vector:5", 5),    # vfadd.vv: no SEW = 8 instantiation
             0x0c0071d7: ("vsetvli", 0),     # vsetvli x3, x0, e8, m1, ta, ma: rd = VLMAX = 32
             0x02828087: ("vector:6", 5),    # vl1re8.v (whole register)
             0x02218057: ("vector:2", 0)}    # vadd.vv: a no-op at vl = 0
    for w, (name, fault) in cases.items():
        assert oracle_mod.mnemonic(w) == name, (hex(w), oracle_mod.mnemonic(w))
        assert P(w, 0x1000, regs).fault == fault, hex(w)
    assert P(0x0c0071d7, 0x1000, regs).rd_value == 32


def _vsetvli(rd, rs1, zimm):
    return (zimm << 20) | (rs1 << 15) | (7 << 12) | (rd << 7) | 0x57


def _vsetivli(rd, uimm, zimm):
    return (3 << 30) | (zimm << 20) | (uimm << 15) | (7 << 12) | (rd << 7) | 0x57


def _vsetvl(rd, rs1, rs2):
    return (1 << 31) | (rs2 << 20) | (rs1 << 15) | (7 << 12) | (rd << 7) | 0x57


VILL = 1 << 63


def vset_model(vtype, vl, form, rd, rs1, req, avl):
    """VConfOp::execute (formats/vector_conf.isa:115-186) restated: the new
    (vtype, vl), or None where getSew's assert (vsew > 3) aborts.  form 0
    vsetvli (req = zimm11, avl = x[rs1]), 1 vsetvl (req = x[rs2]), 2 vsetivli
    (req = zimm10, avl = uimm, rs1 taken as nonzero).  VLEN 256, ELEN 64."""
    nt = vtype
    if req != vtype:
        vsew, vlmul = (req >> 3) & 7, req & 7
        if vsew > 3:
            return None
        lmul = {0: 1, 1: 2, 2: 4, 3: 8, 5: 1 / 8, 6: 1 / 4, 7: 1 / 2}.get(vlmul, 1 / 16)
        sew = 8 << vsew
        illegal = not (0.125 <= lmul <= 8) or sew > min(lmul, 1.0) * 64 or (req >> 8) & ((1 << 55) - 1)
        nt = VILL if illegal else req
    vlmax = 0 if nt >> 63 else int((256 // (8 << ((nt >> 3) & 7))) *
                                   {0: 1, 1: 2, 2: 4, 3: 8, 5: 1 / 8, 6: 1 / 4, 7: 1 / 2}[nt & 7])
    rs1_bits = 1 if form == 2 else rs1
    req_vl = avl & 0xFFFFFFFF
    if vlmax == 0:
        nvl = 0
    elif rd == 0 and rs1_bits == 0:
        nvl = min(vl, vlmax)
    elif rs1_bits == 0:
        nvl = vlmax
    else:
        nvl = min(req_vl, vlmax)
    return nt, nvl


def _vset_word_model(w, regs, vtype=VILL, vl=0):
    rd, rs1, rs2 = (w >> 7) & 31, (w >> 15) & 31, (w >> 20) & 31
    form = 0 if not w >> 31 else 2 if (w >> 30) & 1 else 1
    req = (w >> 20) & 0x7FF if form == 0 else regs[rs2] if form == 1 else (w >> 20) & 0x3FF
    avl = rs1 if form == 2 else (regs[rs1] if rs1 else 0)
    return vset_model(vtype, vl, form, rd, rs1, req, avl)


def test_vset_from_the_start_state(oracle_mod):
    """vset* (formats/vector_conf.isa:115-186) from the process-start state
    (vtype = vill, vl = 0) against the restated model: a request equal to the
    current vtype or an illegal one (LMUL 1/16, SEW > min(LMUL, 1) x ELEN,
    reserved bits) leaves that state and writes vl = 0 to rd; vsew > 3 trips
    getSew's assert (abort: fault 11, crash sub-code 14); a legal vtype
    writes rd = the new vl (AVL, VLMAX or the uint32_t truncation of x[rs1])."""
    P = oracle_mod.probe
    regs = [0] * 32
    regs[6], regs[7] = 5, 0x1234
    words = [_vsetvli(7, 6, 0x100), _vsetvli(7, 0, 0x004), _vsetvli(7, 6, 0x01D), _vsetvli(7, 6, 0x00D),
             _vsetivli(7, 31, 0x104), _vsetivli(7, 5, 0x016), _vsetvli(7, 6, 0x005), _vsetivli(7, 5, 0x00E),
             _vsetvli(7, 6, 0x0C0), _vsetvli(7, 6, 0x020), _vsetivli(7, 1, 0x3FF), _vsetvli(7, 6, 0x13C),
             _vsetvli(7, 0, 0x018), _vsetvli(0, 0, 0x018), _vsetvli(7, 6, 0x0D3), _vsetivli(7, 31, 0x0C5),
             _vsetivli(0, 3, 0x01F)]
    faults = {}
    for w in words:
        p = P(w, 0x1000, regs)
        assert oracle_mod.mnemonic(w) == ("vsetvli" if w >> 31 == 0 else "vsetivli"), hex(w)
        m = _vset_word_model(w, regs)
        assert p.fault == (11 if m is None else 0), (hex(w), p.fault)
        if m is not None and (w >> 7) & 31:
            assert p.rd == 7 and p.rd_value == m[1], (hex(w), p.rd_value, m)
        faults[p.fault] = faults.get(p.fault, 0) + 1
    assert faults == {0: 14, 11: 3}
    for t0 in (1 << 63, 1 << 62, 0x104, (1 << 63) | 0x8, 0x8, 0x38, 0xC3, 1 << 8):
        for avl in (0, 3, 1 << 32, (1 << 32) + 7, 1 << 20):
            regs[5], regs[6] = t0, avl
            p = P(_vsetvl(7, 6, 5), 0x1000, regs)
            m = _vset_word_model(_vsetvl(7, 6, 5), regs)
            assert p.fault == (11 if m is None else 0), (hex(t0), p.fault)
            if m is not None:
                assert p.rd == 7 and p.rd_value == m[1], (hex(t0), avl, p.rd_value, m)


VSET_WORDS = [_vsetvli(7, 6, 0x100), _vsetvli(7, 0, 0x004), _vsetvli(7, 6, 0x01D), _vsetvli(7, 6, 0x00D),
              _vsetivli(7, 31, 0x104), _vsetivli(7, 5, 0x016)]
VSETVL_T0 = [1 << 63, 1 << 62, 0x104]


def vset_program_source() -> str:
    """Illegal vset* requests (rd = t2 written 0, the start state kept), then
    an RVV op that is a no-op in the start state; each t2 printed."""
    L = ["    .text", "_start:", "    la    s2, out", "    mv    s3, s2", "    li    t1, 5"]
    for w in VSET_WORDS:
        L += ["    li    t2, -1", f"    .word {w:#x}", "    sd    t2, 0(s2)", "    addi  s2, s2, 8"]
    for t0 in VSETVL_T0:
        L += [f"    li    t0, {t0}", "    li    t2, -1", f"    .word {_vsetvl(7, 6, 5):#x}", "    sd    t2, 0(s2)",
              "    addi  s2, s2, 8"]
    L += ["    .word 0x02218057",                    # vadd.vv: a no-op at vl = 0
          "    li    a0, 1", "    mv    a1, s3", "    sub   a2, s2, s3", "    li    a7, 64", "    ecall",
          "    li    a0, 0", "    li    a7, 93", "    ecall", "    .bss", "    .balign 8", "out:", "    .zero 256"]
    return "\n".join(L) + "\n"


def vset_program_elf() -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(vset_program_source(), compress=False)


def vset_program_expected() -> bytes:
    return bytes(8 * (len(VSET_WORDS) + len(VSETVL_T0)))


def test_vset_program_on_oracle(oracle_mod):
    o = oracle_mod.Oracle(vset_program_elf(), "vset")
    g = o.run_golden()
    assert g.exit_code == 0 and o.golden_stdout() == vset_program_expected()


# vset* chains through legal configurations: (t0 = vsetvl's vtype, t1 = AVL, word)
VCFG_STEPS = [(0, 5, _vsetvli(7, 6, 0x000)),             # e8 m1, AVL 5 -> 5
              (0, 0, _vsetvli(7, 0, 0x009)),             # e16 m2, rd != 0, rs1 = 0 -> VLMAX 32
              (0, 0, _vsetvli(0, 0, 0x009)),             # the same vtype, x0, x0: vl kept
              (0, 0, _vsetvli(0, 0, 0x010)),             # e32 m1, x0, x0: vl = min(vl, VLMAX 8)
              (0, 0, _vsetvli(7, 0, 0x010)),             # -> VLMAX 8
              (0, 0, _vsetivli(7, 31, 0x01B)),           # e64 m8, uimm 31 -> 31
              (0xC2, (1 << 32) | 7, _vsetvl(7, 6, 5)),   # ta ma e8 m4, AVL truncated to uint32_t -> 7
              (0xC2, 1 << 40, _vsetvl(7, 6, 5)),         # the same vtype, AVL truncates to 0 -> 0
              (0, 1000, _vsetvli(7, 6, 0x005)),          # e8 mf8 -> VLMAX 4
              (0, 3, _vsetvli(7, 6, 0x01F)),             # e64 mf2: SEW > LMUL x ELEN -> vill, 0
              (0, 100, _vsetvli(7, 6, 0x003)),           # e8 m8 -> 100
              (0, 0, _vsetvli(0, 0, 0x00B)),             # e16 m8, x0, x0: vl = min(100, 128)
              (0, 300, _vsetivli(0, 17, 0x007)),         # e8 mf2, rd = 0: vl = 16 (not written)
              ((1 << 63) | 3, 50, _vsetvl(7, 6, 5)),     # vsetvl with vill set on a legal vtype8: VLMAX 0
              ((1 << 63) | 3, 9, _vsetvl(7, 6, 5)),      # the same (vill) vtype: no check, 0
              (0, 9, _vsetvli(7, 6, 0x000)),             # e8 m1 -> 9
              (0, 200, _vsetvli(7, 6, 0x0D1)),           # ta ma e16 m2 -> 32
              (0, 9, _vsetvli(7, 6, 0x100))]             # reserved bit: vill, vl 0 (the start state again)


def vcfg_program_source() -> str:
    """vset* chains through legal vector configurations (each rd printed, -1
    where rd = x0), then back to the start state and an RVV op that is a
    no-op there."""
    L = ["    .text", "_start:", "    la    s2, out", "    mv    s3, s2"]
    for t0, t1, w in VCFG_STEPS:
        L += [f"    li    t0, {t0 - (1 << 64) if t0 >> 63 else t0}", f"    li    t1, {t1}", "    li    t2, -1",
              f"    .word {w:#x}", "    sd    t2, 0(s2)", "    addi  s2, s2, 8"]
    L += ["    .word 0x02218057",                    # vadd.vv: a no-op in the start state
          "    li    a0, 1", "    mv    a1, s3", "    sub   a2, s2, s3", "    li    a7, 64", "    ecall",
          "    li    a0, 0", "    li    a7, 93", "    ecall", "    .bss", "    .balign 8", "out:", "    .zero 512"]
    return "\n".join(L) + "\n"


def vcfg_program_elf() -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(vcfg_program_source(), compress=False)


def vcfg_program_expected() -> bytes:
    vtype, vl, out = VILL, 0, b""
    for t0, t1, w in VCFG_STEPS:
        regs = [0] * 32
        regs[5], regs[6], regs[7] = t0, t1, (1 << 64) - 1
        vtype, vl = _vset_word_model(w, regs, vtype, vl)
        out += (vl if (w >> 7) & 31 else (1 << 64) - 1).to_bytes(8, "little")
    assert (vtype, vl) == (VILL, 0)
    return out


def test_vcfg_program_on_oracle(oracle_mod):
    exp = vcfg_program_expected()
    assert [int.from_bytes(exp[k:k + 8], "little") for k in range(0, len(exp), 8)][:9] == \
        [5, 32, (1 << 64) - 1, (1 << 64) - 1, 8, 31, 7, 0, 4]
    o = oracle_mod.Oracle(vcfg_program_elf(), "vcfg")
    g = o.run_golden()
    assert g.exit_code == 0 and o.golden_stdout() == exp


# ---------------------------------------------------------------- m5end program
# The simulator-control M5 ops under the stdlib run script's default exit
# handlers (oracle/rv64se.c OP_m5op; sim/pseudo_inst.cc:117-204,
# simulate/exit_handler.py:551-557): checkpoint and switchcpu continue with
# a0 = a1 = 0, the golden run ends at m5_fail(0, 0x307) -- "m5_fail
# instruction encountered", exit code 7 -- and three dead branches reach
# m5_quiesce (the only context suspends: a hang), m5_exit(0) (ends the run
# early, output unchanged, code 0: SDC) and m5_exit(100) (a delayed exit: not
# modelled, escape).  A flipped t0 / t1 / t2 takes a branch; a flipped a0
# before m5_fail delays it (escape); a flipped low byte of a1 changes the code
# (SDC), a high bit does not (masked).
M5END_CODE = 0x307


def _m5(fn):
    return f"    .word {(fn << 25) | 0x7B:#x}"


def m5end_program_source() -> str:
    L = ["    .text", "_start:", "    li    a0, 1", "    la    a1, msg", "    li    a2, 3", "    li    a7, 64", "    ecall",
         "    li    a0, -1", "    li    a1, -2", _m5(0x43), "    or    s4, a0, a1", "    li    a0, -1", "    li    a1, -2",
         _m5(0x52), "    or    s4, s4, a0", "    or    s4, s4, a1", "    bnez  s4, wrong",
         "    li    t0, 0", "    bnez  t0, quiesce", "    li    t1, 0", "    bnez  t1, early", "    li    t2, 0",
         "    bnez  t2, delayed", "    li    a0, 0", f"    li    a1, {M5END_CODE}", _m5(0x22),
         "wrong:", "    li    a0, 1", "    la    a1, msg", "    li    a2, 3", "    li    a7, 64", "    ecall",
         "    li    a0, 3", "    li    a7, 93", "    ecall",
         "quiesce:", _m5(0x01), "    j     wrong",
         "early:", "    li    a0, 0", _m5(0x21), "    j     wrong",
         "delayed:", "    li    a0, 100", _m5(0x21), "    j     wrong",
         "    .data", "msg:", "    .ascii \"hi\\n\""]
    return "\n".join(L) + "\n"


def m5end_program_elf() -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(m5end_program_source(), compress=False)


def test_m5end_program_on_oracle(oracle_mod):
    """Golden: ends at m5_fail with code 7 after printing "hi" once; trials on
    t0 / t1 / t2 / a0 / a1 reach every simulator-control outcome."""
    import numpy as np
    o = oracle_mod.Oracle(m5end_program_elf(), "m5end")
    g = o.run_golden()
    assert g.exit_code == M5END_CODE & 0xFF and o.golden_stdout() == b"hi\n", g
    from shrewd_amd.fi import SITE_DT
    n = g.ninst
    L = [(i, 1, reg) for reg in (5, 6, 7) for i in range(n)]
    L += [(n - 1, 1 << 3, 10), (n - 1, 1 << 1, 11), (n - 1, 1 << 9, 11)]
    sites = np.zeros(len(L), dtype=SITE_DT)
    for k, (i, mask, reg) in enumerate(L):
        sites[k] = (i, mask, 0, reg, k)
    r = o.run_trials(sites, protect_mask=0)
    got = {(int(c), int(s), int(x)) for c, s, x in zip(r["cls"], r["sub"], r["exit_code"])}
    assert (0, 2, 7) in got                   # masked: ended at m5_fail, code 7
    assert (3, 2, 0) in got                   # hang: m5_quiesce
    assert (1, 1, 0) in got                   # sdc: m5_exit(0) before the golden end, code 0
    assert (5, 1, 0) in got                   # escape/inst: m5_exit(100)
    last = [(int(c), int(s), int(x)) for c, s, x in zip(r["cls"][-3:], r["sub"][-3:], r["exit_code"][-3:])]
    assert last == [(5, 1, 0), (1, 2, 5), (0, 2, 7)], last


# ---------------------------------------------------------------- endkind programs
# The same output and exit code, reached by another end: the golden run ends
# with exit(0) (endkind_exit) or m5_exit(0) (endkind_m5); a dead branch on t0
# ends the other way after the same output.  A trial is masked only if it
# ends the way the golden run did (an exit syscall's "exiting with last
# active thread context" vs "m5_exit instruction encountered",
# syscall_emul.cc:120-248, sim/pseudo_inst.cc:178): otherwise SDC, with the
# trial's own end sub-code.  (No reference fixture decides this: parity
# unpinned.)
def endkind_program_source(golden_m5: bool) -> str:
    m5_end = ["    li    a0, 0", _m5(0x21)]
    exit_end = ["    li    a0, 0", "    li    a7, 93", "    ecall"]
    L = ["    .text", "_start:", "    li    a0, 1", "    la    a1, msg", "    li    a2, 3", "    li    a7, 64", "    ecall",
         "    li    t0, 0", "    bnez  t0, other"]
    L += m5_end if golden_m5 else exit_end
    L += ["other:"] + (exit_end if golden_m5 else m5_end)
    L += ["    .data", "msg:", "    .ascii \"hi\\n\""]
    return "\n".join(L) + "\n"


def endkind_program_elf(golden_m5: bool) -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(endkind_program_source(golden_m5), compress=False)


def endkind_sites():
    import numpy as np
    from shrewd_amd.fi import SITE_DT
    L = [(i, 1 << b, 0, 5, 0) for i in range(8) for b in (0, 7, 40)]
    s = np.array(L, dtype=SITE_DT)
    s["trial"] = np.arange(len(s))
    return s


@pytest.mark.parametrize("golden_m5", [False, True])
def test_endkind_program_on_oracle(oracle_mod, golden_m5):
    o = oracle_mod.Oracle(endkind_program_elf(golden_m5), "endkind")
    g = o.run_golden()
    assert g.exit_code == 0 and o.golden_stdout() == b"hi\n"
    r = o.run_trials(endkind_sites(), protect_mask=0)
    got = {(int(c), int(s), int(x)) for c, s, x in zip(r["cls"], r["sub"], r["exit_code"])}
    gsub, osub = (1, 0) if golden_m5 else (0, 1)
    assert (0, gsub, 0) in got           # masked: t0 flipped after its last use, the golden end
    assert (1, osub, 0) in got           # the other end, same output and code: SDC
    assert got <= {(0, gsub, 0), (1, osub, 0)}, got


# ---------------------------------------------------------------- sys2 program
# read (63), readlinkat (78) and riscv_hwprobe (258) (oracle/rv64se.c:
# sys_readlinkat / sys_hwprobe; se_workload.cc:221-527, syscall_emul.hh:
# 1066-1129,2798-2822): every result a0 and every buffer is printed.
SYS2_EXE = "/opt/workloads/sys2.riscv"
HW_IMA = ((1 << 0) | (1 << 1) | (1 << 2) | (0x3FFF << 3) | (1 << 28) | (1 << 29) | (1 << 31) | (1 << 32) | (1 << 33) |
          (1 << 36) | (1 << 42) | (1 << 45) | (1 << 46) | (1 << 47))


def sys2_program_source() -> str:
    def call(num, *args):
        out = [f"    li    a{k}, {v}" if isinstance(v, int) else f"    la    a{k}, {v}" for k, v in enumerate(args)]
        return out + [f"    li    a7, {num}", "    ecall", "    sd    a0, 0(s2)", "    addi  s2, s2, 8"]
    L = ["    .text", "_start:", "    la    s2, out", "    mv    s3, s2"]
    L += call(63, 5, "buf", 8)                          # read: fd 5 has no entry -> -EBADF
    L += call(57, 0)                                    # close(0), then read(0) -> -EBADF
    L += call(63, 0, "buf", 8)
    L += call(78, -100, "exe", "buf", 64)              # /proc/self/exe -> the path, NUL-padded to 64
    L += call(78, -100, "exe", "buf2", 5)              # truncated to bufsiz
    L += call(78, 7, "rel", "buf3", 16)                # relative path, dirfd 7: -EBADF
    L += call(78, -100, 0x10, "buf3", 16)              # unmapped path: -EFAULT
    # hwprobe, get values for keys 0..10 on all CPUs
    L += ["    la    t0, pairs"] + [f"    li    t1, {k}\n    sd    t1, {16 * k}(t0)" for k in range(11)]
    L += call(258, "pairs", 11, 0, 0, 0)
    L += call(258, "pairs", 1, 4, "mask", 0)            # cpusetsize 4: -EINVAL
    L += call(258, "pairs", 1, 8, "mask", 2)            # unknown flags: -EINVAL
    L += call(258, "pairs", 2, 16, "mask", 0)           # cpusetsize clamped to 8, CPU 0 set
    # which-cpus with a one-byte mask: pair {IMAExt0, FD|C} holds on CPU 0; then an unknown key
    L += ["    la    t0, pq", "    li    t1, 4", "    sd    t1, 0(t0)", "    li    t1, 3", "    sd    t1, 8(t0)",
          "    li    t1, 3", "    sd    t1, 16(t0)", "    li    t1, 2", "    sd    t1, 24(t0)",
          "    li    t1, 77", "    sd    t1, 32(t0)"]
    L += call(258, "pq", 2, 1, "mask1", 1)
    L += call(258, "pq", 3, 1, "mask1", 1)
    L += ["    li    a0, 1", "    mv    a1, s3", "    la    a2, end", "    sub   a2, a2, s3", "    li    a7, 64",
          "    ecall", "    li    a0, 0", "    li    a7, 93", "    ecall",
          "    .data", "    .balign 8", "exe:", '    .asciz "/proc/self/exe"', "rel:", '    .asciz "x/y"',
          "    .balign 8", "mask:", "    .dword 1", "    .dword 0", "mask1:", "    .dword 0x0101",
          "    .bss", "    .balign 8", "out:", "    .zero 128", "buf:", "    .zero 64", "buf2:", "    .zero 8",
          "buf3:", "    .zero 16", "pairs:", "    .zero 176", "pq:", "    .zero 48", "end:"]
    return "\n".join(L) + "\n"


def sys2_program_elf() -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(sys2_program_source(), compress=False)


def sys2_program_expected() -> bytes:
    """The output from the reference's handlers, restated by hand."""
    M = (1 << 64) - 1
    exe = SYS2_EXE.encode()
    res = [-9, 0, -9, len(exe), 5, -9, -14, 0, -22, -22, 0, 0, 0]
    out = b"".join((v & M).to_bytes(8, "little") for v in res)
    out += bytes(128 - len(out))
    out += exe + bytes(64 - len(exe))                           # buf
    out += exe[:5] + bytes(3)                                   # buf2
    out += bytes(16)                                            # buf3
    vals = {0: 0, 1: 0, 2: 0, 3: 1, 4: HW_IMA, 5: 2, 6: 64, 7: 0x4000000000000000, 9: 2}
    pairs = b""
    for k in range(11):   # the third call rewrote pairs 0, 1 once more (same answers)
        key = k if k in vals else -1
        pairs += (key & M).to_bytes(8, "little") + vals.get(k, 0).to_bytes(8, "little")
    out += pairs
    # pq after the which-cpus calls: unchanged, then the unknown key's pair set to {-1, 0}
    pq = [4, 3, 3, 2, M, 0]
    out += b"".join(v.to_bytes(8, "little") for v in pq)
    return out


def test_sys2_program_on_oracle(oracle_mod):
    o = oracle_mod.Oracle(sys2_program_elf(), "sys2")
    o.set_exe_path(SYS2_EXE)
    g = o.run_golden()
    assert g.exit_code == 0, g
    got, exp = o.golden_stdout(), sys2_program_expected()
    assert len(got) == len(exp), (len(got), len(exp))
    for k in range(0, len(exp), 8):
        assert got[k:k + 8] == exp[k:k + 8], (k, got[k:k + 8].hex(), exp[k:k + 8].hex())


# ------------------------------------------------------------ runoff program
# Scan loops whose faulted trials run off their buffers (the run-off loop
# proofs of the clean translated body, fi_translate.cpp / fi_trial.hip
# loop_outcome): a forward byte scan of a .bss buffer (past its end: the page
# after .bss is outside every VMA -- a page-fault crash), a backward word scan
# with a table lookup per word (down through .data and the text, then below
# it), and a byte scan of the first brk page (past it: heap pages the fault
# handler maps, MemState::fixupFault -- the proof stays undecided there).
RUNOFF_BUF = 4096


def runoff_program_source() -> str:
    return f"""    .text
_start:
    la    s0, buf
    la    s4, table
    li    s6, 0
    li    t0, 0
    li    t1, {RUNOFF_BUF}
fill:
    add   t2, s0, t0
    andi  t3, t0, 255
    sb    t3, 0(t2)
    addi  t0, t0, 1
    bne   t0, t1, fill
    li    t0, 0
    li    t1, 64
tfill:
    slli  t2, t0, 3
    add   t2, t2, s4
    mul   t3, t0, t0
    sd    t3, 0(t2)
    addi  t0, t0, 1
    bne   t0, t1, tfill
    li    s5, 4
passA:
    mv    a0, s0
    li    t0, {RUNOFF_BUF}
    add   a1, s0, t0
    li    t4, 0
scanA:
    lbu   t1, 0(a0)
    add   t4, t4, t1
    addi  a0, a0, 1
    bne   a0, a1, scanA
    add   s6, s6, t4
    addi  s5, s5, -1
    bnez  s5, passA
    li    s5, 2
passB:
    li    t0, {RUNOFF_BUF - 4}
    add   a0, s0, t0
    addi  a1, s0, -4
    li    t4, 0
scanB:
    lw    t1, 0(a0)
    andi  t2, t1, 63
    slli  t2, t2, 3
    add   t2, t2, s4
    ld    t3, 0(t2)
    xor   t4, t4, t3
    addi  a0, a0, -4
    bne   a0, a1, scanB
    add   s6, s6, t4
    addi  s5, s5, -1
    bnez  s5, passB
    li    a0, 0
    li    a7, 214
    ecall
    mv    s7, a0
    li    t0, 0x10000
    add   a0, s7, t0
    li    a7, 214
    ecall
    li    t0, 0
    li    t1, 64
hfill:
    add   t2, s7, t0
    sb    t0, 0(t2)
    addi  t0, t0, 1
    bne   t0, t1, hfill
    li    s5, 8
passC:
    mv    a0, s7
    addi  a1, s7, 64
    li    t4, 0
scanC:
    lbu   t1, 0(a0)
    add   t4, t4, t1
    addi  a0, a0, 1
    bne   a0, a1, scanC
    add   s6, s6, t4
    addi  s5, s5, -1
    bnez  s5, passC
    la    a1, out
    sd    s6, 0(a1)
    li    a0, 1
    li    a2, 8
    li    a7, 64
    ecall
    li    a0, 0
    li    a7, 93
    ecall
    .bss
    .balign 8
out:
    .zero 8
table:
    .zero 512
buf:
    .zero {RUNOFF_BUF}
"""


def runoff_program_elf() -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(runoff_program_source(), compress=False)


def runoff_program_expected() -> bytes:
    M = (1 << 64) - 1
    buf = [i & 255 for i in range(RUNOFF_BUF)]
    table = [(i * i) & M for i in range(64)]
    s6 = 4 * sum(buf)
    words = [int.from_bytes(bytes(buf[k:k + 4]), "little") for k in range(0, RUNOFF_BUF, 4)]
    t4 = 0
    for w in reversed(words):
        w = w - (1 << 32) if w >> 31 else w   # lw sign-extends (andi 63 sees the low bits only)
        t4 ^= table[w & 63]
    s6 += 2 * t4
    s6 += 8 * sum(range(64))
    return (s6 & M).to_bytes(8, "little")


def runoff_sites(ninst, n=3000, seed=11):
    """Single-bit faults on the scan pointer (a0) and the scan end (a1)."""
    import numpy as np
    from oracle.pyoracle import SITE_DT
    r = np.random.default_rng(seed)
    s = np.zeros(n, SITE_DT)
    s["inst"] = r.integers(1, ninst, n)
    s["mask"] = np.uint64(1) << r.integers(0, 64, n).astype(np.uint64)
    s["target"] = r.choice([10, 11], n)
    s["trial"] = np.arange(n)
    return s


# ------------------------------------------------------------ storeoff program
# Store walks whose faulted trials run off their buffers (the run-off proofs'
# counter stores, round 6: fi_translate.cpp kind 2, fi_trial.hip loop_outcome):
# a forward byte store over a .bss buffer (past its end: outside every VMA, a
# page-fault crash -- mem_state.cc:387-447, sim/faults.cc:95-105), a backward
# read-modify-write word walk (down through .data into the text: a store walk
# that could rewrite code stays undecided and runs on), and a byte store over
# the first brk page (past it: heap pages the fault handler maps, undecided);
# then a word store and a byte load at a pointer that steps beside a separate
# down-counter (kinds 3 / 4: another induction register).
STOREOFF_BUF = 4096


def storeoff_program_source() -> str:
    return f"""    .text
_start:
    la    s0, buf
    li    s5, 3
    li    t4, 1
passA:
    mv    a0, s0
    li    t0, {STOREOFF_BUF}
    add   a1, s0, t0
storeA:
    sb    t4, 0(a0)
    addi  a0, a0, 1
    bne   a0, a1, storeA
    addi  t4, t4, 7
    addi  s5, s5, -1
    bnez  s5, passA
    li    s5, 2
passB:
    li    t0, {STOREOFF_BUF - 4}
    add   a0, s0, t0
    addi  a1, s0, -4
storeB:
    lw    t1, 0(a0)
    addi  t1, t1, 3
    sw    t1, 0(a0)
    addi  a0, a0, -4
    bne   a0, a1, storeB
    addi  s5, s5, -1
    bnez  s5, passB
    li    s1, {STOREOFF_BUF // 4}
    mv    t2, s0
    li    t4, 0x01020304
storeD:
    sw    t4, 0(t2)
    addi  t2, t2, 4
    addi  s1, s1, -1
    bnez  s1, storeD
    li    a0, 0
    li    a7, 214
    ecall
    mv    s7, a0
    li    t0, 0x10000
    add   a0, s7, t0
    li    a7, 214
    ecall
    li    s5, 4
passC:
    mv    a0, s7
    addi  a1, s7, 64
storeC:
    sb    s5, 0(a0)
    addi  a0, a0, 1
    bne   a0, a1, storeC
    addi  s5, s5, -1
    bnez  s5, passC
    li    s6, 0
    mv    t2, s0
    li    t1, {STOREOFF_BUF}
sum:
    lbu   t3, 0(t2)
    slli  s6, s6, 1
    xor   s6, s6, t3
    addi  t2, t2, 1
    addi  t1, t1, -1
    bnez  t1, sum
    li    t0, 0
    li    t1, 64
hsum:
    add   t2, s7, t0
    lbu   t3, 0(t2)
    add   s6, s6, t3
    addi  t0, t0, 1
    bne   t0, t1, hsum
    la    a1, out
    sd    s6, 0(a1)
    li    a0, 1
    li    a2, 8
    li    a7, 64
    ecall
    li    a0, 0
    li    a7, 93
    ecall
    .bss
    .balign 8
out:
    .zero 8
buf:
    .zero {STOREOFF_BUF}
"""


def storeoff_program_elf() -> bytes:
    from tools.rvasm.rvasm import assemble
    return assemble(storeoff_program_source(), compress=False)


def storeoff_program_expected() -> bytes:
    M = (1 << 64) - 1
    buf = bytearray([1 + 7 * 2] * STOREOFF_BUF)   # the third pass's byte
    for _ in range(2):                               # two read-modify-write passes, word by word
        for k in range(0, STOREOFF_BUF, 4):
            w = (int.from_bytes(buf[k:k + 4], "little") + 3) & 0xFFFFFFFF
            buf[k:k + 4] = w.to_bytes(4, "little")
    buf = bytearray(bytes([4, 3, 2, 1]) * (STOREOFF_BUF // 4))   # storeD: every word 0x01020304
    s6 = 0
    for b in buf:
        s6 = ((s6 << 1) ^ b) & M
    s6 = (s6 + 64 * 1) & M                           # the last heap pass stores 1
    return s6.to_bytes(8, "little")


def storeoff_sites(ninst, n=3000, seed=12):
    """Single-bit faults on the walks' pointers (a0, t2), ends (a1) and
    counters (s1, t1)."""
    import numpy as np
    from oracle.pyoracle import SITE_DT
    r = np.random.default_rng(seed)
    s = np.zeros(n, SITE_DT)
    s["inst"] = r.integers(1, ninst, n)
    s["mask"] = np.uint64(1) << r.integers(0, 64, n).astype(np.uint64)
    s["target"] = r.choice([10, 11, 9, 7, 6], n)
    s["trial"] = np.arange(n)
    return s


def test_storeoff_program_on_oracle(oracle_mod):
    o = oracle_mod.Oracle(storeoff_program_elf(), "storeoff")
    g = o.run_golden()
    assert g.exit_code == 0, g
    assert o.golden_stdout() == storeoff_program_expected()
    res = o.run_trials(storeoff_sites(g.ninst, 400), protect_mask=0)
    assert (res["cls"] == 2).sum() > 20 and (res["sub"][res["cls"] == 2] == 3).any()


def test_runoff_program_on_oracle(oracle_mod):
    o = oracle_mod.Oracle(runoff_program_elf(), "runoff")
    g = o.run_golden()
    assert g.exit_code == 0, g
    assert o.golden_stdout() == runoff_program_expected()
    res = o.run_trials(runoff_sites(g.ninst, 400), protect_mask=0)
    assert (res["cls"] == 2).sum() > 20 and (res["sub"][res["cls"] == 2] == 3).any()
