#!/usr/bin/env python3
"""rvasm -- a small RV64IMC assembler and static ELF64 writer.

There is no RISC-V cross toolchain in this image, so the
campaign workloads are hand-written assembly turned into static Linux ELFs by
this tool.  The ELF it writes is shaped like what gem5's loader expects:

* ``ELFOSABI_LINUX`` so gem5 picks the Linux SE workload
  (``src/base/loader/elf_object.cc:305-308`` in the reference);
* PT_LOAD segments whose ``p_paddr == p_vaddr`` -- gem5 loads segments at
  ``p_paddr`` (``elf_object.cc:383``);
* the first PT_LOAD starts at file offset 0 so the program-header table is
  inside the image and ``AT_PHDR`` is meaningful (``elf_object.cc:396-402``);
* bss is expressed as ``p_memsz > p_filesz`` (zero-filled by the loader,
  ``elf_object.cc:384-392``).

With ``compress=True`` (the default) every instruction whose operands fit a
compressed (RVC) encoding and that does not reference a label is emitted as a
16-bit instruction, mirroring what GNU as does for register/immediate forms.
Branches, jumps and label references stay 32-bit so sizes are known after one
pass.  The result is a realistic mix of 16- and 32-bit instructions, including
32-bit instructions at ``pc % 4 == 2`` (the decoder's straddle case).
"""
from __future__ import annotations

import re
import struct
import sys

REG_ALIASES = {
    "zero": 0, "ra": 1, "sp": 2, "gp": 3, "tp": 4, "t0": 5, "t1": 6, "t2": 7,
    "s0": 8, "fp": 8, "s1": 9, "a0": 10, "a1": 11, "a2": 12, "a3": 13,
    "a4": 14, "a5": 15, "a6": 16, "a7": 17, "s2": 18, "s3": 19, "s4": 20,
    "s5": 21, "s6": 22, "s7": 23, "s8": 24, "s9": 25, "s10": 26, "s11": 27,
    "t3": 28, "t4": 29, "t5": 30, "t6": 31,
}
for _i in range(32):
    REG_ALIASES[f"x{_i}"] = _i

FREG = {f"f{_i}": _i for _i in range(32)}
FREG.update({n: i for i, n in enumerate(
    ["ft0", "ft1", "ft2", "ft3", "ft4", "ft5", "ft6", "ft7", "fs0", "fs1", "fa0", "fa1", "fa2", "fa3", "fa4",
     "fa5", "fa6", "fa7", "fs2", "fs3", "fs4", "fs5", "fs6", "fs7", "fs8", "fs9", "fs10", "fs11", "ft8", "ft9",
     "ft10", "ft11"])})


def freg(tok: str) -> int:
    tok = tok.strip()
    if tok not in FREG:
        raise AsmError(f"bad FP register {tok!r}")
    return FREG[tok]


TEXT_BASE = 0x10000
PAGE = 0x1000


class AsmError(Exception):
    pass


def reg(tok: str) -> int:
    tok = tok.strip()
    if tok not in REG_ALIASES:
        raise AsmError(f"bad register {tok!r}")
    return REG_ALIASES[tok]


def sext(v: int, bits: int) -> int:
    v &= (1 << bits) - 1
    return v - (1 << bits) if v >> (bits - 1) else v


def fits(v: int, bits: int) -> bool:
    return -(1 << (bits - 1)) <= v < (1 << (bits - 1))


def fitsu(v: int, bits: int) -> bool:
    return 0 <= v < (1 << bits)


# ---------------------------------------------------------------- 32-bit encodings
def enc_r(op, f3, f7, rd, rs1, rs2):
    return (f7 << 25) | (rs2 << 20) | (rs1 << 15) | (f3 << 12) | (rd << 7) | op


def enc_i(op, f3, rd, rs1, imm):
    if not fits(imm, 12):
        raise AsmError(f"imm {imm} out of 12-bit range")
    return ((imm & 0xFFF) << 20) | (rs1 << 15) | (f3 << 12) | (rd << 7) | op


def enc_s(op, f3, rs1, rs2, imm):
    if not fits(imm, 12):
        raise AsmError(f"imm {imm} out of 12-bit range")
    imm &= 0xFFF
    return ((imm >> 5) << 25) | (rs2 << 20) | (rs1 << 15) | (f3 << 12) | ((imm & 31) << 7) | op


def enc_b(op, f3, rs1, rs2, off):
    if off & 1 or not fits(off, 13):
        raise AsmError(f"branch offset {off} invalid")
    o = off & 0x1FFF
    return (((o >> 12) & 1) << 31) | (((o >> 5) & 0x3F) << 25) | (rs2 << 20) | (rs1 << 15) | \
        (f3 << 12) | (((o >> 1) & 0xF) << 8) | (((o >> 11) & 1) << 7) | op


def enc_u(op, rd, imm20):
    return ((imm20 & 0xFFFFF) << 12) | (rd << 7) | op


def enc_j(op, rd, off):
    if off & 1 or not fits(off, 21):
        raise AsmError(f"jump offset {off} invalid")
    o = off & 0x1FFFFF
    return (((o >> 20) & 1) << 31) | (((o >> 1) & 0x3FF) << 21) | (((o >> 11) & 1) << 20) | \
        (((o >> 12) & 0xFF) << 12) | (rd << 7) | op


R_OPS = {  # name: (opcode, funct3, funct7)
    "add": (0x33, 0, 0x00), "sub": (0x33, 0, 0x20), "sll": (0x33, 1, 0), "slt": (0x33, 2, 0),
    "sltu": (0x33, 3, 0), "xor": (0x33, 4, 0), "srl": (0x33, 5, 0), "sra": (0x33, 5, 0x20),
    "or": (0x33, 6, 0), "and": (0x33, 7, 0),
    "mul": (0x33, 0, 1), "mulh": (0x33, 1, 1), "mulhsu": (0x33, 2, 1), "mulhu": (0x33, 3, 1),
    "div": (0x33, 4, 1), "divu": (0x33, 5, 1), "rem": (0x33, 6, 1), "remu": (0x33, 7, 1),
    "addw": (0x3B, 0, 0), "subw": (0x3B, 0, 0x20), "sllw": (0x3B, 1, 0), "srlw": (0x3B, 5, 0),
    "sraw": (0x3B, 5, 0x20), "mulw": (0x3B, 0, 1), "divw": (0x3B, 4, 1), "divuw": (0x3B, 5, 1),
    "remw": (0x3B, 6, 1), "remuw": (0x3B, 7, 1),
    # Zbb / Zba subset
    "andn": (0x33, 7, 0x20), "orn": (0x33, 6, 0x20), "xnor": (0x33, 4, 0x20),
    "min": (0x33, 4, 0x05), "minu": (0x33, 5, 0x05), "max": (0x33, 6, 0x05), "maxu": (0x33, 7, 0x05),
    "rol": (0x33, 1, 0x30), "ror": (0x33, 5, 0x30),
    "sh1add": (0x33, 2, 0x10), "sh2add": (0x33, 4, 0x10), "sh3add": (0x33, 6, 0x10),
}
I_OPS = {
    "addi": (0x13, 0), "slti": (0x13, 2), "sltiu": (0x13, 3), "xori": (0x13, 4),
    "ori": (0x13, 6), "andi": (0x13, 7), "addiw": (0x1B, 0), "jalr": (0x67, 0),
}
SHIFT_OPS = {  # name: (opcode, funct3, funct6/7 high bits, shamt bits)
    "slli": (0x13, 1, 0x00, 6), "srli": (0x13, 5, 0x00, 6), "srai": (0x13, 5, 0x10, 6),
    "slliw": (0x1B, 1, 0x00, 5), "srliw": (0x1B, 5, 0x00, 5), "sraiw": (0x1B, 5, 0x20, 5),
}
LOADS = {"lb": 0, "lh": 1, "lw": 2, "ld": 3, "lbu": 4, "lhu": 5, "lwu": 6}
STORES = {"sb": 0, "sh": 1, "sw": 2, "sd": 3}
BRANCHES = {"beq": 0, "bne": 1, "blt": 4, "bge": 5, "bltu": 6, "bgeu": 7}
# F/D/Zfh subset without rounding: loads/stores, moves, sign injection, classify
FLOADS = {"flh": 1, "flw": 2, "fld": 3}
FSTORES = {"fsh": 1, "fsw": 2, "fsd": 3}
F_RR = {  # name: (funct7, funct3) -- fd, fs1, fs2
    "fsgnj.s": (0x10, 0), "fsgnjn.s": (0x10, 1), "fsgnjx.s": (0x10, 2),
    "fsgnj.d": (0x11, 0), "fsgnjn.d": (0x11, 1), "fsgnjx.d": (0x11, 2),
    "fsgnj.h": (0x12, 0), "fsgnjn.h": (0x12, 1), "fsgnjx.h": (0x12, 2)}
F_TO_X = {"fmv.x.w": (0x70, 0), "fclass.s": (0x70, 1), "fmv.x.d": (0x71, 0), "fclass.d": (0x71, 1),
          "fmv.x.h": (0x72, 0), "fclass.h": (0x72, 1)}   # rd, fs1
X_TO_F = {"fmv.w.x": 0x78, "fmv.d.x": 0x79, "fmv.h.x": 0x7A}   # fd, rs1
# F/D/Zfh arithmetic: name -> (funct5, rs2 or None, operand kinds, rounding mode or fixed funct3)
#   kinds: "ff" fd,fs1,fs2  "f" fd,fs1  "xff" rd,fs1,fs2  "xf" rd,fs1  "fx" fd,rs1; rm None = optional
#   rounding-mode operand (default dyn), an int = fixed funct3
FP_FMT = {"s": 0, "d": 1, "h": 2}
FP_RM = {"rne": 0, "rtz": 1, "rdn": 2, "rup": 3, "rmm": 4, "dyn": 7}
F_ARITH = {}
for _f in FP_FMT:
    F_ARITH.update({f"fadd.{_f}": (0x00, None, "ff", None), f"fsub.{_f}": (0x01, None, "ff", None),
                    f"fmul.{_f}": (0x02, None, "ff", None), f"fdiv.{_f}": (0x03, None, "ff", None),
                    f"fsqrt.{_f}": (0x0B, 0, "f", None), f"fmin.{_f}": (0x05, None, "ff", 0),
                    f"fmax.{_f}": (0x05, None, "ff", 1),
                    f"fminm.{_f}": (0x05, None, "ff", 3 if _f == "h" else 2),
                    f"fmaxm.{_f}": (0x05, None, "ff", 4 if _f == "h" else 3),
                    f"fle.{_f}": (0x14, None, "xff", 0), f"flt.{_f}": (0x14, None, "xff", 1),
                    f"feq.{_f}": (0x14, None, "xff", 2), f"fleq.{_f}": (0x14, None, "xff", 4),
                    f"fltq.{_f}": (0x14, None, "xff", 5)})
    for _k, _n in (("w", 0), ("wu", 1), ("l", 2), ("lu", 3)):
        F_ARITH[f"fcvt.{_k}.{_f}"] = (0x18, _n, "xf", None)
        F_ARITH[f"fcvt.{_f}.{_k}"] = (0x1A, _n, "fx", None)
    for _g in FP_FMT:
        if _g != _f:
            F_ARITH[f"fcvt.{_f}.{_g}"] = (0x08, FP_FMT[_g], "f", None)
F_FMA = {"fmadd": 0x43, "fmsub": 0x47, "fnmsub": 0x4B, "fnmadd": 0x4F}
AMO_F5 = {"amoadd": 0x00, "amoswap": 0x01, "lr": 0x02, "sc": 0x03, "amoxor": 0x04, "amoor": 0x08, "amoand": 0x0C,
          "amomin": 0x10, "amomax": 0x14, "amominu": 0x18, "amomaxu": 0x1C}


def amo_parse(name):
    """amoadd.w / amoswap.d.aqrl / lr.w.aq -> (funct5, funct3, aq, rl) or None"""
    p = name.split(".")
    if len(p) < 2 or p[0] not in AMO_F5 or p[1] not in ("w", "d"):
        return None
    sfx = p[2] if len(p) > 2 else ""
    if sfx not in ("", "aq", "rl", "aqrl"):
        return None
    return AMO_F5[p[0]], 2 if p[1] == "w" else 3, int("aq" in sfx), int("rl" in sfx)


# ---------------------------------------------------------------- compressed encodings
def creg(r):
    return 8 <= r <= 15


def c_ci(f3, rd, imm6, op=1):
    imm6 &= 0x3F
    return (f3 << 13) | (((imm6 >> 5) & 1) << 12) | (rd << 7) | ((imm6 & 0x1F) << 2) | op


def try_compress(name, ops):
    """Return a 16-bit encoding for a fully-resolved instruction, or None."""
    if name == "addi":
        rd, rs1, imm = ops
        if rd == rs1 and rd != 0 and imm != 0 and fits(imm, 6):
            return c_ci(0, rd, imm)
        if rs1 == 0 and rd != 0 and fits(imm, 6):
            return c_ci(2, rd, imm)  # c.li
        if imm == 0 and rd != 0 and rs1 != 0:
            return (4 << 13) | (rd << 7) | (rs1 << 2) | 2  # c.mv
        if rd == 2 and rs1 == 2 and imm != 0 and imm % 16 == 0 and fits(imm, 10):
            i = imm & 0x3FF
            return (3 << 13) | (((i >> 9) & 1) << 12) | (2 << 7) | (((i >> 4) & 1) << 6) | \
                (((i >> 6) & 1) << 5) | (((i >> 7) & 3) << 3) | (((i >> 5) & 1) << 2) | 1
        if rs1 == 2 and creg(rd) and imm > 0 and imm % 4 == 0 and imm < 1024:
            i = imm
            return (0 << 13) | (((i >> 4) & 3) << 11) | (((i >> 6) & 0xF) << 7) | \
                (((i >> 2) & 1) << 6) | (((i >> 3) & 1) << 5) | ((rd - 8) << 2) | 0
        return None
    if name == "addiw":
        rd, rs1, imm = ops
        if rd == rs1 and rd != 0 and fits(imm, 6):
            return c_ci(1, rd, imm)
        return None
    if name == "lui":
        rd, imm20 = ops
        s = sext(imm20, 20)
        if rd not in (0, 2) and s != 0 and fits(s, 6):
            return c_ci(3, rd, s)
        return None
    if name in ("slli", "srli", "srai"):
        rd, rs1, sh = ops
        if sh == 0 or rd != rs1:
            return None
        if name == "slli" and rd != 0:
            return (0 << 13) | (((sh >> 5) & 1) << 12) | (rd << 7) | ((sh & 31) << 2) | 2
        if creg(rd):
            f2 = 0 if name == "srli" else 1
            if name == "slli":
                return None
            return (4 << 13) | (((sh >> 5) & 1) << 12) | (f2 << 10) | ((rd - 8) << 7) | ((sh & 31) << 2) | 1
        return None
    if name == "andi":
        rd, rs1, imm = ops
        if rd == rs1 and creg(rd) and fits(imm, 6):
            i = imm & 0x3F
            return (4 << 13) | (((i >> 5) & 1) << 12) | (2 << 10) | ((rd - 8) << 7) | ((i & 31) << 2) | 1
        return None
    if name == "add":
        rd, rs1, rs2 = ops
        if rd != 0 and rs2 != 0 and rd == rs1:
            return (4 << 13) | (1 << 12) | (rd << 7) | (rs2 << 2) | 2
        if rd != 0 and rs2 != 0 and rs1 == 0:
            return (4 << 13) | (rd << 7) | (rs2 << 2) | 2  # c.mv
        return None
    if name in ("sub", "xor", "or", "and", "subw", "addw"):
        rd, rs1, rs2 = ops
        if rd == rs1 and creg(rd) and creg(rs2):
            f = {"sub": (0, 0), "xor": (0, 1), "or": (0, 2), "and": (0, 3), "subw": (1, 0), "addw": (1, 1)}[name]
            return (4 << 13) | (f[0] << 12) | (3 << 10) | ((rd - 8) << 7) | (f[1] << 5) | ((rs2 - 8) << 2) | 1
        return None
    if name in ("ld", "lw", "sd", "sw"):
        r, off, base = ops
        is_d = name[1] == "d"
        if base == 2:
            if name in ("ld", "lw") and r == 0:
                return None
            if is_d and off % 8 == 0 and 0 <= off < 512:
                if name == "ld":
                    return (3 << 13) | (((off >> 5) & 1) << 12) | (r << 7) | (((off >> 3) & 3) << 5) | \
                        (((off >> 6) & 7) << 2) | 2
                return (7 << 13) | (((off >> 3) & 7) << 10) | (((off >> 6) & 7) << 7) | (r << 2) | 2
            if not is_d and off % 4 == 0 and 0 <= off < 256:
                if name == "lw":
                    return (2 << 13) | (((off >> 5) & 1) << 12) | (r << 7) | (((off >> 2) & 7) << 4) | \
                        (((off >> 6) & 3) << 2) | 2
                return (6 << 13) | (((off >> 2) & 0xF) << 9) | (((off >> 6) & 3) << 7) | (r << 2) | 2
            return None
        if creg(r) and creg(base):
            if is_d and off % 8 == 0 and 0 <= off < 256:
                f3 = 3 if name == "ld" else 7
                return (f3 << 13) | (((off >> 3) & 7) << 10) | ((base - 8) << 7) | (((off >> 6) & 3) << 5) | \
                    ((r - 8) << 2)
            if not is_d and off % 4 == 0 and 0 <= off < 128:
                f3 = 2 if name == "lw" else 6
                return (f3 << 13) | (((off >> 3) & 7) << 10) | ((base - 8) << 7) | (((off >> 2) & 1) << 6) | \
                    (((off >> 6) & 1) << 5) | ((r - 8) << 2)
        return None
    if name in ("fld", "fsd"):
        # c.fld / c.fsd / c.fldsp / c.fsdsp: the c.ld / c.sd layouts with funct3 1 / 5
        r, off, base = ops
        c = try_compress("ld" if name == "fld" else "sd", (max(r, 1) if base == 2 else r, off, base))
        if c is None:
            return None
        if base == 2 and name == "fld":
            c = (c & ~(0x1F << 7)) | (r << 7)
        return (c & 0x1FFF) | ((1 if name == "fld" else 5) << 13)
    if name == "jalr":
        rd, rs1, imm = ops
        if imm == 0 and rs1 != 0 and rd in (0, 1):
            return (4 << 13) | ((1 if rd == 1 else 0) << 12) | (rs1 << 7) | 2
        return None
    return None


# ---------------------------------------------------------------- parser
class Item:
    __slots__ = ("kind", "name", "args", "size", "addr", "section", "line")

    def __init__(self, kind, name, args, section, line):
        self.kind, self.name, self.args, self.section, self.line = kind, name, args, section, line
        self.size = 0
        self.addr = 0


_num_re = re.compile(r"^[-+]?(0x[0-9a-fA-F]+|0b[01]+|\d+)$")


def parse_int(tok):
    tok = tok.strip()
    if tok.startswith("'") and tok.endswith("'") and len(tok) == 3:
        return ord(tok[1])
    if not _num_re.match(tok):
        raise AsmError(f"not a number: {tok!r}")
    return int(tok, 0)


def split_args(s):
    out, depth, cur = [], 0, ""
    in_str = False
    for ch in s:
        if ch == '"':
            in_str = not in_str
        if ch == "," and depth == 0 and not in_str:
            out.append(cur.strip())
            cur = ""
            continue
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def parse_mem(tok):
    m = re.match(r"^(.*)\((\w+)\)$", tok.strip())
    if not m:
        raise AsmError(f"bad memory operand {tok!r}")
    off = m.group(1).strip() or "0"
    return off, reg(m.group(2))


def li_sequence(rd, val):
    """Expand `li rd, val` into base instructions (name, ops) deterministically."""
    val = sext(val, 64)
    if fits(val, 12):
        return [("addi", (rd, 0, val))]
    if fits(val, 32):
        lo = sext(val, 12)
        hi = ((val - lo) >> 12) & 0xFFFFF
        seq = [("lui", (rd, hi))]
        if lo:
            seq.append(("addiw", (rd, rd, lo)))
        return seq
    # 64-bit: recursive on upper part then shift/add (like GNU as)
    lo = sext(val, 12)
    hi = (val - lo) >> 12
    shift = 12
    while hi & 1 == 0 and shift < 63:
        hi >>= 1
        shift += 1
    seq = li_sequence(rd, hi)
    seq.append(("slli", (rd, rd, shift)))
    if lo:
        seq.append(("addi", (rd, rd, lo)))
    return seq


class Assembler:
    def __init__(self, compress=True):
        self.compress = compress
        self.items = {".text": [], ".data": [], ".bss": []}
        self.labels = {}
        self.entry_label = "_start"

    # --- pass 0: parse ----------------------------------------------------
    def parse(self, src: str):
        section = ".text"
        for lineno, raw in enumerate(src.splitlines(), 1):
            line = raw.split("#", 1)[0].strip()
            while line:
                m = re.match(r"^([A-Za-z_.][\w.]*):\s*(.*)$", line)
                if m:
                    self.items[section].append(Item("label", m.group(1), None, section, lineno))
                    line = m.group(2).strip()
                    continue
                break
            if not line:
                continue
            parts = line.split(None, 1)
            op = parts[0].lower()
            rest = parts[1] if len(parts) > 1 else ""
            if op in (".text", ".data", ".bss"):
                section = op
                continue
            if op == ".section":
                section = rest.split(",")[0].strip()
                continue
            if op in (".globl", ".global", ".type", ".size", ".option", ".file"):
                continue
            if op.startswith("."):
                self.items[section].append(Item("dir", op, rest, section, lineno))
            else:
                self.items[section].append(Item("ins", op, split_args(rest), section, lineno))

    # --- instruction expansion: returns list of (name, ops, label_refs) ----
    def expand(self, it):
        n, a = it.name, it.args
        if n == "nop":
            return [("addi", (0, 0, 0))]
        if n == "li":
            return li_sequence(reg(a[0]), parse_int(a[1]))
        if n == "mv":
            return [("addi", (reg(a[0]), reg(a[1]), 0))]
        if n == "not":
            return [("xori", (reg(a[0]), reg(a[1]), -1))]
        if n == "neg":
            return [("sub", (reg(a[0]), 0, reg(a[1])))]
        if n == "negw":
            return [("subw", (reg(a[0]), 0, reg(a[1])))]
        if n == "sext.w":
            return [("addiw", (reg(a[0]), reg(a[1]), 0))]
        if n == "seqz":
            return [("sltiu", (reg(a[0]), reg(a[1]), 1))]
        if n == "snez":
            return [("sltu", (reg(a[0]), 0, reg(a[1])))]
        if n == "ret":
            return [("jalr", (0, 1, 0))]
        if n == "jr":
            return [("jalr", (0, reg(a[0]), 0))]
        if n == "j":
            return [("jal", (0, ("label", a[0])))]
        if n == "call":
            return [("jal", (1, ("label", a[0])))]
        if n == "jal" and len(a) == 1:
            return [("jal", (1, ("label", a[0])))]
        if n == "jal":
            return [("jal", (reg(a[0]), ("label", a[1])))]
        if n == "la":
            return [("auipc", (reg(a[0]), ("pcrel_hi", a[1]))),
                    ("addi", (reg(a[0]), reg(a[0]), ("pcrel_lo", a[1], -4)))]
        if n in ("beqz", "bnez", "blez", "bgez", "bltz", "bgtz"):
            r = reg(a[0])
            m = {"beqz": ("beq", r, 0), "bnez": ("bne", r, 0), "blez": ("bge", 0, r),
                 "bgez": ("bge", r, 0), "bltz": ("blt", r, 0), "bgtz": ("blt", 0, r)}[n]
            return [(m[0], (m[1], m[2], ("label", a[1])))]
        if n in ("bgt", "ble", "bgtu", "bleu"):
            base = {"bgt": "blt", "ble": "bge", "bgtu": "bltu", "bleu": "bgeu"}[n]
            return [(base, (reg(a[1]), reg(a[0]), ("label", a[2])))]
        if n in BRANCHES:
            return [(n, (reg(a[0]), reg(a[1]), ("label", a[2])))]
        if n in R_OPS:
            return [(n, (reg(a[0]), reg(a[1]), reg(a[2])))]
        if n in SHIFT_OPS:
            return [(n, (reg(a[0]), reg(a[1]), parse_int(a[2])))]
        if n == "jalr":
            if len(a) == 1:
                return [("jalr", (1, reg(a[0]), 0))]
            if len(a) == 2:
                off, base = parse_mem(a[1])
                return [("jalr", (reg(a[0]), base, parse_int(off)))]
            return [("jalr", (reg(a[0]), reg(a[1]), parse_int(a[2])))]
        if n in I_OPS:
            return [(n, (reg(a[0]), reg(a[1]), parse_int(a[2])))]
        if n in LOADS or n in STORES:
            off, base = parse_mem(a[1])
            return [(n, (reg(a[0]), parse_int(off), base))]
        if n in ("lui", "auipc"):
            return [(n, (reg(a[0]), parse_int(a[1]) & 0xFFFFF))]
        if n in ("ecall", "ebreak", "fence", "fence.i"):
            return [(n, ())]
        if n in ("csrr",):
            return [("csrrs", (reg(a[0]), parse_int(a[1]), 0))]
        if n in ("csrrw", "csrrs", "csrrc"):
            return [(n, (reg(a[0]), parse_int(a[1]), reg(a[2])))]
        if n in ("csrrwi", "csrrsi", "csrrci"):
            return [(n, (reg(a[0]), parse_int(a[1]), parse_int(a[2]) & 31))]
        if n in F_ARITH:
            f5, rs2, kinds, rmf = F_ARITH[n]
            rd = reg(a[0]) if kinds[0] == "x" else freg(a[0])
            rs1 = reg(a[1]) if kinds == "fx" else freg(a[1])
            if kinds in ("ff", "xff"):
                rs2v, rest = freg(a[2]), a[3:]
            else:
                rs2v, rest = rs2, a[2:]
            f3 = rmf if isinstance(rmf, int) else FP_RM[rest[0]] if rest else 7
            return [(n, (rd, rs1, rs2v, f3))]
        if n.rsplit(".", 1)[0] in F_FMA and n.rsplit(".", 1)[-1] in FP_FMT:
            f3 = FP_RM[a[4]] if len(a) > 4 else 7
            return [(n, (freg(a[0]), freg(a[1]), freg(a[2]), freg(a[3]), f3))]
        if n == ".insn16" or n == ".insn32":
            return [(n, (parse_int(a[0]),))]
        if n in FLOADS or n in FSTORES:
            off, base = parse_mem(a[1])
            return [(n, (freg(a[0]), parse_int(off), base))]
        if n in F_RR:
            return [(n, (freg(a[0]), freg(a[1]), freg(a[2])))]
        if n in F_TO_X:
            return [(n, (reg(a[0]), freg(a[1])))]
        if n in X_TO_F:
            return [(n, (freg(a[0]), reg(a[1])))]
        if amo_parse(n) is not None:
            # amoadd.w rd, rs2, (rs1)   lr.w rd, (rs1)
            f5 = amo_parse(n)[0]
            if f5 == 0x02:
                _, base = parse_mem(a[1])
                return [(n, (reg(a[0]), 0, base))]
            _, base = parse_mem(a[2])
            return [(n, (reg(a[0]), reg(a[1]), base))]
        raise AsmError(f"line {it.line}: unknown instruction {n!r}")

    @staticmethod
    def has_label(ops):
        return any(isinstance(o, tuple) for o in ops)

    def inst_size(self, name, ops):
        if name == ".insn16":
            return 2
        if name == ".insn32":
            return 4
        if self.compress and not self.has_label(ops):
            if try_compress(name, ops) is not None:
                return 2
        return 4

    # --- pass 1: layout ---------------------------------------------------
    def layout(self):
        # ELF header (64) + 2 program headers (56 each) precede .text in page 0
        hdr = 64 + 2 * 56
        addr = TEXT_BASE + hdr
        self.text_start = addr
        for sec in (".text", ".data", ".bss"):
            if sec == ".data":
                self.text_end = addr
                addr = (addr + PAGE - 1) // PAGE * PAGE
                self.data_start = addr
            if sec == ".bss":
                self.data_end = addr
                self.bss_start = addr
            for it in self.items[sec]:
                if it.kind == "label":
                    if it.name in self.labels:
                        raise AsmError(f"duplicate label {it.name}")
                    self.labels[it.name] = addr
                    it.addr = addr
                    continue
                if it.kind == "dir":
                    it.addr = addr
                    it.size = self.dir_size(it, addr)
                    addr += it.size
                    continue
                exp = self.expand(it)
                it.addr = addr
                it.size = sum(self.inst_size(nm, ops) for nm, ops in exp)
                addr += it.size
        self.bss_end = addr

    def dir_size(self, it, addr):
        d, rest = it.name, it.args
        if d == ".align" or d == ".p2align":
            al = 1 << parse_int(rest.split(",")[0])
            return (-addr) % al
        if d == ".balign":
            al = parse_int(rest.split(",")[0])
            return (-addr) % al
        if d in (".space", ".zero", ".skip"):
            return parse_int(rest.split(",")[0])
        if d in (".ascii", ".asciz", ".string"):
            s = self.parse_str(rest)
            return len(s) + (0 if d == ".ascii" else 1)
        width = {".byte": 1, ".half": 2, ".short": 2, ".word": 4, ".long": 4, ".dword": 8, ".quad": 8}.get(d)
        if width:
            return width * len(split_args(rest))
        raise AsmError(f"line {it.line}: unknown directive {d}")

    @staticmethod
    def parse_str(rest):
        rest = rest.strip()
        if not (rest.startswith('"') and rest.endswith('"')):
            raise AsmError(f"bad string {rest!r}")
        return rest[1:-1].encode("latin-1").decode("unicode_escape").encode("latin-1")

    def value(self, expr):
        expr = expr.strip()
        m = re.match(r"^([A-Za-z_.][\w.]*)\s*([-+])\s*(.+)$", expr)
        if m and m.group(1) in self.labels:
            v = parse_int(m.group(3))
            return self.labels[m.group(1)] + (v if m.group(2) == "+" else -v)
        if expr in self.labels:
            return self.labels[expr]
        return parse_int(expr)

    # --- pass 2: encode ---------------------------------------------------
    def encode_inst(self, name, ops, pc):
        ops = list(ops)
        for i, o in enumerate(ops):
            if isinstance(o, tuple):
                kind = o[0]
                target = self.value(o[1])
                if kind == "label":
                    ops[i] = target - pc
                elif kind == "pcrel_hi":
                    off = target - pc
                    ops[i] = ((off + 0x800) >> 12) & 0xFFFFF
                elif kind == "pcrel_lo":
                    off = target - (pc + o[2])
                    ops[i] = sext(off, 12)
        if name == ".insn16":
            return struct.pack("<H", ops[0] & 0xFFFF)
        if name == ".insn32":
            return struct.pack("<I", ops[0] & 0xFFFFFFFF)
        if self.compress and self.inst_size(name, tuple(ops)) == 2 and not self.has_label(ops):
            pass
        c = try_compress(name, tuple(ops)) if self.compress else None
        if c is not None and self._was_compressed:
            return struct.pack("<H", c)
        if name in R_OPS:
            op, f3, f7 = R_OPS[name]
            w = enc_r(op, f3, f7, *ops)
        elif name in SHIFT_OPS:
            op, f3, hi, bits = SHIFT_OPS[name]
            rd, rs1, sh = ops
            if not fitsu(sh, bits):
                raise AsmError(f"shift amount {sh}")
            w = (hi << 26 if bits == 6 else hi << 25) | (sh << 20) | (rs1 << 15) | (f3 << 12) | (rd << 7) | op
        elif name in I_OPS:
            op, f3 = I_OPS[name]
            w = enc_i(op, f3, *ops)
        elif name in LOADS:
            rd, off, base = ops
            w = enc_i(0x03, LOADS[name], rd, base, off)
        elif name in STORES:
            rs2, off, base = ops
            w = enc_s(0x23, STORES[name], base, rs2, off)
        elif name in BRANCHES:
            w = enc_b(0x63, BRANCHES[name], *ops)
        elif name == "jal":
            w = enc_j(0x6F, ops[0], ops[1])
        elif name == "lui":
            w = enc_u(0x37, ops[0], ops[1])
        elif name == "auipc":
            w = enc_u(0x17, ops[0], ops[1])
        elif name == "ecall":
            w = 0x00000073
        elif name == "ebreak":
            w = 0x00100073
        elif name == "fence":
            w = 0x0FF0000F
        elif name == "fence.i":
            w = 0x0000100F
        elif name in FLOADS:
            fd, off, base = ops
            w = enc_i(0x07, FLOADS[name], fd, base, off)
        elif name in FSTORES:
            fs2, off, base = ops
            w = enc_s(0x27, FSTORES[name], base, fs2, off)
        elif name in F_RR:
            f7, f3 = F_RR[name]
            w = enc_r(0x53, f3, f7, *ops)
        elif name in F_TO_X:
            f7, f3 = F_TO_X[name]
            w = enc_r(0x53, f3, f7, ops[0], ops[1], 0)
        elif name in X_TO_F:
            w = enc_r(0x53, 0, X_TO_F[name], ops[0], ops[1], 0)
        elif amo_parse(name) is not None:
            f5, f3, aq, rl = amo_parse(name)
            rd, rs2, base = ops
            w = enc_r(0x2F, f3, (f5 << 2) | (aq << 1) | rl, rd, base, rs2)
        elif name in ("csrrw", "csrrs", "csrrc", "csrrwi", "csrrsi", "csrrci"):
            rd, csr, rs1 = ops
            f3 = {"csrrw": 1, "csrrs": 2, "csrrc": 3, "csrrwi": 5, "csrrsi": 6, "csrrci": 7}[name]
            w = (csr << 20) | (rs1 << 15) | (f3 << 12) | (rd << 7) | 0x73
        elif name in F_ARITH:
            f5 = F_ARITH[name][0]
            rd, rs1, rs2, f3 = ops
            # the format field: the destination's for fcvt.X.{w,..} and fcvt.X.Y, else the last suffix
            fmt = name.split(".")[1] if f5 in (0x08, 0x1A) else name.rsplit(".", 1)[1]
            w = enc_r(0x53, f3, (f5 << 2) | FP_FMT[fmt], rd, rs1, rs2)
        elif name.rsplit(".", 1)[0] in F_FMA:
            fd, fs1, fs2, fs3, f3 = ops
            w = (fs3 << 27) | (FP_FMT[name.rsplit(".", 1)[1]] << 25) | (fs2 << 20) | (fs1 << 15) | (f3 << 12) | \
                (fd << 7) | F_FMA[name.rsplit(".", 1)[0]]
        else:
            raise AsmError(f"cannot encode {name}")
        return struct.pack("<I", w)

    def emit_section(self, sec):
        out = bytearray()
        for it in self.items[sec]:
            if it.kind == "label":
                continue
            if it.kind == "dir":
                out += self.emit_dir(it)
                continue
            pc = it.addr
            for nm, ops in self.expand(it):
                self._was_compressed = self.compress and not self.has_label(ops) and \
                    try_compress(nm, ops) is not None
                b = self.encode_inst(nm, ops, pc)
                out += b
                pc += len(b)
            if pc - it.addr != it.size:
                raise AsmError(f"line {it.line}: size drift")
        return bytes(out)

    def emit_dir(self, it):
        d, rest = it.name, it.args
        if d in (".align", ".p2align", ".balign", ".space", ".zero", ".skip"):
            if it.section == ".text" and d in (".align", ".p2align", ".balign") and it.size:
                # pad code with c.nop / nop
                pad = bytearray()
                n = it.size
                while n >= 4 and not self.compress:
                    pad += struct.pack("<I", 0x00000013)
                    n -= 4
                while n >= 2:
                    pad += struct.pack("<H", 0x0001)
                    n -= 2
                return bytes(pad)
            return bytes(it.size)
        if d in (".ascii", ".asciz", ".string"):
            s = self.parse_str(rest)
            return s + (b"" if d == ".ascii" else b"\0")
        width = {".byte": 1, ".half": 2, ".short": 2, ".word": 4, ".long": 4, ".dword": 8, ".quad": 8}[d]
        out = b""
        for v in split_args(rest):
            out += (self.value(v) & ((1 << (8 * width)) - 1)).to_bytes(width, "little")
        return out

    def assemble(self, src):
        self.parse(src)
        self.layout()
        if self.items[".bss"] and any(it.kind == "ins" for it in self.items[".bss"]):
            raise AsmError("instructions in .bss")
        text = self.emit_section(".text")
        data = self.emit_section(".data")
        for it in self.items[".bss"]:
            if it.kind == "dir" and it.name not in (".space", ".zero", ".skip", ".align", ".p2align", ".balign"):
                raise AsmError(".bss may only hold .space/.zero/.align")
        entry = self.labels.get(self.entry_label, self.text_start)
        return write_elf(text, self.text_start, data, self.data_start,
                         self.bss_end - self.bss_start, entry)


def write_elf(text, text_vaddr, data, data_vaddr, bss_size, entry):
    """Static ELF64 RISC-V executable with two PT_LOAD segments and minimal sections."""
    ehsize, phentsize, shentsize = 64, 56, 64
    phnum = 2
    hdr_len = ehsize + phnum * phentsize
    assert text_vaddr == TEXT_BASE + hdr_len
    seg0 = bytearray(hdr_len) + text  # segment 0: headers + text, file offset 0
    data_off = (len(seg0) + PAGE - 1) // PAGE * PAGE
    body = bytearray(seg0)
    body += bytes(data_off - len(body))
    body += data
    # section headers: null, .text, .data, .bss, .shstrtab
    shstr = b"\0.text\0.data\0.bss\0.shstrtab\0"
    shstr_off = len(body)
    body += shstr
    while len(body) % 8:
        body += b"\0"
    shoff = len(body)
    shnum = 5

    def sh(name, typ, flags, addr, off, size, align):
        return struct.pack("<IIQQQQIIQQ", name, typ, flags, addr, off, size, 0, 0, align, 0)

    shdrs = sh(0, 0, 0, 0, 0, 0, 0)
    shdrs += sh(1, 1, 0x6, text_vaddr, hdr_len, len(text), 2)
    shdrs += sh(7, 1, 0x3, data_vaddr, data_off, len(data), 8)
    shdrs += sh(13, 8, 0x3, data_vaddr + len(data), data_off + len(data), bss_size, 8)
    shdrs += sh(18, 3, 0, 0, shstr_off, len(shstr), 1)
    body += shdrs

    e_ident = b"\x7fELF" + bytes([2, 1, 1, 3, 0]) + bytes(7)  # ELFCLASS64, LE, v1, ELFOSABI_LINUX
    ehdr = e_ident + struct.pack("<HHIQQQIHHHHHH", 2, 243, 1, entry, ehsize, shoff,
                                 0x1, ehsize, phentsize, phnum, shentsize, shnum, 4)
    ph0 = struct.pack("<IIQQQQQQ", 1, 5, 0, TEXT_BASE, TEXT_BASE, len(seg0), len(seg0), PAGE)
    ph1 = struct.pack("<IIQQQQQQ", 1, 6, data_off, data_vaddr, data_vaddr, len(data),
                      len(data) + bss_size, PAGE)
    body[0:hdr_len] = ehdr + ph0 + ph1
    return bytes(body)


def assemble(src: str, compress: bool = True) -> bytes:
    return Assembler(compress=compress).assemble(src)


def main(argv):
    import argparse
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("src")
    ap.add_argument("-o", "--output", required=True)
    ap.add_argument("--no-compress", action="store_true")
    a = ap.parse_args(argv)
    with open(a.src) as f:
        elf = assemble(f.read(), compress=not a.no_compress)
    with open(a.output, "wb") as f:
        f.write(elf)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
