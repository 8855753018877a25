#!/usr/bin/env python3
"""gem5 OpClass of every instruction the engine executes, from the reference's
own ISA description.

Runs only in the build container.  It runs the reference's ISA parser over
src/arch/riscv/isa/main.isa (gen_decode_vectors.run_isa_parser) and reads the
generated decoder-ns.cc.inc as DATA: every StaticInst constructor names its
mnemonic and OpClass (`X::X(ExtMachInst machInst) : Base("mnem", machInst,
IntAluOp)`).  An AMO's destination register is written by its load micro-op
("amoadd_w[l]", MemReadOp; decoder.isa:2067 / amo.isa), so AMOs take that
micro-op's class.  The OpClass enum order is src/cpu/FuncUnit.py:43-125.

Outputs (inputs/outputs only, nothing from the reference's source text):
  tests/golden/opclass_rv64.json          {"enum": [...], "ops": {op: class}}
  shrewd_amd/csrc/gem5_opclass_table.h    X(op, enum value) rows for the
                                          device and the oracle

Usage: python tools/oracle/gen_opclass_table.py [--ref /root/reference] [--generated DIR]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
from gen_decode_vectors import run_isa_parser  # noqa: E402

# `[Outer::]Cls::Cls(ExtMachInst machInst[, ...]) : Base("mnem", machInst, XxxOp)`
# (the vector-configuration classes name it _machInst: formats/vector_conf.isa)
CTOR = re.compile(r'(\w+)::\1\(\s*ExtMachInst _?machInst[^)]*\)\s*:\s*[\w<>:, ]+?\(\s*"([^"]+)",\s*_?machInst,'
                  r'[^"]*?(No_OpClass|\w+?Op)\b')


def opclass_enum(ref: str) -> list[str]:
    s = open(os.path.join(ref, "src", "cpu", "FuncUnit.py")).read()
    vals = re.search(r"class OpClass\(Enum\):\s*vals = \[(.*?)\]", s, re.S).group(1)
    return re.findall(r'"(\w+)"', vals)


def engine_ops() -> list[str]:
    s = open(os.path.join(REPO, "shrewd_amd", "csrc", "hip", "rv64_isa.h")).read()
    body = s[s.index("#define FI_OPS(X)"):s.index("namespace fi")]
    return [n for n in re.findall(r"X\((\w+)\)", body) if n != "UNKNOWN" and not n.startswith("ESC_")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--generated", default=None, help="existing isa_parser output dir")
    ap.add_argument("--json", default=os.path.join(REPO, "tests", "golden", "opclass_rv64.json"))
    ap.add_argument("--header", default=os.path.join(REPO, "shrewd_amd", "csrc", "gem5_opclass_table.h"))
    a = ap.parse_args()
    gen = a.generated
    if not gen:
        gen = tempfile.mkdtemp(prefix="isagen_")
        run_isa_parser(a.ref, gen)
    src = open(os.path.join(gen, "decoder-ns.cc.inc")).read()
    by_mnem = {}
    for m in CTOR.finditer(src):
        mnem, cls = m.group(2), m.group(3)
        by_mnem.setdefault(mnem, cls if cls == "No_OpClass" else cls[:-2])
    enum = opclass_enum(a.ref)
    ops = {}
    fm, ik = ("s", "d", "h"), ("w", "wu", "l", "lu")
    # the engine's FP arithmetic ops stand for gem5's per-format (and Zfa
    # variant) classes; every member must carry the same OpClass
    groups = {op: [f"{op}_{f}" for f in fm] for op in ("fadd", "fsub", "fmul", "fdiv", "fsqrt", "fmadd", "fmsub",
                                                       "fnmsub", "fnmadd", "feq")}
    groups.update({"fmin": [f"fmin{v}_{f}" for v in ("", "m") for f in fm],
                   "fmax": [f"fmax{v}_{f}" for v in ("", "m") for f in fm],
                   "flt": [f"flt{v}_{f}" for v in ("", "q") for f in fm],
                   "fle": [f"fle{v}_{f}" for v in ("", "q") for f in fm],
                   "fcvt_f2i": [f"fcvt_{i}_{f}" for i in ik for f in fm],
                   "fcvt_i2f": [f"fcvt_{f}_{i}" for i in ik for f in fm],
                   "fcvt_f2f": [f"fcvt_{a}_{b}" for a in fm for b in fm if a != b],
                   # the privileged SYSTEM members that commit (the warn-only no-ops);
                   # the others raise IllegalInst before committing anything
                   "priv": ["sinval_vvma", "sfence_w_inval", "sfence_inval_ir", "hinval_vvma", "hinval_gvma"],
                   "cbo": [f"cbo_{k}" for k in ("inval", "clean", "flush", "zero")],
                   "m5op": ["M5Op"],
                   "fli": [f"fli_{f}" for f in fm],
                   "fround": [f"fround{x}_{f}" for x in ("", "nx") for f in fm],
                   "fcvtmod": ["fcvtmod_w_d"],
                   # RVV before any vset*: nothing commits a result (VectorNopMicroInst)
                   "vec": ["ecall"],
                   # vset* from the start state (vill, vl 0): SimdConfigOp
                   "vset": ["vsetvli", "vsetvl", "vsetivli"],
                   "crypto": [f"sha256{k}" for k in ("sum0", "sum1", "sig0", "sig1")] +
                             [f"sha512{k}" for k in ("sum0", "sum1", "sig0", "sig1")] +
                             ["sm3p0", "sm3p1", "aes64im", "aes64ks1i", "brev8", "sm4ed", "sm4ks", "aes64es",
                              "aes64esm", "aes64ds", "aes64dsm", "aes64ks2", "xperm4", "xperm8"]})
    for op in engine_ops():
        base = op.rstrip("_")
        if op in groups:
            classes = {by_mnem[n] for n in groups[op]}
            if len(classes) != 1:
                raise SystemExit(f"{op}: members of different classes {classes}")
            ops[op] = classes.pop()
            continue
        if op == "csr":        # CSR instructions (csrrw etc.) are No_OpClass; the engine never commits one
            cls = by_mnem["csrrw"]
        elif op.startswith("amo"):
            cls = by_mnem[base + "[l]"]
        else:
            cls = by_mnem.get(base) or by_mnem.get(base.replace("_", "."))
        if cls is None:
            raise SystemExit(f"no gem5 constructor for {op}")
        ops[op] = cls
    with open(a.json, "w") as f:
        json.dump({"enum": enum, "ops": ops}, f, indent=0, sort_keys=True)
    with open(a.header, "w") as f:
        f.write("// Generated by tools/oracle/gen_opclass_table.py from the reference's ISA\n"
                "// description (src/arch/riscv/isa/*.isa via the gem5 ISA parser) and\n"
                "// src/cpu/FuncUnit.py: the gem5 OpClass enum value of each executed op.\n"
                "#pragma once\n\n// X(op, OpClass enum value)\n#define FI_GEM5_OPCLASS(X) \\\n")
        for op, cls in ops.items():
            f.write(f"    X({op}, {enum.index(cls)}) /* {cls} */ \\\n")
        f.write("\n")
        for n in ("IntAlu", "IntMult", "IntDiv", "FloatAdd", "FloatMisc", "FloatSqrt", "MemRead", "MemWrite"):
            f.write(f"#define FI_OPC_{n.upper()} {enum.index(n)}\n")
        f.write("#define FI_OPC_COUNT %d\n" % len(enum))
    print(f"{len(ops)} ops -> {a.json}, {a.header}")


if __name__ == "__main__":
    main()
