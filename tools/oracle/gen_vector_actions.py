#!/usr/bin/env python3
"""What each RVV instruction does in an SE process that has not executed a
vset* yet, read from the reference's generated ISA code.

Runs only in the build container, on the output of the reference's ISA parser
(gen_decode_vectors.run_isa_parser), read as DATA.  At process start the
decoder's vector state is vtype = 1 << 63 (vill, vtype8 = 0: SEW = 8,
LMUL = 1) and vl = 0 (src/arch/riscv/decoder.hh:68-69, pcstate.hh:69-70); it
changes only through vset* and the vl trim of a fault-only-first load.  For
every vector class the decode picks the SEW = 8 instantiation (or reaches
GEM5_UNREACHABLE when the class has none: undefined behaviour in gem5.opt),
the macro-op constructor builds its micro-ops for vl = 0, and the first
micro-op's execute() either is a VectorNopMicroInst (no architectural
effect) or starts with updateVPUStatus(check_vill = true) -> IllegalInstFault
("VILL is set", src/arch/riscv/isa.cc:1400-1402).

Actions (the `known` column of shrewd_amd/csrc/gem5_decode_table.h):
  2  no-op, one tick                 (micro_vl == 0 -> one VectorNopMicroInst)
  3  no-op, two ticks                (fault-only-first: + VlFFTrimVlMicroOp, which
                                      rewrites vl = 0; saturating: + VxsatMicroInst,
                                      which writes vxsat = 0)
  4  IllegalInstFault (VILL is set)  (first micro-op / non-split execute checks vill)
  5  undefined in gem5 (SEW = 8 decode reaches GEM5_UNREACHABLE) -> escape
  6  needs vector state -> escape    (vset*, whole-register load / store / move:
                                      check_vill = false, they move register data)
"""
from __future__ import annotations

import os
import re

NOP1, NOP2, ILLEGAL, UNDEF, VSTATE = 2, 3, 4, 5, 6
WHOLE_FMTS = ("VlWholeOp", "VsWholeOp", "VMvWholeFormat")
VSET = ("Vsetvli", "Vsetvl", "Vsetivli")


def _ctor(src: str, cls: str):
    m = re.search(r"\n(?:template<[^>]*>\n)?%s(?:<[^>]*>)?::%s\(ExtMachInst _machInst[^\n]*\n" % (cls, cls), src)
    if not m:
        return None
    return src[m.start():src.find("\n}\n", m.start()) + 3]


def _exec(ex: str, cls: str):
    m = re.search(r"\n\s*%s(?:<[^>]*>)?::execute\(ExecContext\s*\*\s*xc" % cls, ex)
    if not m:
        return None
    return ex[m.start():ex.find("\n    }\n", m.start())]


def _checks_vill_first(body: str) -> bool:
    """execute() begins (before any memory access or register write) with
    updateVPUStatus(..., check_vill = true)."""
    i = body.find("updateVPUStatus(")
    if i < 0:
        return False
    head = body[:i]
    if any(k in head for k in ("readMem", "writeMem", "setRegOperand", "setMiscReg", "pcState(")):
        return False
    return re.search(r"bool check_vill = true;", head) is not None


def vector_actions(generated: str, classes: dict[str, str], sew0: dict[str, bool]) -> dict[str, int]:
    """classes: vector class -> gem5 format name; sew0: class -> whether its
    decode has an SEW = 8 instantiation (False: GEM5_UNREACHABLE)."""
    src = open(os.path.join(generated, "decoder-ns.cc.inc")).read()
    ex = open(os.path.join(generated, "exec-ns.cc.inc")).read()
    out = {}
    for cls, fmt in classes.items():
        if cls in VSET or fmt in WHOLE_FMTS:
            out[cls] = VSTATE
            continue
        if not sew0.get(cls, True):
            out[cls] = UNDEF
            continue
        body = _ctor(src, cls)
        if body is None:
            raise SystemExit(f"{cls}: no constructor")
        if "VectorNonSplitInst(" in body or "microops" not in body:
            e = _exec(ex, cls)
            if e is None or not _checks_vill_first(e):
                raise SystemExit(f"{cls}: non-split execute does not start with the vill check")
            out[cls] = ILLEGAL
            continue
        nop = re.search(r"if \((?:micro_vl|this->vl) == 0\) \{\s*microop = new VectorNopMicroInst\(_machInst\);", body)
        els = re.search(r"if \(micro_vl == 0\) \{\s*microop = new VectorNopMicroInst\(_machInst\);\s*"
                        r"(?:this->microops.push_back\(microop\);\s*)?\} else \{", body)
        if els:   # every other micro-op is built in the else branch
            depth, i = 1, els.end()
            while depth:
                depth += {"{": 1, "}": -1}.get(body[i], 0)
                i += 1
            if "new " in body[i:]:
                raise SystemExit(f"{cls}: micro-ops after the vl == 0 branch")
            out[cls] = NOP1
            continue
        # the conditions of the top-level loops (brace depth 1 in the body)
        loops, depth = [], 0
        for i, ch in enumerate(body):
            if ch == "{":
                depth += 1
            elif ch == "}":
                depth -= 1
            elif depth == 1 and body.startswith("for (", i):
                loops.append(body[i:].split(";")[1])
        # counts that are 0 at vl = 0: ceil(vl / n)
        zero = set(re.findall(r"(\w+) = ceil\(\(float\) this->vl\s*/", body))
        def dead(c):   # a loop that runs no iteration at vl = 0 (micro_vl = 0)
            return ("micro_vl > 0" in c or re.search(r"< micro_vl\b", c) is not None or
                    "ceil((float) this->vl" in c or
                    any(re.search(r"< %s\b" % z, c) for z in zero))
        if nop and loops and all(dead(c) for c in loops):
            # micro-ops pushed unconditionally after the loop(s)
            tail = body[body.rfind("for ("):]
            tail = tail[tail.find("\n    }\n"):]
            extra = re.findall(r"new (\w+)\(", tail)
            ff = re.search(r'MacroInst\("[\w.]+", _machInst, SimdUnitStrideFaultOnlyFirstLoadOp', body) is not None
            if any(x not in ("VlFFTrimVlMicroOp", "VxsatMicroInst") for x in extra):
                raise SystemExit(f"{cls}: micro-ops after the loop: {extra}")
            # VxsatMicroInst (saturating ops) writes vxsat / vcsr bit 0 from the
            # macro-op's flag, false when no element was computed: no effect
            out[cls] = NOP2 if ((ff and "VlFFTrimVlMicroOp" in extra) or "VxsatMicroInst" in extra) else NOP1
            continue
        if loops and any(">= 0" in c for c in loops):
            first = re.search(r"new (\w+Micro)(?:<[^>]*>)?\(", body).group(1)
            e = _exec(ex, first)
            if e is None or not _checks_vill_first(e):
                raise SystemExit(f"{cls}: first micro-op {first} does not start with the vill check")
            out[cls] = ILLEGAL
            continue
        raise SystemExit(f"{cls}: unrecognised constructor")
    return out
