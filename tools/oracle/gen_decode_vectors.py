#!/usr/bin/env python3
"""Golden decode vectors from the reference's own ISA description.

Runs only in the build container.  It runs the reference's ISA parser
(src/arch/isa_parser, a Python program shipped in /root/reference) over
src/arch/riscv/isa/main.isa into a scratch directory, then reads the generated
decode-method.cc.inc as DATA: a nested `switch (FIELD) { case V: ... return new
Class(machInst); }` tree.  Field positions come from
src/arch/riscv/isa/bitfields.isa and the ExtMachInst BitUnion of
src/arch/riscv/types.hh:57-184; the decoder context fields are fixed to the SE
defaults of this campaign (rv_type = RV64 = 1, RiscvISA.py:77; enable_zcd = 1,
RiscvISA.py:121).  Compressed instructions carry zero upper halves
(decoder.cc:93-99).

For every instruction word in the sample the tree is walked to its leaf class;
the fixture tests/golden/decode_rv64.npz stores (raw word, leaf index) plus the
leaf class / format names.  The sample is every 16-bit compressed encoding, a
set of words built to reach every leaf of the tree, and uniform random 32-bit
words.  Nothing from the reference travels with the fixture except these
input/output pairs.

Usage: python tools/oracle/gen_decode_vectors.py [--ref /root/reference]
                                                 [--generated DIR] [--out PATH]
"""
from __future__ import annotations

import argparse
import os
import random
import re
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

CONTEXT = {"rv_type": 1, "enable_zcd": 1}   # RV64, Zcd on (SE defaults)


def run_isa_parser(ref: str, outdir: str) -> str:
    """Run the reference ISA parser in a child interpreter; returns the path
    of decode-method.cc.inc."""
    code = (
        "import sys, os\n"
        f"ref = {ref!r}\n"
        "for p in ['src/arch', 'ext/ply', 'ext', 'build_tools', 'src/python']:\n"
        "    sys.path.insert(0, os.path.join(ref, p))\n"
        "from isa_parser import ISAParser\n"
        f"ISAParser({outdir!r}).parse_isa_desc(os.path.join(ref, 'src/arch/riscv/isa/main.isa'))\n")
    subprocess.run([sys.executable, "-c", code], check=True, cwd=outdir,
                   stdout=subprocess.DEVNULL)
    return os.path.join(outdir, "decode-method.cc.inc")


def parse_fields(ref: str) -> dict:
    """NAME -> ('bits', hi, lo) | ('ctx', name)."""
    emi = {}
    txt = open(os.path.join(ref, "src/arch/riscv/types.hh")).read()
    body = txt[txt.index("BitUnion64(ExtMachInst)"):txt.index("EndBitUnion(ExtMachInst)")]
    for m in re.finditer(r"Bitfield<\s*(\d+)(?:\s*,\s*(\d+))?\s*>\s*(\w+)\s*;", body):
        hi = int(m.group(1))
        lo = int(m.group(2)) if m.group(2) is not None else hi
        emi[m.group(3)] = (hi, lo)
    fields = {}
    for line in open(os.path.join(ref, "src/arch/riscv/isa/bitfields.isa")):
        m = re.match(r"\s*def bitfield\s+(\w+)\s+(.+?);", line)
        if not m:
            continue
        name, spec = m.group(1), m.group(2).strip()
        r = re.match(r"<\s*(\d+)\s*(?::\s*(\d+))?\s*>", spec)
        if r:
            hi = int(r.group(1))
            lo = int(r.group(2)) if r.group(2) is not None else hi
            fields[name] = ("bits", hi, lo)
        elif spec in CONTEXT:
            fields[name] = ("ctx", spec)
        elif spec in emi:
            hi, lo = emi[spec]
            fields[name] = ("bits", hi, lo)
        else:
            raise SystemExit(f"unresolved bitfield {name} -> {spec}")
    return fields


TOK = re.compile(r"switch\s*\(([^)]*)\)\s*\{|case\s+(0x[0-9a-fA-F]+|0b[01]+|\d+)\s*:|default\s*:|"
                 r"return\s+new\s+(\w+)|GEM5_UNREACHABLE|//\s*(\w+)::(\w+)|\{|\}")


def tokenize(src: str):
    toks = []
    for line in src.splitlines():
        s = line.strip()
        if s.startswith("//"):
            m = re.match(r"//\s*(\w+)::(\w+)", s)
            if m:
                toks.append(("fmt", m.group(1), m.group(2)))
            continue
        for m in TOK.finditer(s):
            t = m.group(0)
            if t.startswith("switch"):
                toks.append(("switch", m.group(1).strip()))
            elif t.startswith("case"):
                toks.append(("case", int(m.group(2), 0)))
            elif t.startswith("default"):
                toks.append(("default",))
            elif t.startswith("return"):
                toks.append(("ret", m.group(3)))
            elif t == "GEM5_UNREACHABLE":
                toks.append(("unreach",))
            elif t == "{":
                toks.append(("{",))
            elif t == "}":
                toks.append(("}",))
    return toks


class Parser:
    """switch := SWITCH '{' (label+ stmt)* '}' ; stmt := switch | ret | '{' stmt* '}'."""

    def __init__(self, toks):
        self.t = toks
        self.i = 0
        self.fmt = None

    def peek(self):
        while self.i < len(self.t) and self.t[self.i][0] == "fmt":
            self.fmt = self.t[self.i][1:]
            self.i += 1
        return self.t[self.i] if self.i < len(self.t) else ("eof",)

    def take(self):
        tok = self.peek()
        self.i += 1
        return tok

    def stmt(self):
        tok = self.peek()
        if tok[0] == "switch":
            return self.switch()
        if tok[0] == "ret":
            self.take()
            fmt = self.fmt or ("?", "?")
            return ("leaf", tok[1], fmt[0], fmt[1])
        if tok[0] == "{":
            self.take()
            node = None
            while self.peek()[0] != "}":
                n = self.stmt()
                node = node or n
            self.take()
            return node
        if tok[0] == "unreach":
            self.take()
            return None
        raise SyntaxError(f"unexpected {tok} at {self.i}")

    def switch(self):
        _, field = self.take()      # the token includes the opening brace
        cases, default = {}, None
        while True:
            tok = self.peek()
            if tok[0] == "}":
                self.take()
                break
            labels, is_default = [], False
            while self.peek()[0] in ("case", "default"):
                t = self.take()
                if t[0] == "case":
                    labels.append(t[1])
                else:
                    is_default = True
            body = self.stmt()
            # trailing statements of a case (break / UNREACHABLE) are not tokens
            while self.peek()[0] == "unreach":
                self.take()
            for v in labels:
                cases[v] = body
            if is_default:
                default = body
        return ("switch", field, cases, default)


def field_value(fields, name, word):
    if name.startswith("machInst."):
        return None      # vector context (vtype); all leaves below are vector classes
    f = fields[name]
    if f[0] == "ctx":
        return CONTEXT[f[1]]
    _, hi, lo = f
    return (word >> lo) & ((1 << (hi - lo + 1)) - 1)


def first_leaf(node):
    if node is None:
        return None
    if node[0] == "leaf":
        return node
    for v in node[2].values():
        leaf = first_leaf(v)
        if leaf:
            return leaf
    return first_leaf(node[3])


def walk(tree, fields, word):
    node = tree
    while node[0] == "switch":
        v = field_value(fields, node[1], word)
        if v is None:
            return first_leaf(node)
        nxt = node[2].get(v, node[3])
        if nxt is None:
            raise RuntimeError(f"fell off switch {node[1]}={v} for {word:#x}")
        node = nxt
    return node


def leaf_words(tree, fields, rng, per_leaf=6):
    """Random words that reach each leaf: collect path constraints and fill."""
    out = []

    def rec(node, cons):
        if node is None:
            return
        if node[0] == "leaf":
            for _ in range(per_leaf):
                for _try in range(64):
                    w = rng.getrandbits(32)
                    ok = True
                    for (name, val, excl) in cons:
                        f = fields.get(name)
                        if f is None or f[0] != "bits":
                            continue
                        _, hi, lo = f
                        m = ((1 << (hi - lo + 1)) - 1) << lo
                        if val is not None:
                            w = (w & ~m) | ((val << lo) & m)
                    for (name, val, excl) in cons:
                        f = fields.get(name)
                        if val is None and f is not None and f[0] == "bits":
                            if field_value(fields, name, w) in excl:
                                ok = False
                    if ok:
                        out.append(w)
                        break
            return
        _, name, cases, default = node
        if name.startswith("machInst."):
            return rec(first_leaf(node), cons)
        f = fields[name]
        for v, sub in cases.items():
            if f[0] == "ctx" and v != CONTEXT[f[1]]:
                continue
            rec(sub, cons + [(name, v, None)])
        if default is not None:
            rec(default, cons + [(name, None, set(cases))])

    rec(tree, [])
    return out


ESCAPE_OPCODES = (0x01, 0x09, 0x0b, 0x10, 0x11, 0x12, 0x13, 0x14, 0x15, 0x1c)


def flatten(node, fields, cons, out):
    """First-match (mask, match, known) patterns of a subtree: explicit cases
    precede the default branch at every switch, and a default leaf carries only
    the positive constraints of its path, so first match == tree walk."""
    if node is None:
        return
    if node[0] == "leaf":
        mask = match = 0
        for name, val in cons:
            _, hi, lo = fields[name]
            m = ((1 << (hi - lo + 1)) - 1) << lo
            mask |= m
            match |= (val << lo) & m
        out.append((mask, match, 0 if node[1] == "Unknown" else 1, node[1], node[2]))
        return
    _, name, cases, default = node
    if name.startswith("machInst."):
        # the SEW switch of a vector class: without an SEW = 8 case (vsew 0)
        # the decode of a process that has not run vset* is GEM5_UNREACHABLE
        if name == "machInst.vtype8.vsew":
            lf = first_leaf(node)
            SEW0[lf[1]] = 0 in cases
        leaves = []
        def collect(n):
            if n is None:
                return
            if n[0] == "leaf":
                leaves.append(n)
                return
            for v in n[2].values():
                collect(v)
            collect(n[3])
        collect(node)
        assert all(lf[1] != "Unknown" for lf in leaves)
        return flatten(leaves[0], fields, cons, out)
    f = fields[name]
    if f[0] == "ctx":
        return flatten(cases.get(CONTEXT[f[1]], default), fields, cons, out)
    for v, sub in cases.items():
        flatten(sub, fields, cons + [(name, v)], out)
    flatten(default, fields, cons, out)


SEW0: dict[str, bool] = {}


def emit_table(tree, fields, path, generated=None):
    """Known-vs-Unknown first-match table for the opcode groups the engine does
    not execute (FP, vector, AMO, SYSTEM privileged / hypervisor).  With the
    ISA parser's output (generated), vector classes carry their action in a
    process that has not run vset* (gen_vector_actions.py) instead of 1."""
    q3 = tree[2][3]
    assert q3[1] == "OPCODE5"
    rows = []
    index = []
    for op in ESCAPE_OPCODES:
        pats = []
        flatten(q3[2].get(op, q3[3]), fields, [], pats)
        # drop trailing Unknown patterns: no match means Unknown anyway
        while pats and pats[-1][2] == 0:
            pats.pop()
        index.append((op, len(rows), len(pats)))
        rows += pats
    if generated:
        from gen_vector_actions import vector_actions
        vec = {r[3]: r[4] for r in rows if r[2] and r[4].startswith("V")}
        act = vector_actions(generated, vec, SEW0)
        rows = [(m, v, act.get(c, k) if k else 0, c, f) for m, v, k, c, f in rows]
    with open(path, "w") as f:
        f.write("// GENERATED by tools/oracle/gen_decode_vectors.py --emit-table from the\n"
                "// reference's ISA description (src/arch/riscv/isa/decoder.isa via its\n"
                "// isa_parser; RV64, enable_zcd = 1).  Do not edit.\n"
                "//\n"
                "// For the major opcodes the engine does not execute (LOAD-FP/STORE-FP incl.\n"
                "// vector memory ops, AMO, FMADD..FNMADD, OP-FP, OP-V, SYSTEM) it tells an\n"
                "// encoding gem5 decodes to a real instruction (-> escape outcome) from one\n"
                "// it decodes to Unknown (-> illegal-instruction crash).  Rows are\n"
                "// first-match (mask, match, known) patterns grouped per opcode5.\n"
                "// known: 0 Unknown, 1 known; vector classes: what they do before any\n"
                "// vset* (tools/oracle/gen_vector_actions.py): 2 no-op (one tick), 3 no-op\n"
                "// (two ticks), 4 IllegalInst (vill), 5 undefined in gem5 (escape), 6 needs\n"
                "// vector state (escape).\n"
                "#pragma once\n\n")
        f.write(f"#define FI_GEM5_DEC_ROWS {len(rows)}\n")
        f.write("// X(mask, match, known)\n#define FI_GEM5_DEC_TABLE(X) \\\n")
        for mask, match, known, cls, _ in rows:
            f.write(f"    X(0x{mask:08x}u, 0x{match:08x}u, {known}) /* {cls} */ \\\n")
        f.write("\n// X(opcode5, first row, row count)\n#define FI_GEM5_DEC_INDEX(X) \\\n")
        for op, first, cnt in index:
            f.write(f"    X(0x{op:02x}, {first}, {cnt}) \\\n")
        f.write("\n")
    print(f"{len(rows)} rows -> {path}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--generated", default=None, help="existing isa_parser output dir")
    ap.add_argument("--out", default=os.path.join(REPO, "tests", "golden", "decode_rv64.npz"))
    ap.add_argument("--random", type=int, default=200_000)
    ap.add_argument("--seed", type=int, default=20251031)
    ap.add_argument("--emit-table", default=os.path.join(REPO, "shrewd_amd", "csrc", "gem5_decode_table.h"))
    a = ap.parse_args()

    if a.generated:
        path = os.path.join(a.generated, "decode-method.cc.inc")
    else:
        tmp = tempfile.mkdtemp(prefix="isagen_")
        path = run_isa_parser(a.ref, tmp)
    fields = parse_fields(a.ref)
    src = open(path).read()
    src = src[src.index("decodeInst"):]
    p = Parser(tokenize(src))
    while p.peek()[0] != "switch":
        p.take()
    tree = p.switch()

    if a.emit_table:
        emit_table(tree, fields, a.emit_table, os.path.dirname(path))

    rng = random.Random(a.seed)
    words = [w for w in range(1 << 16) if (w & 3) != 3]
    words += [w | 3 for w in leaf_words(tree, fields, rng)]
    words += [rng.getrandbits(32) | 3 for _ in range(a.random)]
    words = sorted(set(words))

    names, index, out = [], {}, []
    for w in words:
        leaf = walk(tree, fields, w)
        key = (leaf[1], leaf[2], leaf[3])
        if key not in index:
            index[key] = len(names)
            names.append(key)
        out.append(index[key])
    np.savez_compressed(
        a.out,
        raw=np.asarray(words, dtype=np.uint32),
        leaf=np.asarray(out, dtype=np.uint16),
        cls=np.asarray([k[0] for k in names]),
        fmt=np.asarray([k[1] for k in names]),
        mnem=np.asarray([k[2] for k in names]))
    print(f"{len(words)} words, {len(names)} leaf classes -> {a.out}")


if __name__ == "__main__":
    main()
