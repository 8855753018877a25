#!/usr/bin/env python3
"""Zfa fli constants as the reference's decoder lists them.

Runs only in the build container: reads the fli_s / fli_d / fli_h tables of
src/arch/riscv/isa/decoder.isa as DATA (index -> bit pattern; defaultNaN*UI
is the canonical NaN of ext/softfloat/RISCV/specialize.h) and writes them as
a fixture: tests/golden/fli_rv64.json {"h": [32 ints], "s": [...], "d": [...]}.

Usage: python tools/oracle/gen_fli_table.py [--ref /root/reference]
"""
import argparse
import json
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
NAN = {"defaultNaNF16UI": 0x7E00, "defaultNaNF32UI": 0x7FC00000, "defaultNaNF64UI": 0x7FF8000000000000}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(REPO, "tests", "golden", "fli_rv64.json"))
    a = ap.parse_args()
    src = open(os.path.join(a.ref, "src", "arch", "riscv", "isa", "decoder.isa")).read()
    out = {}
    for f in ("s", "d", "h"):
        body = src[src.index(f"fli_{f}({{{{"):]
        body = body[:body.index("};")]
        vals = {}
        for idx, val in re.findall(r"\[0b([01]{5})\]\s*=\s*(\w+)", body):
            vals[int(idx, 2)] = NAN[val] if val in NAN else int(val.rstrip("ul").rstrip("UL"), 16)
        assert sorted(vals) == list(range(32)), f
        out[f] = [vals[i] for i in range(32)]
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=0)
    print(f"fli tables -> {a.out}")


if __name__ == "__main__":
    main()
