#!/usr/bin/env python3
"""Indices of the RISC-V misc registers a SE checkpoint's
[<cpu>.isa] miscRegFile array holds (ISA::serialize, src/arch/riscv/isa.cc:
977-983: SERIALIZE_CONTAINER(miscRegFile), NUM_PHYS_MISCREGS entries in
MiscRegIndex order, src/arch/riscv/regs/misc.hh).  Reads the enum as data and
writes tests/golden/riscv_miscreg.json (the fixture the checkpoint reader's
constants are tested against).

python tools/oracle/gen_miscreg_index.py [/root/reference]"""
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
src = open(os.path.join(ref, "src/arch/riscv/regs/misc.hh")).read()
body = src[src.index("enum MiscRegIndex"):]
body = body[body.index("{") + 1:body.index("};")]
names = []
for line in body.splitlines():
    line = line.split("//")[0].strip()
    for tok in filter(None, (t.strip() for t in line.split(","))):
        m = re.match(r"(MISCREG_\w+|NUM_\w+)\s*(=\s*(\w+))?$", tok)
        if not m:
            continue
        if m.group(3) and not m.group(3).isdigit():
            continue   # an alias (MISCREG_FFLAGS_EXE = NUM_PHYS_MISCREGS)
        names.append(m.group(1))
idx = {n: i for i, n in enumerate(names)}
keep = ["MISCREG_FFLAGS", "MISCREG_FRM", "MISCREG_VL", "MISCREG_VTYPE", "MISCREG_VSTART", "MISCREG_VXSAT",
        "MISCREG_VXRM", "NUM_PHYS_MISCREGS"]
out = {k: idx[k] for k in keep}
out["source"] = "src/arch/riscv/regs/misc.hh enum MiscRegIndex (tools/oracle/gen_miscreg_index.py)"
with open(os.path.join(ROOT, "tests", "golden", "riscv_miscreg.json"), "w") as f:
    json.dump(out, f, indent=1)
print(out)
