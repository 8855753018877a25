#!/usr/bin/env python3
"""Derive the RV64 Linux SE syscall classification from the reference tree.

Runs only in the build container (reads /root/reference as text).  Writes
tests/golden/syscalls_rv64.json: {number: [name, category]} where category is
  "unimpl"  -- entry without a handler (unimplementedFunc -> fatal),
  "ignore"  -- ignoreFunc / ignoreWarnOnceFunc (returns 0),
  "impl:<handler>" -- a real handler.
Numbers absent from the table are fatal "out of range"
(src/sim/syscall_desc.hh:204-214).  Source: the syscallDescs64 table of
src/arch/riscv/linux/se_workload.cc (lines 529-895 in the pinned tree); of
each `#if defined(SYS_x)` pair the first branch is taken (Linux hosts).
"""
import json
import re
import sys

REF = "/root/reference/src/arch/riscv/linux/se_workload.cc"


def parse(path=REF):
    txt = open(path).read()
    start = txt.index("EmuLinux::syscallDescs64 = {")
    end = txt.index("};", start)
    body = txt[start:end].splitlines()[1:]
    out = {}
    skip = False
    for line in body:
        s = line.strip()
        if s.startswith("#if"):
            skip = False
            continue
        if s.startswith("#else"):
            skip = True
            continue
        if s.startswith("#endif"):
            skip = False
            continue
        if skip:
            continue
        m = re.match(r'\{\s*(\d+)\s*,\s*"([^"]*)"\s*(?:,\s*([^}]+?))?\s*\}', s)
        if not m:
            continue
        num, name, handler = int(m.group(1)), m.group(2), (m.group(3) or "").strip()
        if not handler:
            cat = "unimpl"
        elif handler in ("ignoreFunc", "ignoreWarnOnceFunc"):
            cat = "ignore"
        else:
            cat = "impl:" + re.sub(r"<.*>", "", handler)
        out[num] = [name, cat]
    return out


if __name__ == "__main__":
    tab = parse()
    dst = sys.argv[1] if len(sys.argv) > 1 else "tests/golden/syscalls_rv64.json"
    with open(dst, "w") as f:
        json.dump({str(k): v for k, v in sorted(tab.items())}, f, indent=0, sort_keys=False)
    print(f"{len(tab)} entries -> {dst}")
