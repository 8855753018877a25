#!/usr/bin/env python3
"""Where one trial spends its instructions (oracle, CPU): pc histogram by
64-byte text line and the stores it makes into the text range.

python tools/trial_trace.py WORKLOAD SEED TRIAL [MAXPCS]"""
import ctypes as C
import os
import sys
from collections import Counter

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.pyoracle import OUTCOME_DT, Oracle  # noqa: E402

REGS_PC = ((1 << 32) - 2) | (1 << 32)
name, seed, tid = sys.argv[1], int(sys.argv[2], 0), int(sys.argv[3])
cap = int(sys.argv[4]) if len(sys.argv) > 4 else 4_000_000
o = Oracle(open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb").read(), name)
g = o.run_golden()
site = o.sample(seed, tid, 1, REGS_PC)
L = o.L
L.or_debug_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64,
                             C.POINTER(C.c_uint64), C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
pcs = np.zeros(cap, np.uint64)
wrs = np.zeros(1 << 20, np.uint64)
out = np.zeros(1, OUTCOME_DT)
pn, wn = C.c_uint64(), C.c_uint64()
L.or_debug_trace(o.h, site.ctypes.data, 0, out.ctypes.data, pcs.ctypes.data, cap, C.byref(pn), wrs.ctypes.data,
                 len(wrs), C.byref(wn))
n = min(pn.value, cap)
print("site", site[0], "outcome", out[0], "committed", pn.value, "text stores", wn.value)
lines = Counter((int(p) & ~63) for p in pcs[:n])
print("pc lines (top 12):", [(hex(a), c) for a, c in lines.most_common(12)])
odd = int((pcs[:n] & 1).sum())
print("odd-pc instructions:", odd)
w = wrs[:min(wn.value, len(wrs))]
if len(w):
    print("text store range:", hex(int(w.min())), hex(int(w.max())), "distinct 64B lines:",
          len(set(int(x) & ~63 for x in w)))
    first = int(np.argmax(pcs[:n] != pcs[:n]))  # placeholder
    print("text store lines:", sorted(hex(x) for x in set(int(x) & ~63 for x in w)))
    print("first stores:", [hex(int(x)) for x in w[:16]])
