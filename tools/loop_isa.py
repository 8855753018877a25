"""Print the innermost loop of a function in a disassembly that contains a
marker (an immediate such as a block's exit pc), with instruction counts by
kind -- for reading the code the translator's blocks compile to.

python tools/loop_isa.py DISASM.s FUNC_SUBSTR MARKER [BACKEDGE_REGEX]
(BACKEDGE_REGEX: the instruction before the loop's back edge, e.g. "s_cmp_eq_u64
s\\[66:67\\]"; default: the innermost loop around the marker)"""
import re
import sys

path, func, marker = sys.argv[1], sys.argv[2], sys.argv[3]
lines, inside = [], False
for ln in open(path):
    if re.match(r"^[0-9a-f]+ <", ln):
        inside = func in ln
        continue
    if inside and "//" in ln:
        m = re.search(r"// ([0-9A-F]{12}):", ln)
        if m:
            lines.append((int(m.group(1), 16), ln.split("//")[0].strip()))
addr = [a for a, t in lines]
mk = [a for a, t in lines if marker in t]
if not mk:
    sys.exit("marker not found")
best = None
want = re.compile(sys.argv[4]) if len(sys.argv) > 4 else None
prev = ""
for a, t in lines:
    p, prev = prev, t
    m = re.match(r"s_(cbranch_\w+|branch) (\d+)", t)
    if not m:
        continue
    off = int(m.group(2))
    if off >= 32768:
        off -= 65536
    tgt = a + 4 + 4 * off
    if want is not None and not want.search(p):
        continue
    if tgt <= a and (want is not None or any(tgt <= x <= a for x in mk)):
        if best is None or a - tgt < best[1] - best[0]:
            best = (tgt, a)
lo, hi = best
body = [(a, t) for a, t in lines if lo <= a <= hi]
kinds = {}
for a, t in body:
    op = t.split()[0]
    k = ("smem" if op.startswith("s_load") or op.startswith("s_buffer") else
         "branch" if op.startswith("s_cbranch") or op == "s_branch" else
         "wait" if op.startswith("s_waitcnt") else
         "salu" if op.startswith("s_") else
         "vmem" if op.startswith(("global_", "buffer_", "flat_")) else
         "lds" if op.startswith("ds_") else "valu")
    kinds[k] = kinds.get(k, 0) + 1
    print(f"{a:8x}  {t}")
print(kinds, "total", len(body))
