"""Offline translation + hipRTC build + disassembly (no GPU).

python tools/jit_inspect.py gpurun_out/golden_crc32.npz [out.s]   # translate the saved golden inputs
python tools/jit_inspect.py gpurun_out/tx_crc32.inc [out.s]       # a saved body as is
Prints the kernel's resource use (VGPRs, SGPRs, spills, scratch)."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from shrewd_amd.fi import lib  # noqa: E402

L = lib()
L.fi_debug_jit_compile.argtypes = [C.c_char_p, C.c_char_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64),
                                   C.c_char_p, C.c_uint64]
src = sys.argv[1]
if src.endswith(".npz"):
    z = np.load(src)
    pre, tr = np.ascontiguousarray(z["pre"]), np.ascontiguousarray(z["trace"])
    n = C.c_uint64()
    L.fi_debug_translate(pre.ctypes.data, len(pre), int(z["text_lo"]), tr.ctypes.data, len(tr), None, 0, C.byref(n))
    buf = C.create_string_buffer(n.value + 1)
    L.fi_debug_translate(pre.ctypes.data, len(pre), int(z["text_lo"]), tr.ctypes.data, len(tr), buf, n.value + 1,
                         C.byref(n))
    body = buf.value
    open("/tmp/fi_jit_inspect.inc", "wb").write(body)
else:
    body = open(src, "rb").read()
n = C.c_uint64()
err = C.create_string_buffer(8192)
if L.fi_debug_jit_compile(body, b"gfx950", None, 0, C.byref(n), err, 8192):
    sys.exit("compile failed:\n" + err.value.decode())
buf = C.create_string_buffer(n.value)
L.fi_debug_jit_compile(body, b"gfx950", buf, n.value, C.byref(n), err, 8192)
co = "/tmp/fi_jit_inspect.co"
open(co, "wb").write(buf.raw[:n.value])
notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
# per kernel (each kernel's metadata block is sorted by key; .wavefront_size closes it)
keys = (".vgpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count", ".private_segment_fixed_size")
cur = {}
for line in notes.splitlines():
    t = line.strip().lstrip("- ")
    for key in keys:
        if t.startswith(key + ":"):
            cur[key] = t.split(":", 1)[1].strip()
    if t.startswith(".name:"):
        cur["name"] = t.split(":", 1)[1].strip()
    if t.startswith(".wavefront_size:"):   # the last key of a kernel's block
        print(cur.get("name"), " ".join(f"{k[1:]}={cur.get(k)}" for k in keys))
        cur = {}
if len(sys.argv) > 2:
    dis = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", co], capture_output=True, text=True).stdout
    open(sys.argv[2], "w").write(dis)
    print("disassembly ->", sys.argv[2])
