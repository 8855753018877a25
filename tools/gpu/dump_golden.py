"""Dump each workload's pre-decoded text and golden trace (the translator's
inputs) to gpurun_out/golden_NAME.npz, for offline work on the translator
(tools/jit_inspect.py).  python tools/gpu/dump_golden.py [NAME ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from shrewd_amd import Engine  # noqa: E402

os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
for name in sys.argv[1:] or ["hello", "crc32", "qsort", "intmix", "fpamo"]:
    e = Engine()
    e.load_elf(open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb").read(), [name])
    e.golden_run()
    pre, tr, lo = e.debug_golden_trace()
    np.savez(os.path.join(ROOT, "gpurun_out", f"golden_{name}.npz"), pre=pre, trace=tr, text_lo=np.uint64(lo))
    print(name, len(pre), len(tr), e.translate_status()[:100], flush=True)
    e.close()
