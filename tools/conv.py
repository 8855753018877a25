"""One converged 64-lane wave running the golden path from process start
(no faults): the per-instruction cost of the interpreter or translated path.
python tools/conv.py [workload] [--interp]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shrewd_amd import Engine  # noqa: E402
from shrewd_amd.fi import CFG_NO_SNAPSHOT_START, CFG_NO_TRANSLATE  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("workload", nargs="?", default="crc32")
ap.add_argument("--interp", action="store_true")
ap.add_argument("--waves", type=int, default=1)
a = ap.parse_args()
fl = CFG_NO_SNAPSHOT_START | (CFG_NO_TRANSLATE if a.interp else 0)
e = Engine(max_trials_per_launch=65536, flags=fl)
e.load_elf(open(f"workloads/{a.workload}.elf", "rb").read(), [a.workload])
g = e.golden_run()
e.set_campaign(0x5EED0002, ((1 << 32) - 2) | (1 << 32), 1)
s = e.sample(0, 64 * a.waves)
s["inst"] = 1 << 40
for _ in range(3):
    e.run_sites(s)
ms = e.last_kernel_ms()
print(f"{a.workload} {'interp' if a.interp else 'translated'} waves={a.waves}: {ms:.3f} ms, "
      f"{ms * 1e6 / g.ninst:.1f} ns/inst, golden {g.ninst} insts", flush=True)
