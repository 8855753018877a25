"""Single-trial speed of each execution path: the same trial alone with the
translated blocks on/off and on the 64-lane or solo kernel.
python tools/gpu/path_speed.py WORKLOAD SEED ID [ID ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from shrewd_amd import Engine  # noqa: E402

REGS_PC = ((1 << 32) - 2) | (1 << 32)
name, seed, ids = sys.argv[1], int(sys.argv[2], 0), [int(x) for x in sys.argv[3:]]
elf = open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb").read()
for label, flags in (("solo_tx", 128), ("solo_interp", 128 | 4), ("wave_tx", 64), ("wave_interp", 64 | 4)):
    e = Engine(flags=flags | 8 | 1 | 2)   # no epochs, from process start, no early exit
    e.load_elf(elf, [name])
    e.golden_run()
    e.set_campaign(seed, REGS_PC, 1)
    sites = e.sample(0, max(ids) + 1)
    for i in ids:
        s = sites[[i]]
        e.run_sites(s)
        o, _ = e.run_sites(s)
        ms = e.last_kernel_ms()
        st = e.debug_stats()
        print(json.dumps({"path": label, "trial": i, "cls": int(o["cls"][0]), "ninst": int(o["ninst"][0]),
                          "ns_per_inst": round(ms * 1e6 / max(1, int(o["ninst"][0])), 1), "slow": int(st[8]),
                          "tx": int(st[16])}), flush=True)
    e.close()
