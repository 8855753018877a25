"""Diverged-lanes step loop A/B: 100k-trial campaigns under several path
configurations; every configuration's outcomes must equal the default's bit
for bit.  python tools/gpu/simt_sweep.py [WORKLOAD:SEED ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from shrewd_amd import Engine  # noqa: E402

REGS_PC = ((1 << 32) - 2) | (1 << 32)
CFGS = [("default", 0, 0), ("simt", 256, 0), ("simt_no_solo", 256 | 64, 0), ("simt_no_solo_3ep", 256 | 64, 3),
        ("simt_no_solo_no_epochs", 256 | 64 | 8, 0), ("no_solo", 64, 0)]
jobs = sys.argv[1:] or ["crc32:0x5EED0002", "qsort:0x5EED0003", "intmix:0x5EED0003"]
for job in jobs:
    name, seed = job.split(":")
    seed = int(seed, 0)
    elf = open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb").read()
    ref = None
    for label, flags, epochs in CFGS:
        e = Engine(max_trials_per_launch=100000, flags=flags, epochs=epochs)
        e.load_elf(elf, [name])
        e.golden_run()
        e.set_campaign(seed, REGS_PC, 1)
        sites = e.sample(0, 100000)
        for rep in range(2):
            e.kernel_timer_reset()
            out, h = e.run_sites(sites)
            st = e.debug_stats()
        same = None
        if ref is None:
            ref = out.copy()
        else:
            same = bool(out.tobytes() == ref.tobytes())
        print(json.dumps({"w": name, "cfg": label, "kernel_ms": round(e.last_kernel_ms(), 2),
                          "dispatch_ms": [round(x, 2) for x in e.debug_dispatch_ms()],
                          "survivors": e.debug_epochs()[:4], "device_insts": int(h["device_insts"]),
                          "simt_insts": int(st[24]), "tx_insts": int(st[16]), "slow": int(st[8]),
                          "identical_to_default": same}), flush=True)
        e.close()
