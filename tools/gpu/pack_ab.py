"""A/B of resume strategies on the GPU: fixed resume_lanes vs pc-run packing
(FI_CFG_PACK_RUNS), with several epoch counts.  Outcomes must be identical
across configurations; prints device ms and trials/s per (workload, config).

python tools/gpu/pack_ab.py [workload ...]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
from shrewd_amd import Engine  # noqa: E402
from shrewd_amd.fi import CFG_PACK_RUNS  # noqa: E402

REGS_PC = ((1 << 32) - 2) | (1 << 32)
N = {"crc32": 100_000, "qsort": 100_000, "intmix": 125_000}
CONFIGS = [("fixed8_e4", dict()),
           ("pack_e4", dict(flags=CFG_PACK_RUNS)),
           ]
for name in (sys.argv[1:] or ["crc32", "qsort", "intmix"]):
    elf = open(f"workloads/{name}.elf", "rb").read()
    ref = None
    for label, kw in CONFIGS:
        e = Engine(max_trials_per_launch=131072, **kw)
        e.load_elf(elf, [name])
        e.golden_run()
        e.set_campaign(0x5EED0003, REGS_PC, 1)
        e.run_trials(0, N[name])   # warm: code objects, work buffers
        e.kernel_timer_reset()
        t0 = time.perf_counter()
        out, h = e.run_trials(0, N[name])
        dt = time.perf_counter() - t0
        kt = e.kernel_timer_read()
        same = True if ref is None else bool(np.array_equal(out, ref))
        ref = out if ref is None else ref
        print(json.dumps({"workload": name, "config": label, "wall_s": round(dt, 3),
                          "trials_per_s": round(N[name] / dt), "kernel": kt,
                          "epochs": e.debug_epochs()[:8], "dispatch_ms": e.debug_dispatch_ms(), "same_outcomes": same}), flush=True)
        e.close()
        if not same:
            sys.exit(1)
