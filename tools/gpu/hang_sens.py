"""How much of a workload's step is its hang trials: the same campaign step at
several hang caps (hang_factor_x16), ms per step and per-kernel ms each.

python tools/gpu/hang_sens.py [WORKLOAD] [TRIALS] [FACTORS_X16...] -> JSON lines"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from shrewd_amd import Engine  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "crc32"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
factors = [int(x) for x in sys.argv[3:]] or [32, 24, 17]
elf = open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb").read()
for f in factors:
    e = Engine(max_trials_per_launch=N, hang_factor_x16=f)
    e.load_elf(elf, [name])
    e.golden_run()
    e.set_campaign(0x5EED0002, ((1 << 32) - 2) | (1 << 32), 1)
    e.run_trials(0, N, want_outcomes=False)
    ts = []
    for k in range(5):
        t0 = time.perf_counter()
        out, h = e.run_trials((k + 1) * N, N)
        ts.append(time.perf_counter() - t0)
    cls = np.bincount(out["cls"], minlength=6).tolist()
    print(json.dumps({"workload": name, "hang_factor_x16": f, "ms_per_step": round(1e3 * min(ts), 3),
                      "ms_median": round(1e3 * sorted(ts)[2], 3), "classes": cls,
                      "device_insts": int(h["device_insts"])}), flush=True)
    e.close()
