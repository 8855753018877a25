"""One configuration of an A/B run on the GPU: campaigns on crc32/qsort/intmix
with the engine's defaults (the environment selects build knobs, e.g.
SHREWD_FI_WAVES_PER_EU); prints device ms per dispatch and a digest of the
outcomes so runs can be compared.

python tools/gpu/ab_run.py LABEL [workload ...] [--resume-lanes N] [--epochs N]
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from shrewd_amd import Engine  # noqa: E402

REGS_PC = ((1 << 32) - 2) | (1 << 32)
N = {"crc32": 100_000, "qsort": 100_000, "intmix": 125_000}
ap = argparse.ArgumentParser()
ap.add_argument("label")
ap.add_argument("workloads", nargs="*", default=["crc32", "qsort", "intmix"])
ap.add_argument("--resume-lanes", type=int, default=0)
ap.add_argument("--epochs", type=int, default=0)
ap.add_argument("--flags", type=int, default=0)
ap.add_argument("--epoch-iters", type=int, default=0)
a = ap.parse_args()
for name in a.workloads:
    e = Engine(max_trials_per_launch=131072, resume_lanes=a.resume_lanes, epochs=a.epochs, flags=a.flags,
               epoch_iters=a.epoch_iters)
    e.load_elf(open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb").read(), [name])
    e.golden_run()
    e.set_campaign(0x5EED0003, REGS_PC, 1)
    e.run_trials(0, N[name])   # warm
    e.kernel_timer_reset()
    t0 = time.perf_counter()
    out, h = e.run_trials(0, N[name])
    dt = time.perf_counter() - t0
    print(json.dumps({"label": a.label, "workload": name, "wall_s": round(dt, 4), "trials_per_s": round(N[name] / dt),
                      "dispatch_ms": e.debug_dispatch_ms(), "epochs": e.debug_epochs()[:6],
                      "digest": hashlib.sha1(out.tobytes()).hexdigest()[:12]}), flush=True)
    e.close()
