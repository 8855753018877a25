"""Where the step time of a campaign goes: per-dispatch (epoch) times and
survivor counts of the benched configuration, then the longest trials run
alone (one lane) with their per-instruction latency and path counters.

python tools/gpu/tail_profile.py [WORKLOAD] [SEED] [N]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from shrewd_amd import Engine  # noqa: E402

REGS_PC = ((1 << 32) - 2) | (1 << 32)
name = sys.argv[1] if len(sys.argv) > 1 else "crc32"
seed = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0x5EED0002
n = int(sys.argv[3]) if len(sys.argv) > 3 else 100000
e = Engine(max_trials_per_launch=max(n, 1024))
e.load_elf(open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb").read(), [name])
g = e.golden_run()
e.set_campaign(seed, REGS_PC, 1)
sites = e.sample(0, n)
for rep in range(2):
    e.kernel_timer_reset()
    out, h = e.run_sites(sites)
    st = e.debug_stats()
print(json.dumps({"workload": name, "golden_ninst": int(g.ninst), "dispatch_ms": e.debug_dispatch_ms(),
                  "survivors": e.debug_epochs()[:4], "kernel_ms": e.last_kernel_ms(),
                  "classes": np.bincount(out["cls"], minlength=6).tolist(),
                  "device_insts": int(h["device_insts"]), "tx_insts": int(st[16]), "slow_fetches": int(st[8]),
                  "slowest_wave": {"iters": int(st[18]) >> 32, "tx_permille": (int(st[18]) >> 20) & 0xFFF,
                                   "entries": int(st[18]) & 0xFFFFF}}), flush=True)
# work after injection (instructions a serial run executes past the inject point)
early = (out["cls"] == 0) & (out["ninst"] == g.ninst)
work = out["ninst"].astype(np.int64) - sites["inst"].astype(np.int64)
order = np.argsort(-work)
print(json.dumps({"work_quantiles": {q: int(np.quantile(work, q)) for q in (0.5, 0.9, 0.99, 0.999, 1.0)},
                  "top_classes": np.bincount(out["cls"][order[:500]], minlength=6).tolist()}), flush=True)
picked = []
for cls in (3, 1, 2, 0):
    idx = [int(i) for i in order if out["cls"][i] == cls][:3]
    picked += idx
for i in picked:
    s = sites[[i]]
    e.run_sites(s)
    o, _ = e.run_sites(s)
    ms = e.last_kernel_ms()
    st = e.debug_stats()
    ran = int(o["ninst"][0]) - int(s["inst"][0])
    print(json.dumps({"trial": i, "target": int(s["target"][0]), "bit": int(np.log2(float(s["mask"][0]))),
                      "cls": int(o["cls"][0]), "sub": int(o["sub"][0]), "ran": ran, "ms": round(ms, 3),
                      "ns_per_inst": round(ms * 1e6 / max(1, ran), 1), "iters": int(st[6]), "slow": int(st[8]),
                      "tx_insts": int(st[16]), "tx_entries": int(st[17]), "dispatch_ms": e.debug_dispatch_ms()}),
          flush=True)
