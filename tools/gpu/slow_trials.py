"""Per-instruction cost of chosen trials run alone on the solo kernel.

python tools/gpu/slow_trials.py WORKLOAD SEED STRUCTS ID [ID ...]
  STRUCTS: regs_pc | mem | result
Prints, per trial: outcome class, device-executed guest instructions,
kernel ms, ns per executed instruction, translated instructions / entries and
slow fetches (debug stats), for the default build (SHREWD_FI_LIB selects a
-DFI_PROF build, whose phase stamps are added: cycles per iteration)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from shrewd_amd import Engine  # noqa: E402

S = {"regs_pc": ((1 << 32) - 2) | (1 << 32), "mem": 1 << 33, "result": 1 << 34}
name, seed, structs = sys.argv[1], int(sys.argv[2], 0), S[sys.argv[3]]
ids = [int(x) for x in sys.argv[4:]]
flags = int(os.environ.get("SLOW_FLAGS", "128"), 0)      # FI_CFG_SOLO_ALL
e = Engine(max_trials_per_launch=131072, flags=flags)
e.load_elf(open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb").read(), [name])
e.golden_run()
e.set_campaign(seed, structs, 1)
allsites = e.sample(0, max(ids) + 1)
for i in ids:
    s = allsites[[i]]
    e.run_sites(s)                  # warm
    out, h = e.run_sites(s)
    ms = e.last_kernel_ms()
    st = e.debug_stats().astype(np.int64)
    xi = int(h["device_insts"])
    rec = {"trial": i, "site": {k: int(s[0][k]) for k in ("inst", "target", "mask")}, "cls": int(out["cls"][0]),
           "ninst_end": int(out["ninst"][0]), "executed": xi, "kernel_ms": round(ms, 3),
           "ns_per_inst": round(ms * 1e6 / max(xi, 1), 1), "translated": int(st[16]), "tx_entries": int(st[17]),
           "slow_fetches": int(st[8]), "iters": int(st[6]), "trips": int(st[9]),
           "fast_calls": int(st[53]), "fast_insts": int(st[54]), "fast_backs": int(st[55]),
           "proofs_56_63": [int(x) for x in st[56:64]]}
    if os.environ.get("SHREWD_FI_LIB"):
        rec["cycles_per_iter_by_stamp"] = [round(int(st[32 + k]) / max(1, int(st[6])), 1) for k in range(8)]
        rec["stats_32_40"] = [int(x) for x in st[32:40]]
    print(json.dumps(rec), flush=True)
