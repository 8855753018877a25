"""One trial run alone on the product path (translation on, solo kernel after
the first epoch): kernel time and where its instructions ran.

python tools/gpu/one_trial.py WORKLOAD SEED ID [ID ...]  -> JSON lines"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from shrewd_amd import Engine  # noqa: E402

REGS_PC = ((1 << 32) - 2) | (1 << 32)
name, seed, ids = sys.argv[1], int(sys.argv[2], 0), [int(x) for x in sys.argv[3:]]
e = Engine(max_trials_per_launch=65536)
e.load_elf(open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb").read(), [name])
e.golden_run()
e.set_campaign(seed, REGS_PC, 1)
allsites = e.sample(0, max(ids) + 1)
for rep in range(2):
    for i in ids:
        s = allsites[[i]]
        e.kernel_timer_reset()
        out, _ = e.run_sites(s)
        st = e.debug_stats().astype(np.int64)
        dms, kinds = e.debug_dispatch_ms(), e.debug_dispatch_kinds()
        rec = {"trial": i, "rep": rep, "site": [int(s["inst"][0]), hex(int(s["mask"][0])), int(s["target"][0])],
               "cls": int(out["cls"][0]), "sub": int(out["sub"][0]), "ninst": int(out["ninst"][0]),
               "dispatch_ms": [round(float(x), 3) for x in dms], "kinds": [int(k) for k in kinds],
               "device_insts": int(st[23]), "tx_insts": int(st[16]), "tx_entries": int(st[17]),
               "fast_calls": int(st[53]), "fast_insts": int(st[54]), "fast_handbacks": int(st[55]),
               "loop_iters": int(st[6]), "slow_fetches": int(st[8])}
        tot = sum(dms)
        rec["ns_per_inst"] = round(tot * 1e6 / max(1, int(st[23])), 1)
        print(json.dumps(rec), flush=True)
