"""Serial latency of chosen trials on the GPU: each given trial id runs alone
(one lane) and as part of its category; prints device ms, ns per guest
instruction and the wave's loop counters.

python tools/gpu/tail.py WORKLOAD SEED ID [ID ...]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from shrewd_amd import Engine  # noqa: E402

REGS_PC = ((1 << 32) - 2) | (1 << 32)
name, seed, ids = sys.argv[1], int(sys.argv[2], 0), [int(x) for x in sys.argv[3:]]
e = Engine(max_trials_per_launch=131072)
e.load_elf(open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb").read(), [name])
e.golden_run()
e.set_campaign(seed, REGS_PC, 1)
allsites = e.sample(0, max(ids) + 1)
for i in ids + [ids]:
    s = allsites[np.atleast_1d(i)]
    e.run_sites(s)
    out, _ = e.run_sites(s)
    ms = sum(e.debug_dispatch_ms()[-4:]) if False else e.last_kernel_ms()
    st = e.debug_stats()
    ran = int(out["ninst"].max()) - int(s["inst"].min())
    print(json.dumps({"trial": i if isinstance(i, int) else "all", "cls": out["cls"].tolist()[:8],
                      "ninst_after_inject": ran, "kernel_ms": round(ms, 3),
                      "ns_per_inst": round(ms * 1e6 / max(1, ran), 1), "iters": int(st[6]), "slow": int(st[8]),
                      "minpc": int(st[9]), "tx_insts": int(st[16]), "tx_entries": int(st[17]),
                      "checks": int(st[11])}), flush=True)
