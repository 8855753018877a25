"""FI_PROF phase cycles of chosen trials run alone through the interpreter
(no translation): python tools/gpu/prof_trial.py WORKLOAD SEED ID [ID ...]
(run with SHREWD_FI_LIB pointing at a -DFI_PROF build; PROF_FLAGS adds engine
flags, e.g. 128 for the solo kernel)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from shrewd_amd import Engine  # noqa: E402
from shrewd_amd.fi import CFG_NO_TRANSLATE  # noqa: E402

REGS_PC = ((1 << 32) - 2) | (1 << 32)
name, seed, ids = sys.argv[1], int(sys.argv[2], 0), [int(x) for x in sys.argv[3:]]
e = Engine(max_trials_per_launch=131072, flags=CFG_NO_TRANSLATE | 8 | int(os.environ.get("PROF_FLAGS", "0"), 0))
e.load_elf(open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb").read(), [name])
e.golden_run()
e.set_campaign(seed, REGS_PC, 1)
allsites = e.sample(0, max(ids) + 1)
for i in ids:
    s = allsites[[i]]
    out, _ = e.run_sites(s)
    ms = e.last_kernel_ms()
    st = e.debug_stats().astype(np.int64)
    it = max(1, int(st[6]))
    print(json.dumps({"trial": i, "cls": int(out["cls"][0]), "kernel_ms": round(ms, 3), "iters": it,
                      "slow": int(st[8]), "ns_per_iter": round(ms * 1e6 / it, 1),
                      "cycles_per_iter_by_stamp": [round(int(st[32 + k]) / it, 1) for k in range(8)]}), flush=True)
