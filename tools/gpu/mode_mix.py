"""Where the solo epoch's time goes, per library build: one bench-shaped step
(WORKLOAD, N trials, seeded regs+pc sites) on the translated kernels, then the
per-wave debug records of the solo dispatch (fi_trial.hip wave_dbg) summed:
instructions by mode (translated blocks, interpreter), translated-code
entries, loop trips, page-table misses, wave cycles -- and a least-squares fit
of wave cycles on (translated insts, other insts, entries, misses).

SHREWD_FI_LIB=... python tools/gpu/mode_mix.py [WORKLOAD] [N] [SEED] -> one JSON line"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from shrewd_amd import Engine  # noqa: E402

REGS_PC = ((1 << 32) - 2) | (1 << 32)
name = sys.argv[1] if len(sys.argv) > 1 else "crc32"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
SEED = int(sys.argv[3], 0) if len(sys.argv) > 3 else 0x5EED0002
e = Engine(max_trials_per_launch=N)
e.load_elf(open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb").read(), [name])
e.golden_run()
e.wait_translation()
e.set_campaign(SEED, REGS_PC, 1)
rec = {"lib": os.environ.get("SHREWD_FI_LIB", "default"), "workload": name, "trials": N}
for rep in range(3):
    e.kernel_timer_reset()
    out, h = e.run_trials(0, N, want_outcomes=False)
    ms = e.debug_dispatch_ms()
    kinds = e.debug_dispatch_kinds()
rec["dispatch_ms"] = {str(k): round(m, 3) for m, k in zip(ms, kinds)}
ep = e.debug_epochs()
ns = int(ep[0])
w = e.debug_waves(ns).reshape(ns, 10).astype(np.int64)
w = w[(w[:, 5] > 0) & (w[:, 6] >= 0)]
tx, insts = w[:, 2], w[:, 7]
other = np.maximum(insts - tx, 0)
cyc = w[:, 0]
rec.update({"solo_waves": int(len(w)), "insts": int(insts.sum()), "tx_insts": int(tx.sum()),
            "other_insts": int(other.sum()), "iters": int(w[:, 1].sum()), "tx_entries": int(w[:, 8].sum()),
            "trips": int((w[:, 3] >> 32).sum()), "slow": int((w[:, 3] & 0xFFFFFFFF).sum()),
            "nmiss": int(w[:, 9].sum()), "wave_cycles": int(cyc.sum())})
A = np.stack([tx, other, w[:, 8], w[:, 9], np.ones(len(w))], 1).astype(np.float64)
coef = np.linalg.lstsq(A, cyc.astype(np.float64), rcond=None)[0]
rec["fit_cycles_per"] = {"tx_inst": round(coef[0], 2), "other_inst": round(coef[1], 2),
                         "tx_entry": round(coef[2], 1), "miss": round(coef[3], 1), "wave": round(coef[4], 1)}
print(json.dumps(rec), flush=True)
e.close()
