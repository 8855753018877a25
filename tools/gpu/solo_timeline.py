"""Timeline of the solo kernel of one campaign step: per wave (one trial each)
its start / end (s_memrealtime, 100 MHz), the instructions it ran and its
trial's outcome -- which trials set the kernel's span, when they started and
how fast they ran in the crowd.

python tools/gpu/solo_timeline.py [WORKLOAD] [SEED] [N] [TOP]  -> JSON lines"""
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
n = int(sys.argv[3]) if len(sys.argv) > 3 else 100_000
top = int(sys.argv[4]) if len(sys.argv) > 4 else 12
e = Engine(max_trials_per_launch=n)
e.load_elf(open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb").read(), [name])
e.golden_run()
e.set_campaign(seed, REGS_PC, 1)
sites = e.sample(0, n)
e.run_sites(sites)
e.kernel_timer_reset()
out, h = e.run_sites(sites)
w = e.debug_waves(n).reshape(n, 10).astype(np.int64)
live = (w[:, 6] >= 0) & (w[:, 6] < n) & (w[:, 5] > 0)
w = w[live]
t0 = w[:, 4].min()
start, end = (w[:, 4] - t0) / 100.0, (w[:, 5] - t0) / 100.0        # us
ins = w[:, 7]
span = end.max()
busy = ins > 0
rec = {"workload": name, "trials": n, "dispatch_ms": e.debug_dispatch_ms(), "solo_waves_with_work": int(busy.sum()),
       "solo_span_us": round(float(span), 1), "insts_total": int(ins.sum()),
       "end_quantiles_us": {q: round(float(np.quantile(end[busy], q)), 1) for q in (0.5, 0.9, 0.99, 0.999, 1.0)},
       "start_quantiles_us": {q: round(float(np.quantile(start[busy], q)), 1) for q in (0.5, 0.9, 0.99, 1.0)},
       "active_at_us": {t: int(((start <= t) & (end > t) & busy).sum()) for t in (100, 500, 1000, 2000, 3000, 4000)}}
print(json.dumps(rec), flush=True)
# the solo order's key (fi_surv_keys_kernel): instructions committed when the
# solo dispatch began (a proved hang's record says the cap: skip those)
tids = w[:, 6]
n0 = out["ninst"][tids].astype(np.int64) - ins
ok = busy & (out["cls"][tids] != 3)
late = ok & (start > 1000.0)
print(json.dumps({"ninst_at_solo_start_quantiles": {q: int(np.quantile(n0[ok], q)) for q in (0.01, 0.1, 0.5, 0.9)},
                  "late_starters": int(late.sum()),
                  "late_starters_ninst0_quantiles": {q: int(np.quantile(n0[late], q)) for q in (0.01, 0.1, 0.5, 0.9)}
                  if late.any() else {},
                  "start_rank_corr": round(float(np.corrcoef(np.argsort(np.argsort(start[ok])),
                                                             np.argsort(np.argsort(n0[ok])))[0, 1]), 3)}), flush=True)
# where the solo work goes: instructions by outcome class and injected register
grp = {}
for c, t, k in zip(out["cls"][tids[busy]], sites["target"][tids[busy]], ins[busy]):
    g = grp.setdefault(f"{int(c)}/{int(t)}", [0, 0])
    g[0] += 1
    g[1] += int(k)
print(json.dumps({"insts_by_cls_target": dict(sorted(grp.items(), key=lambda kv: -kv[1][1])[:24])}), flush=True)
order = np.argsort(-end)[:top]
for i in order:
    tid = int(w[i, 6])
    print(json.dumps({"trial": tid, "cls": int(out["cls"][tid]), "target": int(sites["target"][tid]),
                      "bit": int(np.log2(float(sites["mask"][tid]))) if int(sites["mask"][tid]) else -1,
                      "start_us": round(float(start[i]), 1), "end_us": round(float(end[i]), 1),
                      "insts": int(ins[i]), "ninst0": int(n0[i]), "ns_per_inst": round(1e3 * float(end[i] - start[i]) / max(1, int(ins[i])), 1),
                      "tx_entries": int(w[i, 8]), "tx_insts": int(w[i, 2])}), flush=True)
# every solo trial, for offline scheduling studies (SOLO_TL_DUMP=path.npz)
if os.environ.get("SOLO_TL_DUMP"):
    np.savez(os.environ["SOLO_TL_DUMP"], tid=tids, start_us=start, end_us=end, insts=ins, n0=n0,
             cls=out["cls"][tids], ninst=out["ninst"][tids], target=sites["target"][tids], mask=sites["mask"][tids],
             inst=sites["inst"][tids], golden_ninst=int(e.golden.ninst))
