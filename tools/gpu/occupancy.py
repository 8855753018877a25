"""Residency timeline of the last dispatch of a campaign (the solo epoch by
default): per-wave start/end s_memrealtime stamps -> waves resident over time.
python tools/gpu/occupancy.py [WORKLOAD] [SEED] [N] [FLAGS] [STRUCTURES] [BURST]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from shrewd_amd import Engine  # noqa: E402

REGS_PC = ((1 << 32) - 2) | (1 << 32)
name = sys.argv[1] if len(sys.argv) > 1 else "qsort"
seed = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0x5EED0003
n = int(sys.argv[3]) if len(sys.argv) > 3 else 100000
flags = int(sys.argv[4], 0) if len(sys.argv) > 4 else 0
structures = int(sys.argv[5], 0) if len(sys.argv) > 5 else REGS_PC
burst = int(sys.argv[6]) if len(sys.argv) > 6 else 1
e = Engine(max_trials_per_launch=n, flags=flags)
e.load_elf(open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb").read(), [name])
e.golden_run()
e.set_campaign(seed, structures, burst)
sites = e.sample(0, n)
for rep in range(2):
    e.kernel_timer_reset()
    out, h = e.run_sites(sites)
wv = e.debug_waves(n).astype(np.int64)
live = wv[:, 4] > 0
st, en, it = wv[live, 4], wv[live, 5], wv[live, 1]
t0 = st.min()
st, en = (st - t0) / 100.0, (en - t0) / 100.0   # microseconds (100 MHz)
ev = np.concatenate([np.stack([st, np.ones_like(st)], 1), np.stack([en, -np.ones_like(en)], 1)])
ev = ev[np.argsort(ev[:, 0], kind="stable")]
conc = np.cumsum(ev[:, 1])
tt = ev[:, 0]
dur = np.diff(np.concatenate([tt, tt[-1:]]))
span = tt[-1] - tt[0]
avg = float((conc * dur).sum() / span) if span else 0.0
q = {f"t_conc_below_{k}_us": float(tt[np.nonzero(conc >= k)[0][-1]]) if (conc >= k).any() else 0.0
     for k in (3000, 1000, 300, 100, 30, 10, 1)}
print(json.dumps({"workload": name, "flags": flags, "structures": hex(structures), "burst": burst, "dispatch_ms": e.debug_dispatch_ms(), "waves": int(live.sum()),
                  "span_us": round(float(span), 1), "max_resident": int(conc.max()), "avg_resident": round(avg, 1),
                  "last_start_us": round(float(st.max()), 1),
                  "start_quantiles_us": {p: round(float(np.quantile(st, p)), 1) for p in (0.1, 0.5, 0.9, 0.99)},
                  "duration_quantiles_us": {p: round(float(np.quantile(en - st, p)), 1)
                                            for p in (0.5, 0.9, 0.99, 0.999, 1.0)},
                  **q}), flush=True)
# the slowest waves: lane 0's trial, its instructions in the dispatch, loop
# iterations, translated instructions, slow fetches, loop trips (solo) or
# min-PC reductions (64-lane)
dur_all = np.where(live, wv[:, 5] - wv[:, 4], 0)
for b in np.argsort(-dur_all)[:8]:
    tr = int(wv[b, 6])
    s = sites[tr] if tr < n else None
    print(json.dumps({"wave": int(b), "us": round(dur_all[b] / 100.0, 1), "trial": tr, "insts": int(wv[b, 7]),
                      "ns_per_inst": round(dur_all[b] * 10.0 / max(1, int(wv[b, 7])), 1), "iters": int(wv[b, 1]),
                      "tx": int(wv[b, 2]), "slow": int(wv[b, 3]) & 0xFFFFFFFF, "trips": int(wv[b, 3]) >> 32,
                      "tx_entries": int(wv[b, 8]),
                      "page_lookups": int(wv[b, 9]),
                      "target": int(s["target"]) if s is not None else None,
                      "mask": hex(int(s["mask"])) if s is not None else None,
                      "inst": int(s["inst"]) if s is not None else None,
                      "cls": int(out["cls"][tr]) if tr < n else None}), flush=True)
# where the dispatch's wave-time goes, by the outcome class of each wave's
# (lane 0) trial: waves, summed wave-microseconds, summed instructions
trs = wv[live, 6]
ok = trs < n
cls_of = np.where(ok, out["cls"][np.minimum(trs, n - 1)], 255)
us = (wv[live, 5] - wv[live, 4]) / 100.0
agg = {}
for c in np.unique(cls_of):
    m = cls_of == c
    agg[["masked", "sdc", "crash", "hang", "detected", "escape"][c] if c < 6 else "?"] = {
        "waves": int(m.sum()), "wave_us": round(float(us[m].sum()), 1), "insts": int(wv[live, 7][m].sum()),
        "median_insts": int(np.median(wv[live, 7][m]))}
print(json.dumps({"by_class": agg}), flush=True)
