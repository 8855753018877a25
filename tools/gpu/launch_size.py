"""Why does one 1M-trial launch run slower per trial than 100k-trial launches?
Runs the same N seeded trials once per launch size and reports, per size:
wall time, per-dispatch kernel time by kind (0 64-lane, 1 solo, 2 solo-odd),
epoch survivor counts, the redo count (stats[30]) and the solo dispatch's
slowest waves (start / end, instructions, outcome) of the LAST chunk.

python tools/gpu/launch_size.py [WORKLOAD] [N] [SEED] [SIZES...] -> JSON lines"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from shrewd_amd import Engine  # noqa: E402

REGS_PC = ((1 << 32) - 2) | (1 << 32)
name = sys.argv[1] if len(sys.argv) > 1 else "qsort"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
SEED = int(sys.argv[3], 0) if len(sys.argv) > 3 else 0x5EED0003
SIZES = [int(s) for s in sys.argv[4:]] or [N, 100_000]
PP = int(os.environ.get("LS_PAGES", "16"))
elf = open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb").read()
ref = None
for size in SIZES:
    e = Engine(max_trials_per_launch=size, private_pages=PP)
    e.load_elf(elf, [name])
    e.golden_run()
    e.set_campaign(SEED, REGS_PC, 1)
    e.run_trials(0, size, want_outcomes=False)     # warm-up (buffers)
    e.kernel_timer_reset()
    t0 = time.perf_counter()
    out, h = e.run_trials(0, N)
    wall = time.perf_counter() - t0
    ms = e.debug_dispatch_ms()
    kinds = e.debug_dispatch_kinds()
    by = {}
    for m, k in zip(ms, kinds):
        by.setdefault(str(k), []).append(m)
    st = e.debug_stats()
    ep = e.debug_epochs()
    k_last = N - size * ((N - 1) // size)
    w = e.debug_waves(k_last).reshape(k_last, 10).astype(np.int64)
    live = (w[:, 6] >= 0) & (w[:, 6] < k_last) & (w[:, 5] > 0) & (w[:, 7] > 0)
    w = w[live]
    rec = {"workload": name, "trials": N, "per_launch": size, "private_pages": PP, "wall_s": round(wall, 4),
           "trials_per_s": round(N / wall), "device_insts": int(h["device_insts"]),
           "dispatch_ms_by_kind": {k: [round(sum(v), 2), len(v)] for k, v in by.items()},
           "epochs_last_chunk": ep[:4], "redo_last_chunk": int(st[30]), "stats_0_24": st[:64].tolist(),
           "same_as_first": None if ref is None else int((out != ref).sum())}
    if len(w):
        t0w = w[:, 4].min()
        start, end = (w[:, 4] - t0w) / 100.0, (w[:, 5] - t0w) / 100.0
        rec["solo_waves"] = int(len(w))
        rec["solo_span_us"] = round(float(end.max()), 1)
        rec["solo_insts"] = int(w[:, 7].sum())
        rec["end_q_us"] = {q: round(float(np.quantile(end, q)), 1) for q in (0.5, 0.9, 0.99, 0.999, 1.0)}
        rec["active_at_us"] = {t: int(((start <= t) & (end > t)).sum())
                               for t in (100, 1000, 5000, 20000, 50000, 100000, 200000, 400000)}
        order = np.argsort(-(end - start))[:int(os.environ.get("LS_TOP", "8"))]
        rec["slowest"] = [{"trial": int(w[i, 6]) + N - k_last, "cls": int(out["cls"][int(w[i, 6]) + N - k_last]),
                           "start_us": round(float(start[i]), 1), "end_us": round(float(end[i]), 1),
                           "insts": int(w[i, 7]), "iters": int(w[i, 1]), "tx_insts": int(w[i, 2]),
                           "slow": int(w[i, 3]) & 0xFFFFFFFF, "trips": int(w[i, 3]) >> 32,
                           "tx_entries": int(w[i, 8]), "nmiss": int(w[i, 9]),
                           "ns_per_inst": round(1e3 * float(end[i] - start[i]) / max(1, int(w[i, 7])), 1)}
                          for i in order]
    esc = np.nonzero(out["cls"] == 5)[0]
    rec["escapes"] = [{"trial": int(i), "sub": int(out["sub"][i]), "detail": hex(int(out["detail"][i])),
                       "ninst": int(out["ninst"][i])} for i in esc[:40]]
    if ref is None:
        ref = out
    print(json.dumps(rec), flush=True)
    e.close()
