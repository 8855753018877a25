"""A tick-domain campaign (cpu_type="timing") on one GPU: N seeded single-bit
register / pc / result tick sites of one workload, timed end to end, every
trial re-run literally on the CPU oracle (checker only) and compared bit for
bit.  The numInst campaign of the same size is timed beside it.

python tools/gpu/tick_campaign.py [WORKLOAD] [N] [SEED] [CHECK]  -> JSON lines"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from shrewd_amd import Engine  # noqa: E402
from shrewd_amd.fi import TICK_ESCAPE_NAMES, escape_breakdown  # noqa: E402

STRUCTS = ((1 << 32) - 2) | (1 << 32) | (1 << 34)
name = sys.argv[1] if len(sys.argv) > 1 else "crc32"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
SEED = int(sys.argv[3], 0) if len(sys.argv) > 3 else 0x5EED7102
CHECK = int(sys.argv[4]) if len(sys.argv) > 4 else N
elf = open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb").read()
e = Engine()
e.load_elf(elf, [name])
e.set_cpu_model("timing")
t0 = time.perf_counter()
g = e.golden_run()
info = e.tick_info()
setup = time.perf_counter() - t0
e.set_campaign(SEED, STRUCTS, 1)
e.run_tick_trials(0, min(N, 20000), want_outcomes=False)   # warm-up (buffers)
t0 = time.perf_counter()
out, h = e.run_tick_trials(0, N)
wall = time.perf_counter() - t0
ts = e.sample_tick_sites(0, N)
_, disp, _ = e.map_tick_sites(ts)
t0 = time.perf_counter()
e.run_trials(0, N, want_outcomes=False)
wall_num = time.perf_counter() - t0
cls = np.bincount(out["cls"], minlength=6).tolist()
tesc = (out["cls"] == 5) & (out["sub"] == 7)
rec = {"workload": name, "trials": N, "seed": hex(SEED), "structures": "int_reg|pc|result",
       "golden_ninst": int(g.ninst), "golden_ticks": info["golden_ticks"], "attempts": info["attempts"],
       "timing_stats": info["stats"], "setup_s": round(setup, 3),
       "wall_s": round(wall, 3), "trials_per_s": round(N / wall),
       "numinst_campaign_trials_per_s": round(N / wall_num),
       "dispositions": {"device": int((disp == 0).sum()), "golden_equal": int((disp == 1).sum()),
                        "timing_escape": int((disp == 2).sum())},
       "classes": dict(zip(["masked", "sdc", "crash", "hang", "detected", "escape"], cls)),
       "escapes": escape_breakdown(out),
       "timing_escape_reasons": {TICK_ESCAPE_NAMES.get(int(k), str(k)): int(v) for k, v in
                                 zip(*np.unique(out["exit_code"][tesc], return_counts=True))}}
print(json.dumps(rec), flush=True)
e.close()
from oracle.pyoracle import Oracle  # noqa: E402
idx = np.arange(N) if CHECK >= N else np.sort(np.random.default_rng(SEED).choice(N, size=CHECK, replace=False))
o = Oracle(elf, name)
o.run_golden()
o.tick_setup()
osites = o.tick_sample(SEED, 0, N, STRUCTS)
assert (osites == ts).all(), "sampled tick sites differ"
t1 = time.perf_counter()
bad = 0
piece = 20_000
for a in range(0, len(idx), piece):
    ref = o.run_tick_trials(osites[idx[a:a + piece]], threads=16)
    bad += int((ref != out[idx[a:a + piece]]).sum())
    print(json.dumps({"progress": a + len(ref), "of": int(len(idx)), "mismatches": bad,
                      "s": round(time.perf_counter() - t1, 1)}), flush=True)
rec["oracle_check"] = {"checked": int(len(idx)), "mismatches": bad, "oracle_s": round(time.perf_counter() - t1, 2),
                       "threads": 16, "which": "all trials" if CHECK >= N else "seeded sample",
                       "kind": "literal tick injection (rv64se.c tk_trial)"}
print(json.dumps(rec), flush=True)
sys.exit(0 if bad == 0 else 1)
