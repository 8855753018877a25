"""The north-star campaign on one GPU: >= 1M seeded single-bit register/PC
trials of one workload in one launch, timed end to end, with CHECK of its
trials (all of them when CHECK >= N, else a seeded sample) re-run on the CPU
oracle and compared bit for bit.

python tools/gpu/north_star.py [WORKLOAD] [N] [SEED] [CHECK] [PER_LAUNCH]  -> JSON lines"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from shrewd_amd import Engine  # noqa: E402
from shrewd_amd.fi import escape_breakdown  # noqa: E402

REGS_PC = ((1 << 32) - 2) | (1 << 32)
name = sys.argv[1] if len(sys.argv) > 1 else "intmix"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
SEED = int(sys.argv[3], 0) if len(sys.argv) > 3 else 0x5EED0003
CHECK = int(sys.argv[4]) if len(sys.argv) > 4 else 100_000
# trials per launch: the whole campaign in one launch by default (1M trials x
# 16 private pages = 65 GiB of copy-on-write frames, well inside 288 GB of
# HBM): one campaign tail instead of one per chunk
PER_LAUNCH = int(sys.argv[5]) if len(sys.argv) > 5 else N
elf = open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb").read()
e = Engine(max_trials_per_launch=PER_LAUNCH)
e.load_elf(elf, [name])
g = e.golden_run()
e.set_campaign(SEED, REGS_PC, 1)
e.run_trials(0, min(PER_LAUNCH, N), want_outcomes=False)   # warm-up (buffers)
t0 = time.perf_counter()
out, h = e.run_trials(0, N)
wall = time.perf_counter() - t0
cls = np.bincount(out["cls"], minlength=6).tolist()
rec = {"workload": name, "trials": N, "trials_per_launch": PER_LAUNCH, "seed": hex(SEED), "golden_ninst": int(g.ninst),
       "wall_s": round(wall, 3), "trials_per_s": round(N / wall), "classes": dict(zip(
           ["masked", "sdc", "crash", "hang", "detected", "escape"], cls)),
       "escapes": escape_breakdown(out), "device_insts": int(h["device_insts"]),
       "guest_insts_gem5_equiv": int(out["ninst"].astype(np.uint64).sum())}
print(json.dumps(rec), flush=True)
# oracle check (checker only), in pieces with a progress line each
from oracle.pyoracle import Oracle  # noqa: E402
if CHECK >= N:
    idx = np.arange(N)
else:
    rng = np.random.default_rng(SEED)
    idx = np.sort(rng.choice(N, size=CHECK, replace=False))
sites = e.sample(0, N)[idx]
e.close()
o = Oracle(elf, name)
o.run_golden()
t1 = time.perf_counter()
bad = 0
piece = 50_000
for a in range(0, len(idx), piece):
    ref = o.run_trials(sites[a:a + piece], threads=16)
    bad += int((ref != out[idx[a:a + piece]]).sum())
    print(json.dumps({"progress": a + len(ref), "of": int(len(idx)), "mismatches": bad,
                      "s": round(time.perf_counter() - t1, 1)}), flush=True)
rec["oracle_check"] = {"checked": int(len(idx)), "mismatches": bad, "oracle_s": round(time.perf_counter() - t1, 2),
                       "threads": 16, "which": "all trials" if CHECK >= N else "seeded sample"}
print(json.dumps(rec), flush=True)
sys.exit(0 if bad == 0 else 1)
