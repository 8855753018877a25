#!/usr/bin/env python3
"""Per-kernel summary of a tools/gpu/kernel_prof.sh run:
python tools/kernel_prof_summary.py TAG > profiles/TAG_kernel_prof.json

For each trial kernel (64-lane, solo): dispatches, average duration (kernel
trace), and per-dispatch averages of every counter; derived: resident waves
per SIMD (SQ_WAVE_CYCLES counts quad-cycles, MI355X_MICROARCH.md), issue-slot
use (instructions / (SIMDs x cycles)), and the share of wave-cycles spent
issuing, waiting on dependencies (SQ_WAIT_INST_ANY) and parked (SQ_WAIT_ANY).
"""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
g = os.path.join(ROOT, "gpurun_out")
SIMDS = 1024


def short(name):
    return name.split("(")[0].strip()


trace = defaultdict(list)
with open(os.path.join(g, f"kp_trace_{tag}", "trace_kernel_trace.csv")) as f:
    for r in csv.DictReader(f):
        if "fi_trial_kernel" in r["Kernel_Name"] and int(r.get("Grid_Size_X", r.get("Grid_Size", "0")) or 0) > 64:
            trace[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
cnt = defaultdict(lambda: defaultdict(list))
for p in ("a", "b"):
    path = os.path.join(g, f"kp_{p}_{tag}", f"{p}_counter_collection.csv")
    if not os.path.exists(path):
        continue
    per = defaultdict(float)
    with open(path) as f:
        for r in csv.DictReader(f):
            if "fi_trial_kernel" not in r["Kernel_Name"] or int(r["Grid_Size"]) <= 64:
                continue
            per[(short(r["Kernel_Name"]), r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, d, c), v in per.items():
        cnt[k][c].append(v)
out = {"tag": tag, "kernels": {}}
for k in sorted(set(trace) | set(cnt)):
    durs = trace.get(k, [])
    avg = {c: sum(v) / len(v) for c, v in cnt[k].items()}
    rec = {"dispatches": len(durs), "avg_ms": round(sum(durs) / len(durs), 3) if durs else None,
           "counters_per_dispatch": {c: round(v) for c, v in sorted(avg.items())}}
    cyc = avg.get("GRBM_GUI_ACTIVE")
    if cyc:
        cyc /= 8   # per XCD (MI355X_MICROARCH.md)
        if "SQ_WAVE_CYCLES" in avg:
            rec["waves_per_simd"] = round(4 * avg["SQ_WAVE_CYCLES"] / (SIMDS * cyc), 3)
        insts = sum(avg.get(c, 0) for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS"))
        rec["issue_frac"] = round(insts / (SIMDS * cyc), 4)
        rec["salu_per_cu_cycle"] = round(avg.get("SQ_INSTS_SALU", 0) / (256 * cyc), 4)
    wc = avg.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_SCA",
                  "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SMEM"):
            if c in avg:
                rec["share_" + c[3:].lower()] = round(avg[c] / wc, 3)
    out["kernels"][k] = rec
print(json.dumps(out, indent=1))
