#!/usr/bin/env python3
"""Summarise a tools/gpu_profile.sh run into profiles/.

Reads gpurun_out/{bench,prof_trace,prof_fetch,prof_write,prof_sq}_TAG and writes
  profiles/TAG_bench.json           the bench JSON line
  profiles/TAG_kernel_stats.csv     rocprofv3 --kernel-trace --stats summary
  profiles/TAG_pmc.json             per-launch PMC values of each trial kernel
  profiles/pmc_traffic.json         HBM bytes + issue roof per launch and kernel (read by bench.py)

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes): on gfx950
FETCH_SIZE reports half the bytes of coalesced reads (MI355X_MICROARCH.md,
"HBM [CDNA4]").  Only the campaign launches (grid > 64 lanes) are averaged;
the one-lane golden run is excluded.
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("fi_trial_kernel_tx", "fi_trial_kernel_tx_solo", "fi_trial_kernel_tx_solo_odd",
           "fi_trial_kernel", "fi_trial_kernel_solo")
SQ = ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES",
      "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE")
SQB = ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VALU",
       "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SMEM", "SQ_INSTS_VMEM")


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def kname(r):
    n = r["Kernel_Name"].split("(")[0].strip()
    return n if n in KERNELS else None


def per_launch(rs, counter, kernel):
    vals = [float(r["Counter_Value"]) for r in rs
            if kname(r) == kernel and r["Counter_Name"] == counter and int(r["Grid_Size"]) > 64]
    return sum(vals) / len(vals) if vals else None, len(vals)


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    g = os.path.join(ROOT, "gpurun_out")
    p = os.path.join(ROOT, "profiles")
    os.makedirs(p, exist_ok=True)
    with open(os.path.join(g, f"bench_{tag}.json")) as f:
        bench = json.loads(f.read().strip().splitlines()[-1])
    with open(os.path.join(p, f"{tag}_bench.json"), "w") as f:
        json.dump(bench, f, indent=1)
    shutil.copy(os.path.join(g, f"prof_trace_{tag}", "trace_kernel_stats.csv"),
                os.path.join(p, f"{tag}_kernel_stats.csv"))
    fr = rows(os.path.join(g, f"prof_fetch_{tag}", "fetch_counter_collection.csv"))
    wr = rows(os.path.join(g, f"prof_write_{tag}", "write_counter_collection.csv"))
    sr = rows(os.path.join(g, f"prof_sq_{tag}", "sq_counter_collection.csv"))
    # the wait / active-instruction pass (tools/gpu_profile.sh), when taken
    sqb_path = os.path.join(g, f"prof_sqb_{tag}", "sqb_counter_collection.csv")
    sbr = rows(sqb_path) if os.path.exists(sqb_path) else []
    trace = rows(os.path.join(g, f"prof_trace_{tag}", "trace_kernel_trace.csv"))
    wl = bench["config"]["workload"].split()[0]
    bk = bench["roofline"].get("per_kernel", {})
    out = {"tag": tag, "dominant": bench["roofline"].get("kernel"), "per_kernel": {}}
    for kn in KERNELS:
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace
                if kname(r) == kn and int(r["Grid_Size_X"]) > 64]
        if not durs:
            continue
        fetch, nf = per_launch(fr, "FETCH_SIZE", kn)
        write, nw = per_launch(wr, "WRITE_SIZE", kn)
        sq = {name: per_launch(sr, name, kn)[0] for name in SQ}
        for name in SQB:
            if sbr:
                sq[name] = per_launch(sbr, name, kn)[0]
        if sq.get("SQ_WAIT_INST_ANY") is not None and sq.get("SQ_WAVE_CYCLES"):
            # shares of wave-cycles (both counted in quad-cycles per wave)
            sq["share_wait_inst_any"] = sq["SQ_WAIT_INST_ANY"] / sq["SQ_WAVE_CYCLES"]
            sq["share_wait_any"] = sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"]
        if sq.get("GRBM_GUI_ACTIVE") and sq.get("SQ_INSTS_SALU") is not None:
            sq["salu_per_cu_cycle"] = sq["SQ_INSTS_SALU"] / (256 * sq["GRBM_GUI_ACTIVE"] / 8)
        hbm = (2 * fetch + write) * 1024 if fetch is not None and write is not None else None
        # issue roof: instructions issued per SIMD-cycle (MI355X: 256 CUs x 4
        # SIMDs; GRBM_GUI_ACTIVE sums the 8 XCDs, SQ_WAVE_CYCLES counts quad-cycles)
        issue = None
        if sq.get("GRBM_GUI_ACTIVE") and sq.get("SQ_INSTS_VALU") is not None:
            cyc = sq["GRBM_GUI_ACTIVE"] / 8
            simds = 1024
            issue = {"valu_frac": sq["SQ_INSTS_VALU"] / (simds * cyc),
                     "salu_frac": sq["SQ_INSTS_SALU"] / (simds * cyc),
                     "waves_per_simd": sq["SQ_WAVE_CYCLES"] * 4 / cyc / simds,
                     "clock_ghz": cyc / (sum(durs) / len(durs)),
                     "source": f"profiles/{tag}_pmc.json"}
        b = bk.get(kn, {})
        trace_ms = sum(durs) / len(durs) / 1e6
        alg = b.get("algorithmic_bytes_per_launch")
        out["per_kernel"][kn] = {
            "launches_fetch": nf, "launches_write": nw, "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
            "hbm_bytes_per_launch": hbm, "trace_avg_ms": trace_ms, "trace_launches": len(durs),
            "bench_avg_kernel_ms": b.get("avg_kernel_ms"), "algorithmic_bytes_per_launch": alg,
            # the roofline fraction recomputed from the rocprofv3 trace's mean duration
            "frac_from_trace": (alg / (trace_ms / 1e3) / 1e9 / 8000.0) if alg else None,
            "sq": sq, "issue": issue}
    with open(os.path.join(p, f"{tag}_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    # one entry per workload (bench.py looks its own up); the headline
    # workload's entry also stays at the top level
    path = os.path.join(p, "pmc_traffic.json")
    try:
        with open(path) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        tj = {}
    ent = {"tag": tag, "workload": wl, "trials": bench["config"]["trials_per_gpu"],
           "lanes_per_wave": bench["config"].get("lanes_per_wave", 64),
           "per_kernel": {k: {"hbm_bytes_per_launch": v["hbm_bytes_per_launch"], "issue": v["issue"]}
                          for k, v in out["per_kernel"].items()},
           "source": f"profiles/{tag}_pmc.json"}
    wls = tj.get("workloads", {})
    if tj.get("workload"):
        wls.setdefault(tj["workload"], {k: v for k, v in tj.items() if k != "workloads"})
    wls[wl] = ent
    top = ent if wl == "crc32" or not tj.get("workload") else {k: v for k, v in tj.items() if k != "workloads"}
    with open(path, "w") as f:
        json.dump(dict(top, workloads=wls), f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
