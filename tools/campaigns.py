#!/usr/bin/env python3
"""Run the BASELINE.json campaign configs C1-C5 on one MI355X and write one
JSON summary (profiles/TAG_campaigns.json).  Each line: trials, seconds of
device time (sample + sort + interpreter + histogram, inputs resident),
trials/s, outcome classes, crash/escape sub-codes.

  C1 hello, 1k regfile flips
  C2 crc32 / qsort, 100k regfile+PC single-bit trials
  C3 intmix, one GPU's shard of the 1M-trial 8-GPU campaign (125k trials)
  C4 memory-word faults, bursts k = 1, 2, 4, 8 (copy-on-write guest pages)
  C5 SHREWD selective-replication sweep on crc32: protected register masks vs
     residual SDC rate (a fault on a protected register that is read before
     being overwritten is detected-by-replica)
  C5b SHREWD replication by instruction class: result faults (the value an
     instruction writes) on crc32 and qsort with protected gem5 OpClass sets
     (a replicated instruction's shadow execution detects the fault)
  C5c the same with SHREWD FU contention (fi_set_issue_model): a protected
     instruction is replicated only if its shadow found a free unit in the O3
     issue model of the golden run; deferred and priority shadows, the default
     pool and a pool with fewer ALUs
python tools/campaigns.py [TAG] [--only C5c]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from shrewd_amd import Engine  # noqa: E402
from shrewd_amd.fi import CLASS_NAMES, CRASH_NAMES, ESCAPE_NAMES, escape_breakdown  # noqa: E402

REGS = (1 << 32) - 2
PC = 1 << 32
MEM = 1 << 33
RESULT = 1 << 34
OPC = {"none": 0, "IntAlu": 1 << 1, "IntMult+IntDiv": (1 << 2) | (1 << 3), "IntAlu+IntMult+IntDiv": 0b1110,
       "MemRead+MemWrite (no shadow FU)": (1 << 52) | (1 << 53)}
# ABI register groups (x-register numbers)
MASKS = {"none": 0, "sp_ra_gp_tp": (1 << 1) | (1 << 2) | (1 << 3) | (1 << 4),
         "a0-a7": sum(1 << r for r in range(10, 18)),
         "s0-s11": sum(1 << r for r in (8, 9, *range(18, 28))),
         "t0-t6": sum(1 << r for r in (5, 6, 7, 28, 29, 30, 31)),
         "all+pc": REGS | PC}

_engines = {}


def engine(name):
    if name not in _engines:
        e = Engine(max_trials_per_launch=131072)
        e.load_elf(open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb").read(), [name])
        e.golden_run()
        _engines[name] = e
    return _engines[name]


FU_MODELS = {"off": None, "deferred": {}, "priority": {"priority_to_shadow": 1},
             "deferred, 4 IntALU 2 FP_ALU": {"IntALU": 4, "FP_ALU": 2},
             "priority, 4 IntALU 2 FP_ALU": {"IntALU": 4, "FP_ALU": 2, "priority_to_shadow": 1}}


def run(cfg, name, n, structs, burst=1, protect=0, seed=0x5EED0003, opc=0, fu=None):
    e = engine(name)
    e.set_issue_model(fu)
    e.set_campaign(seed, structs, burst)
    e.set_protect(protect)
    e.set_protect_opclasses(opc)
    e.run_trials(0, n)   # warm: code objects and work buffers sized for n
    t0 = time.perf_counter()
    out, h = e.run_trials(0, n)
    dt = time.perf_counter() - t0
    e.set_protect(0)
    e.set_protect_opclasses(0)
    extra = {}
    if fu is not None:
        _, st = e.shadow_map()
        extra = {"issue_model": fu, "issue_stats": st.as_dict()}
    e.set_issue_model(None)
    cls = h["counts"].sum(axis=(0, 1))
    rec = {"config": cfg, "workload": name, "golden_ninst": int(e.golden.ninst), "trials": n,
           "structures": hex(structs), "burst": burst, "protect_mask": hex(protect), "protect_opclasses": hex(opc),
           "seconds": dt,
           "trials_per_s": n / dt, **{CLASS_NAMES[i]: int(cls[i]) for i in range(6)},
           "crash_sub": {CRASH_NAMES.get(i, str(i)): int(h["crash_sub"][i]) for i in range(16) if h["crash_sub"][i]},
           "escape_sub": {ESCAPE_NAMES.get(i, str(i)): int(h["escape_sub"][i]) for i in range(8)
                          if h["escape_sub"][i]},
           "escapes": escape_breakdown(out),
           "sdc_rate": int(cls[1]) / n, **extra}
    print(json.dumps(rec), flush=True)
    return rec, out


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "r01"
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    recs = []
    if only == "C5c":
        c5c(recs)
        return dump(recs, tag)
    # C1 (its bit-exactness against the oracle: tests/test_gpu_parity.py)
    recs.append(run("C1", "hello", 1000, REGS, seed=0x5EED0001)[0])
    for w in ("crc32", "qsort"):
        recs.append(run("C2", w, 100_000, REGS | PC)[0])
    recs.append(run("C3", "intmix", 125_000, REGS | PC)[0])
    for w in ("crc32", "qsort"):
        for k in (1, 2, 4, 8):
            recs.append(run("C4", w, 100_000, MEM, burst=k)[0])
    for label, m in MASKS.items():
        r = run("C5", "crc32", 100_000, REGS | PC, protect=m)[0]
        r["mask_name"] = label
        recs.append(r)
    for w in ("crc32", "qsort"):
        for label, m in OPC.items():
            r = run("C5b", w, 100_000, RESULT, opc=m)[0]
            r["opclass_name"] = label
            recs.append(r)
    c5c(recs)
    dump(recs, tag)


def c5c(recs):
    for w in ("crc32", "qsort"):
        for label, fu in FU_MODELS.items():
            r = run("C5c", w, 100_000, RESULT, opc=OPC["IntAlu+IntMult+IntDiv"], fu=fu)[0]
            r["opclass_name"], r["fu_model"] = "IntAlu+IntMult+IntDiv", label
            recs.append(r)


def dump(recs, tag):
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"{tag}_campaigns.json"), "w") as f:
        json.dump(recs, f, indent=1)


if __name__ == "__main__":
    main()
