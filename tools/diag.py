"""Interpreter diagnostics on the GPU: per-wave loop counters and timings."""
import sys, os, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch  # noqa
from shrewd_amd import Engine

REGS_PC = ((1 << 32) - 2) | (1 << 32)
name = sys.argv[1] if len(sys.argv) > 1 else "crc32"
e = Engine(max_trials_per_launch=200000)
e.load_elf(open(f"workloads/{name}.elf", "rb").read(), [name])
g = e.golden_run()
st = e.debug_stats()
print(json.dumps({"golden_ninst": g.ninst, "golden_ms": e.last_kernel_ms(), "golden_iters": int(st[6]),
                  "golden_ns_per_iter": e.last_kernel_ms() * 1e6 / max(1, int(st[6]))}))
e.set_campaign(0x5EED0002, REGS_PC, 1)
for n in (64, 6400, 100000):
    # trials whose site lies beyond the end: pure golden lanes, no divergence
    sites = e.sample(0, n)
    nofault = sites.copy(); nofault["inst"] = 1 << 40
    for label, s in (("nofault", nofault), ("faults", sites)):
        out, h = e.run_sites(s)
        st = e.debug_stats()
        ms = e.last_kernel_ms()
        waves = (n + 63) // 64
        print(json.dumps({"n": n, "kind": label, "kernel_ms": ms, "iters": int(st[6]), "max_iter_wave": int(st[10]),
                          "iters_per_wave": int(st[6]) / waves, "lane_insts": int(st[7]),
                          "lanes_per_iter": int(st[7]) / max(1, int(st[6])), "slow": int(st[8]), "minpc": int(st[9]),
                          "ns_per_iter_slowest_wave": ms * 1e6 / max(1, int(st[10])),
                          "classes": np.bincount(out["cls"], minlength=6).tolist()}))

if os.environ.get("SHREWD_FI_LIB", "").endswith("_diag.so"):
    e.set_campaign(0x5EED0002, REGS_PC, 1)
    g = e.golden_run()
    st = e.debug_stats()
    seg = ["A_requests", "B_events", "C_leader", "D_fetch_decode", "E_execute", "F_memaccess"]
    it = max(1, int(st[6]))
    print(json.dumps({"golden_cycles_per_iter_by_segment": {seg[k]: int(st[16 + k]) / it for k in range(6)}}))
    sites = e.sample(0, 100000); nof = sites.copy(); nof["inst"] = 1 << 40
    e.run_sites(nof); st = e.debug_stats(); it = max(1, int(st[6]))
    print(json.dumps({"nofault100k_cycles_per_iter_by_segment": {seg[k]: int(st[16 + k]) / it for k in range(6)}}))
