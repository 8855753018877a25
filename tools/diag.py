"""Interpreter diagnostics on the GPU: per-wave loop counters and timings.

python tools/diag.py [workload] [--trials N] [--flags F]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
from shrewd_amd import Engine  # noqa: E402

REGS_PC = ((1 << 32) - 2) | (1 << 32)
ap = argparse.ArgumentParser()
ap.add_argument("workload", nargs="?", default="crc32")
ap.add_argument("--trials", type=int, nargs="*", default=[64, 6400, 100000])
ap.add_argument("--flags", type=int, default=0)
ap.add_argument("--interval", type=int, default=0)
ap.add_argument("--epoch", type=int, default=0)
ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED0002)
ap.add_argument("--converged", action="store_true", help="also time one converged wave from process start")
a = ap.parse_args()
name = a.workload
e = Engine(max_trials_per_launch=200000, flags=a.flags, snapshot_interval=a.interval, epoch_iters=a.epoch)
e.load_elf(open(f"workloads/{name}.elf", "rb").read(), [name])
g = e.golden_run()
gms = e.last_kernel_ms()
st = e.debug_stats()
clk = int(st[20]) / max(1, int(st[21])) * 100.0
print(json.dumps({"golden_ninst": g.ninst, "golden_ms": gms, "golden_ns_per_inst": gms * 1e6 / max(1, g.ninst),
                  "snapshots": g.snapshots, "interval": g.snapshot_interval, "frames": g.snapshot_frames, "capture_pass_clock_mhz": round(clk, 1),
                  "cycles_per_inst_capture_pass": int(st[20]) / max(1, g.ninst),
                  "prof_cycles_per_inst": [round(int(st[24 + k]) / max(1, g.ninst), 1) for k in range(4)],
                  "tx_blocks": g.translated_blocks, "tx_insts": g.translated_insts, "tx_us": g.translate_us,
                  "tx_status": e.translate_status()[:3000]}),
      flush=True)
os.makedirs("gpurun_out", exist_ok=True)
with open(f"gpurun_out/tx_{name}.inc", "w") as f:
    f.write(e.debug_translation())
_pre, _tr, _lo = e.debug_golden_trace()
np.savez(f"gpurun_out/golden_{name}.npz", pre=_pre, trace=_tr, text_lo=np.uint64(_lo))
e.set_campaign(a.seed, REGS_PC, 1)
for n in a.trials:
    sites = e.sample(0, n)
    nofault = sites.copy(); nofault["inst"] = 1 << 40
    for label, s in (("nofault", nofault), ("faults", sites)):
        out, h = e.run_sites(s)
        st = e.debug_stats()
        ms = e.last_kernel_ms()
        waves = (n + 63) // 64
        print(json.dumps({"n": n, "kind": label, "kernel_ms": round(ms, 3), "trials_per_s": n / ms * 1e3,
                          "iters_per_wave": int(st[6]) / waves, "max_iter_wave": int(st[10]),
                          "lane_insts": int(st[7]), "lanes_per_iter": round(int(st[7]) / max(1, int(st[6])), 2),
                          "slow": int(st[8]), "minpc": int(st[9]), "checks": int(st[11]), "early": int(st[12]),
                          "skipped_prefix": int(st[14]), "cow_pages": int(st[2]),
                          "ns_per_iter_slowest_wave": round(ms * 1e6 / max(1, int(st[10])), 1),
                          "clock_mhz": round(int(st[20]) / max(1, int(st[21])) * 100.0, 1),
                          "wave0_cycles": int(st[20]), "survivors": e.debug_epochs()[:4],
                          "tx_insts": int(st[16]), "tx_entries": int(st[17]),
                          "slowest": {"iters": int(st[18]) >> 32, "tx_permille": (int(st[18]) >> 20) & 0xFFF,
                                      "tx_entries": int(st[18]) & 0xFFFFF, "slow": int(st[19]) & 0xFFFFFFFF},
                          "prof_cycles_per_iter": [round(int(st[24 + k]) / max(1, int(st[6])), 1) for k in range(4)],
                          "prof_slow_cycles_per_slow": [round(int(st[24 + k]) / max(1, int(st[8])), 1) for k in range(4, 8)],
                          "classes": np.bincount(out["cls"], minlength=6).tolist()}), flush=True)
        wv = e.debug_waves(waves).astype(np.int64)
        top = np.argsort(-wv[:, 0])[:4]
        print(json.dumps({"longest_waves": [{"wave": int(w), "ms": round(wv[w, 0] / 2.4e6, 2), "iters": int(wv[w, 1]),
                                             "tx": int(wv[w, 2]), "slow": int(wv[w, 3]),
                                             "ns_per_iter": round(wv[w, 0] / 2.4 / max(1, wv[w, 1]), 1)}
                                            for w in top]}), flush=True)
        if label == "faults" and n == a.trials[-1]:
            np.save("gpurun_out/waves.npy", wv)
            np.save("gpurun_out/outcomes.npy", out)
            np.save("gpurun_out/sites.npy", s)

if a.converged:
    from shrewd_amd.fi import CFG_NO_SNAPSHOT_START, CFG_NO_TRANSLATE
    for fl, label in ((CFG_NO_SNAPSHOT_START, "translated"), (CFG_NO_SNAPSHOT_START | CFG_NO_TRANSLATE, "interpreter")):
        e2 = Engine(max_trials_per_launch=200000, flags=fl)
        e2.load_elf(open(f"workloads/{name}.elf", "rb").read(), [name])
        g2 = e2.golden_run()
        e2.set_campaign(0x5EED0002, REGS_PC, 1)
        s = e2.sample(0, 64); s["inst"] = 1 << 40
        e2.run_sites(s)
        ms = e2.last_kernel_ms()
        st = e2.debug_stats()
        print(json.dumps({"converged_wave_from_start": label, "kernel_ms": round(ms, 3),
                          "ns_per_inst": round(ms * 1e6 / g2.ninst, 1),
                          "cycles_per_inst": round(int(st[20]) / g2.ninst, 1), "tx_insts": int(st[16]),
                          "tx_entries": int(st[17]), "status": e2.translate_status()[:200]}), flush=True)
        e2.close()
