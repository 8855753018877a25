#!/usr/bin/env python3
"""Re-validate engine outcomes against a real gem5.

Needs a gem5.opt built with EXTRAS=src/gem5ext (SCons; not available in this
repo's build container, so this script has not been run here).  Steps:

  1. on a GPU host: sites = Engine.sample(0, N); out, _ = Engine.run_sites(sites);
     np.save("sites.npy", sites); np.save("outcomes.npy", out)
  2. on the gem5 host:
     python tools/gem5_revalidate.py --gem5 build/RISCV/gem5.opt --workload crc32.elf \\
         --cmd crc32 --sites sites.npy --outcomes outcomes.npy [--jobs 32]

Each site runs in its own gem5 process (configs/fi_gem5_trial.py with the
FaultInjector SimObject).  A trial is classified the way the engine does
(include/fi_engine.h): masked / SDC by exit code and stdout against the
golden run; hang by the max-insts exit; crash by gem5's own panic / fatal /
abort and the message naming the site (sub-codes of fi_engine.h).  Compared
fields: class, crash sub-code, exit code and committed instructions
(fi_outcome.detail, the final pc, is not observable from outside gem5).
Result faults (structure 34) have no gem5 hook and are skipped.

Tick-domain sites (fi_tick_site records, from Engine.sample_tick_sites /
run_tick_sites of an engine with cpu_type "timing"): each trial runs on
TimingSimpleCPU with the fault at its tick (--cpu timing --tick); trials the
engine reports as FI_ESC_TIMING are skipped, and --golden-ticks (the engine's
fi_tick_info.golden_ticks) is compared with the fault-free run's final tick.
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from shrewd_amd.fi import OUTCOME_DT, SITE_DT, TICK_SITE_DT  # noqa: E402

# gem5 message -> fi_engine.h crash sub-code (the sites named in fi_engine.h)
CRASH_PATTERNS = [
    (re.compile(r"Unknown instruction|UnknownInstFault"), 1),
    (re.compile(r"Illegal instruction|IllegalInstFault"), 2),
    (re.compile(r"[Pp]age table fault|GenericPageTableFault|Tried to access unmapped"), 3),
    (re.compile(r"[Ss]yscall .* out of range"), 4),
    (re.compile(r"unimplemented"), 5),
    (re.compile(r"readBlob|Failed to read|not all bytes"), 6),
    (re.compile(r"fd_array|Assertion .*fd"), 7),
    (re.compile(r"SIGTRAP|Trace/breakpoint trap"), 8),
    (re.compile(r"Maximum stack size"), 9),
    (re.compile(r"AMO.*cache line|crosses a cache line"), 10),
    (re.compile(r"curr_frag_id == 0"), 11),
]


def run_one(args, site, tag):
    d = tempfile.mkdtemp(prefix=f"fi_{tag}_")
    cmd = [args.gem5, "-d", d, os.path.join(ROOT, "configs", "fi_gem5_trial.py"), "--workload", args.workload,
           "--cmd", args.cmd, "--max-insts", str(args.max_insts), "--clock", args.clock]
    if args.tick_sites:
        cmd += ["--cpu", "timing"]
    if site is not None and args.tick_sites:
        cmd += ["--tick", str(int(site["tick"])), "--target", str(int(site["target"])),
                "--mask", hex(int(site["mask"]))]
    elif site is not None:
        cmd += ["--inst", str(int(site["inst"])), "--target", str(int(site["target"])),
                "--mask", hex(int(site["mask"])), "--addr", hex(int(site["addr"]))]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=args.timeout)
    rec = {"rc": p.returncode, "text": p.stdout[-4000:] + p.stderr[-4000:]}
    for line in reversed(p.stdout.splitlines()):
        if line.startswith("{"):
            rec.update(json.loads(line))
            break
    try:
        rec["stdout"] = open(os.path.join(d, "stdout"), "rb").read()
    except OSError:
        rec["stdout"] = b""
    m = None
    try:
        m = re.search(r"numInsts\s+(\d+)", open(os.path.join(d, "stats.txt")).read())
    except OSError:
        pass
    rec["ninst"] = int(m.group(1)) if m else -1
    return rec


def classify(rec, golden):
    """-> (cls, sub, exit_code) as the engine reports them."""
    if "cause" in rec and "max instruction count" in rec["cause"]:
        return 3, 1, 0
    if "cause" in rec and "exiting" in rec["cause"]:
        code = rec["code"] & 0xFF
        same = code == golden["code"] & 0xFF and rec["stdout"] == golden["stdout"]
        return (0 if same else 1), 0, code
    for pat, sub in CRASH_PATTERNS:
        if pat.search(rec["text"]):
            return 2, sub, {1: 134, 2: 134, 3: 134, 8: 133}.get(sub, 1)
    return 2, 0, rec["rc"] & 0xFF


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gem5", required=True)
    ap.add_argument("--workload", required=True)
    ap.add_argument("--cmd", default="")
    ap.add_argument("--sites", required=True)
    ap.add_argument("--outcomes", required=True)
    ap.add_argument("--jobs", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--clock", default="2GHz")
    ap.add_argument("--timeout", type=float, default=3600)
    ap.add_argument("--max-insts", type=int, default=0, help="0: 2 x golden numInst + 1000 (engine default)")
    ap.add_argument("--golden-ticks", type=int, default=0,
                    help="tick sites: the engine's golden run length in ticks, checked against gem5's")
    args = ap.parse_args()
    raw = np.load(args.sites)
    args.tick_sites = "tick" in (raw.dtype.names or ())
    sites = raw.astype(TICK_SITE_DT if args.tick_sites else SITE_DT)
    eng = np.load(args.outcomes).astype(OUTCOME_DT)
    golden = run_one(args, None, "golden")
    if args.max_insts == 0:
        args.max_insts = 2 * golden["ninst"] + 1000
    keep = [i for i in range(len(sites)) if sites[i]["target"] <= 33
            and not (args.tick_sites and eng[i]["cls"] == 5 and eng[i]["sub"] == 7)]
    with ThreadPoolExecutor(args.jobs) as ex:
        recs = list(ex.map(lambda i: run_one(args, sites[i], str(i)), keep))
    bad = []
    for i, rec in zip(keep, recs):
        cls, sub, code = classify(rec, golden)
        e = eng[i]
        want = (int(e["cls"]), int(e["sub"]) if e["cls"] == 2 else 0, int(e["exit_code"]))
        got = (cls, sub if cls == 2 else 0, code)
        if want != got or (rec["ninst"] >= 0 and rec["ninst"] != int(e["ninst"])):
            bad.append({"trial": int(sites[i]["trial"]), "engine": want, "gem5": got,
                        "engine_ninst": int(e["ninst"]), "gem5_ninst": rec["ninst"]})
    res = {"checked": len(keep), "mismatches": len(bad), "first": bad[:20]}
    if args.tick_sites and args.golden_ticks:
        res["golden_ticks"] = {"engine": args.golden_ticks, "gem5": golden.get("tick", -1)}
        if golden.get("tick", -1) != args.golden_ticks:
            bad.append("golden_ticks")
    print(json.dumps(res))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
