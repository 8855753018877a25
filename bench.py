#!/usr/bin/env python3
"""bench.py -- fault-injection campaign throughput on MI355X.

Metric (BASELINE.json): fault-injection trials/sec (whole node) and guest
inst/sec.  Workload (configs[1]): the RV64 MiBench-style CRC32 kernel,
100k register-file + PC single-bit trials per GPU, seeded sites.

One step = one campaign pass over a batch of `--trials` trials per GPU:
device-side site sampling, sort by inject time, the interpreter kernel (each
trial starts from the golden snapshot at or before its inject time and ends
at exit / crash / hang, or early as masked once its whole state equals a later
golden snapshot -- exact), outcome histogram, and the RCCL
all-reduce of the histogram (the campaign's only exchange; N > 1).
Trials shard by id across ranks (weak scaling: per-GPU work fixed).

The same line carries the other C2 workload (qsort, 100k trials per GPU) and
C3's per-GPU shard (intmix, 125k trials per GPU) under "workloads", each with
its own steps, roofline, cold start and (N = 1) a >= 20k-trial parity leg.

Launch: python bench.py [--gpus 1] [--steps 5] [--warmup 1]
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
REGS_PC = ((1 << 32) - 2) | (1 << 32)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="crc32")
    ap.add_argument("--trials", type=int, default=100_000, help="trials per GPU per step")
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED0002)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--parity-trials", type=int, default=0,
                    help="check at least this many trial ids of the headline workload against the oracle")
    ap.add_argument("--workloads", default="qsort:100000:5,intmix:125000:2",
                    help="further workloads on the same line, name:trials_per_gpu:steps (\"\" = none)")
    ap.add_argument("--extra-parity", type=int, default=20000,
                    help="trial ids of each further workload checked against the oracle (N = 1)")
    ap.add_argument("--lanes", type=int, default=0, help="trials per 64-lane wave (0: engine default)")
    ap.add_argument("--resume-lanes", type=int, default=0, help="trials per wave in resumed epochs (0: default)")
    ap.add_argument("--epochs", type=int, default=0, help="epochs per chunk (0: default)")
    ap.add_argument("--epoch-iters", type=int, default=0, help="first epoch's iterations per wave (0: default)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1: the histogram reduce's backend (nccl = RCCL; gloo reduces a host copy -- tests)")
    ap.add_argument("--device-index", type=int, default=-1,
                    help="HIP device of this rank (default LOCAL_RANK; tests run two ranks on device 0)")
    ap.add_argument("--hist-out", default="", help="rank 0: save the headline workload's node histogram (.npy)")
    return ap.parse_args()


def host_cores():
    """Host CPUs this process may run on (the cgroup/affinity share, capped by
    OMP_NUM_THREADS when the box sets it), the machine's total, and the CPU model."""
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        avail = min(avail, int(omp))
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return max(1, avail), os.cpu_count() or 1, model


def cpu_baseline(elf: bytes, argv0: str, seed: int, budget_s: float, min_trials: int = 0):
    """The oracle (plain-C restatement of gem5 RV64 SE, test infrastructure)
    on every host core this process may use, same campaign, bounded sample.
    Like a serial gem5 run, the oracle runs every trial from process start to
    its end (no golden snapshots, no early exit).  Returns the baseline record
    and the sampled trials' outcomes (kept for the parity check)."""
    from oracle.pyoracle import Oracle
    threads, machine_cpus, model = host_cores()
    o = Oracle(elf, argv0)
    o.run_golden()
    calib = o.sample(seed, 0, 64 * threads, REGS_PC, 1)
    t0 = time.perf_counter()
    o.run_trials(calib, threads=threads)
    dt = max(time.perf_counter() - t0, 1e-3)
    n = int(min(2_000_000, max(len(calib), min_trials, len(calib) * budget_s / dt)))
    sites = o.sample(seed, 0, n, REGS_PC, 1)
    t0 = time.perf_counter()
    out = o.run_trials(sites, threads=threads)
    dt = time.perf_counter() - t0
    insts = int(out["ninst"].sum())
    o.close()
    rec = {"value": n / dt, "unit": "trials/s", "cores": threads, "kind": "port",
           "sample": f"first {n} trials of the same {argv0} campaign (seed {seed:#x}, regs+pc), "
                     f"oracle/rv64se.c with {threads} pthreads, each trial from process start to its end "
                     f"(no snapshots, no early exit), {dt:.1f}s wall",
           "host_cpus_total": machine_cpus, "cpu_model": model,
           "guest_inst_per_s": insts / dt}
    return rec, out


def load_traffic(path, workload, trials, lanes):
    """HBM bytes per launch from the PMC passes of the same configuration
    (profiles/pmc_traffic.json), if they were taken on it."""
    try:
        with open(path) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        return {}
    for ent in [tj] + list(tj.get("workloads", {}).values()):
        if ent.get("workload") == workload and ent.get("trials") == trials and ent.get("lanes_per_wave", 64) == lanes:
            return ent
    return {}


def run_workload(a, name, T, steps, warmup, rank, world, dev, cpu_seconds, min_parity):
    """One workload's bench record: cold start (golden run, the first campaign
    step while the translated kernels build in the background), then `warmup`
    + `steps` timed steps of T trials per GPU on the translated kernels, the
    per-kernel roofline, and (N = 1) the CPU baseline + parity leg."""
    import torch
    import torch.distributed as dist
    from shrewd_amd import ESCAPE_NAMES, HIST_DT, Engine
    from shrewd_amd.fi import CFG_JIT_NO_CACHE, escape_breakdown
    with open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb") as f:
        elf = f.read()
    # no code-object cache: the cold start below is the one a fresh campaign pays
    eng = Engine(device=dev.index, max_trials_per_launch=max(T, 1024), lanes_per_wave=a.lanes,
                 resume_lanes=a.resume_lanes, epoch_iters=a.epoch_iters, epochs=a.epochs, flags=CFG_JIT_NO_CACHE)
    lanes = eng.config()["lanes_per_wave"]
    # ---- cold start: load + golden run (+ snapshots, liveness, translation
    # text) until trials can run; the first step runs while the translated
    # kernels build (static kernels, 16k-trial chunks, switching when it lands)
    t0 = time.perf_counter()
    eng.load_elf(elf, [name])
    g = eng.golden_run(wait_translation=False)
    golden_s = time.perf_counter() - t0
    eng.set_campaign(a.seed, REGS_PC, 1)
    t1 = time.perf_counter()
    eng.run_trials(rank * T, T, want_outcomes=False)
    first_step_s = time.perf_counter() - t1
    g = eng.wait_translation()
    jit_ready_s = time.perf_counter() - t0
    cold = {"golden_s": golden_s, "first_step_s": first_step_s,
            "campaign_s": golden_s + first_step_s, "campaign_trials_per_s": T / (golden_s + first_step_s),
            "translated_ready_s": jit_ready_s, "translate_us": int(g.translate_us),
            "translated_blocks": int(g.translated_blocks),
            "note": "load + golden run, then one step of T trials through the product path while the "
                    "translated kernels build in the background (no code-object cache)"}

    d_out = torch.empty(T * 16, dtype=torch.uint8, device=dev)
    hist_words = HIST_DT.itemsize // 8
    d_hist = torch.zeros(hist_words, dtype=torch.int64, device=dev)
    d_hist_node = torch.zeros_like(d_hist)
    # one dedicated stream for engine kernels, histogram copies and RCCL
    tstream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(tstream)
    stream = tstream.cuda_stream

    gloo = world > 1 and dist.get_backend() == "gloo"

    def step():
        d_hist.zero_()
        eng.run_trials_device(rank * T, T, d_out.data_ptr(), d_hist.data_ptr(), stream)
        d_hist_node.copy_(d_hist)
        if world > 1 and not gloo:
            dist.all_reduce(d_hist_node)      # RCCL over xGMI: outcome histogram only
        elif gloo:                            # (tests: a host copy through gloo)
            h = d_hist_node.cpu()
            dist.all_reduce(h)
            d_hist_node.copy_(h)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    eng.kernel_timer_reset()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=None if gloo else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    node_h = np.frombuffer(d_hist_node.cpu().numpy().tobytes(), HIST_DT)[0]
    if rank == 0 and a.hist_out and name == a.workload:
        np.save(a.hist_out, np.array([node_h], HIST_DT))
    if rank != 0:
        eng.close()
        return None
    trials_total = world * T * steps
    # roofline per trial kernel, per launch:
    # algorithmic bytes = fetched instruction bytes + load/store bytes of the
    # guest instructions the kernel executed + 4096 B per copy-on-write page
    # it made, and for the 64-lane kernel (every trial starts there) 264 B of
    # initial state + 16 B of outcome per trial; counted on the device per
    # kernel (DevCtx::stats[40..51]) over the last step -- every step runs
    # the same trial ids, so the last step's counts are every step's.
    # Duration = the mean of that kernel's dispatches (HIP events on its
    # stream); the dominant kernel is the one with the most device time.
    st = eng.debug_stats()
    kinds, dms = eng.debug_dispatch_kinds(), eng.debug_dispatch_ms()
    spans = eng.debug_dispatch_span_ms()
    tx = eng.translate_status() == ""
    names = (["fi_trial_kernel_tx", "fi_trial_kernel_tx_solo", "fi_trial_kernel_tx_solo_odd"] if tx
             else ["fi_trial_kernel", "fi_trial_kernel_solo", "fi_trial_kernel_solo_odd"])
    tj = load_traffic(a.traffic_json, name, T, lanes)
    per_kernel = {}
    for k, kname in enumerate(names):
        ms_k = [m for m, kk in zip(dms, kinds) if kk == k]
        if not ms_k:
            continue
        busy_k = [m for m, kk in zip(spans, kinds) if kk == k]
        disp = len(ms_k) / steps
        b = int(st[40 + 4 * k]) + int(st[41 + 4 * k]) + 4096 * int(st[42 + 4 * k]) + (T * (264 + 16) if k == 0 else 0)
        avg_ms = sum(ms_k) / len(ms_k)
        per_launch = b / disp
        ach = per_launch / (avg_ms / 1e3) / 1e9
        tk = tj.get("per_kernel", {}).get(kname, {})
        per_kernel[kname] = {"avg_kernel_ms": avg_ms, "dispatches_per_step": disp,
                             "ms_per_step": avg_ms * disp, "algorithmic_bytes_per_launch": per_launch,
                             "achieved": ach, "frac": ach / HBM_PEAK_GBS,
                             "device_insts_per_launch": int(st[43 + 4 * k]) / disp,
                             "traffic": tk.get("hbm_bytes_per_launch"), "issue": tk.get("issue"),
                             # the dispatch's own work on the device (first to last stamp of
                             # the waves that ran a trial): the HIP-event / trace time of the
                             # solo-odd kernel also holds its wait for CU slots the solo
                             # kernel on the other stream occupies
                             "device_busy_ms": sum(busy_k) / len(busy_k) if busy_k else None}
    dom = max(per_kernel, key=lambda n: per_kernel[n]["ms_per_step"])
    D = per_kernel[dom]
    cls = node_h["counts"].sum(axis=(0, 1))
    rec = {
        "value": trials_total / elapsed,
        "ms_per_step": elapsed / steps * 1e3,
        "steps": steps, "warmup": warmup,
        "config": {"workload": f"{name} (RV64, {g.ninst} golden insts), {T} single-bit x1..x31+pc trials "
                               f"per GPU per step",
                   "trials_per_gpu": T, "seed": hex(a.seed), "structures": "x1-x31,pc", "burst": 1,
                   "lanes_per_wave": lanes,
                   "parallelism": f"trial-sharded x{world}, RCCL histogram all-reduce"},
        # gem5-equivalent: each trial's numInst at its end, as a serial gem5
        # run commits it (restored snapshot prefix and skipped golden suffix
        # of early-masked trials included); device: instructions the GPU
        # actually executed
        "guest_inst_per_s_gem5_equiv": int(node_h["guest_insts"]) * steps / elapsed,
        "device_inst_per_s": int(node_h["device_insts"]) * steps / elapsed,
        "roofline": {"bound": "hbm", "achieved": D["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": D["frac"], "traffic": D["traffic"], "kernel": dom,
                     "avg_kernel_ms": D["avg_kernel_ms"], "dispatches_per_step": D["dispatches_per_step"],
                     "algorithmic_bytes_per_launch": D["algorithmic_bytes_per_launch"],
                     # the roof that binds: issue slots (SQ counters of the same
                     # command, profiles/)
                     "issue": D["issue"], "per_kernel": per_kernel},
        "outcomes": {n: int(cls[i]) for i, n in enumerate(["masked", "sdc", "crash", "hang", "detected", "escape"])},
        "escape_sub": {ESCAPE_NAMES.get(i, str(i)): int(node_h["escape_sub"][i]) for i in range(8)
                       if node_h["escape_sub"][i]},
        "cold_start": cold,
        "golden_s": golden_s,
        "parity": None,
        "cpu_baseline": None,
    }
    if world == 1 and not a.no_cpu_baseline:
        rec["cpu_baseline"], ref = cpu_baseline(elf, name, a.seed, cpu_seconds, min_parity)
        rec["cold_start"]["campaign_vs_cpu_baseline"] = cold["campaign_trials_per_s"] / rec["cpu_baseline"]["value"]
        # the same trial ids through the device (the timed campaign's first
        # trials): every outcome must equal the oracle's, bit for bit
        dev_out, _ = eng.run_trials(0, len(ref))
        rec["escapes_in_checked"] = escape_breakdown(dev_out)
        rec["parity"] = {"checked": int(len(ref)), "mismatches": int((dev_out != ref).sum()),
                         "against": "oracle/rv64se.c, trial ids [0, checked) of the benched campaign"}
    eng.close()
    return rec


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    if a.device_index >= 0:
        local = a.device_index
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    head = run_workload(a, a.workload, a.trials, a.steps, a.warmup, rank, world, dev, a.cpu_seconds,
                        a.parity_trials)
    # the other C2 / C3 workloads on the same line (BASELINE.json configs[1], [2]):
    # qsort 100k trials per GPU, intmix 125k per GPU (C3's 1M over 8 GPUs)
    extra = {}
    for spec in [w for w in a.workloads.split(",") if w]:
        name, _, rest = spec.partition(":")
        T, _, steps = rest.partition(":")
        T, steps = int(T or a.trials), int(steps or a.steps)
        if name == a.workload:
            continue
        extra[name] = run_workload(a, name, T, steps, 1, rank, world, dev, 2.0, a.extra_parity)
    if rank == 0:
        res = {
            "metric": "fault-injection trials/sec (whole node)",
            "value": head["value"],
            "unit": "trials/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (seeded SplitMix64 fault sites over a hand-assembled RV64 ELF)",
        }
        res.update({k: v for k, v in head.items() if k not in ("value", "ms_per_step", "steps", "warmup")})
        res["workloads"] = extra
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
