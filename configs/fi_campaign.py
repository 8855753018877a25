#!/usr/bin/env python3
"""Fault-injection campaign config script.

Same arguments either way:
  gem5.opt configs/fi_campaign.py --workload crc32.elf --trials 100000 ...
      -> instantiates the FaultCampaign SimObject (src/gem5ext) and calls its
         exported run() (gem5 built with EXTRAS=src/gem5ext);
  python configs/fi_campaign.py --workload crc32.elf --trials 100000 ...
      -> the same campaign through ctypes (shrewd_amd.FaultCampaign);
  torchrun --nproc-per-node 8 configs/fi_campaign.py --num-gpus 8 ...
      -> one rank per GPU, trial shards, RCCL all-reduce of the histogram.
Prints one JSON summary line (rank 0).
"""
import argparse
import json
import os
import sys
import time


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--workload", required=True)
    ap.add_argument("--cmd", default=None, help="comma-separated argv (default: the workload path)")
    ap.add_argument("--env", default="", help="comma-separated K=V")
    ap.add_argument("--checkpoint", default="", help="gem5 SE checkpoint directory to start the trials from")
    # Process.input / Process.executable (src/sim/Process.py:44,69), as se.py passes them
    ap.add_argument("--input", default="cin",
                    help="Process.input: 'cin' = the host's stdin (fd 0 reads escape), else a file fd 0 reads")
    ap.add_argument("--executable", default="",
                    help="Process.executable: what readlinkat('/proc/self/exe') resolves (default: the workload)")
    ap.add_argument("--trials", type=int, default=1000)
    ap.add_argument("--first-trial", type=int, default=0)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED0001)
    ap.add_argument("--structures", default="int_reg", help="comma list: int_reg,pc,mem,xN,<abi name>")
    ap.add_argument("--burst", type=int, default=1)
    ap.add_argument("--bits", default="", help="eligible lowest flipped bit positions: mask or ranges, e.g. 0-31,63")
    ap.add_argument("--protect-mask", type=lambda s: int(s, 0), default=0)
    ap.add_argument("--protect-opclasses", default="", help="comma list of gem5 OpClass names (IntAlu,IntMult,...)")
    ap.add_argument("--shadow-fu-model", action="store_true",
                    help="SHREWD FU contention: replicate only where the shadow finds a free unit")
    ap.add_argument("--priority-to-shadow", action="store_true", help="BaseO3CPU.priorityToShadow")
    ap.add_argument("--issue-width", type=int, default=8)
    ap.add_argument("--load-latency", type=int, default=2)
    ap.add_argument("--cpu-type", default="atomic", choices=["atomic", "timing"],
                    help="fault-site time coordinate: numInst (AtomicSimpleCPU) or ticks (TimingSimpleCPU on the "
                         "NoCache + SingleChannelDDR3_1600 board of simple_binary_run.py)")
    ap.add_argument("--num-gpus", type=int, default=1)
    ap.add_argument("--max-insts-factor", type=float, default=2.0)
    ap.add_argument("--private-pages", type=int, default=16)
    ap.add_argument("--output", default="")
    return ap.parse_args(argv)


def _split(s):
    return [x for x in (s or "").split(",") if x]


def run_gem5(a):
    import m5
    from m5.objects import FaultCampaign, Root
    camp = FaultCampaign(workload=a.workload, cmd=_split(a.cmd) or [a.workload], env=_split(a.env),
                         checkpoint=a.checkpoint, input=a.input, executable=a.executable,
                         trials=a.trials, first_trial=a.first_trial, seed=a.seed,
                         structures=_split(a.structures), bits=a.bits or "0-63", burst=a.burst,
                         protect_mask=a.protect_mask,
                         protect_opclasses=_split(a.protect_opclasses), shadow_fu_model=a.shadow_fu_model,
                         priority_to_shadow=a.priority_to_shadow, issue_width=a.issue_width,
                         load_latency=a.load_latency, num_gpus=a.num_gpus, max_insts_factor=a.max_insts_factor,
                         cpu_type=a.cpu_type,
                         private_pages=a.private_pages, output=a.output)
    root = Root(full_system=False, campaign=camp)
    m5.instantiate()
    root.campaign.run()
    print(root.campaign.summaryJson(), flush=True)
    # histogram(): the fi_histogram counters, flattened (include/fi_engine.h)
    print(len(root.campaign.histogram()), "histogram counters", flush=True)


def run_ctypes(a):
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, here)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from shrewd_amd import FaultCampaign
    c = FaultCampaign(a.workload, cmd=_split(a.cmd) or [a.workload], env=_split(a.env), trials=a.trials,
                      seed=a.seed, structures=_split(a.structures), burst=a.burst, protect_mask=a.protect_mask,
                      num_gpus=max(a.num_gpus, world), max_insts_factor=a.max_insts_factor, output=a.output,
                      device=local, private_pages=a.private_pages,
                      protect_opclasses=_split(a.protect_opclasses), bits=a.bits or None,
                      shadow_fu_model=a.shadow_fu_model, priority_to_shadow=a.priority_to_shadow, checkpoint=a.checkpoint,
                      issue_params={"issue_width": a.issue_width, "load_latency": a.load_latency},
                      input=a.input, executable=a.executable or None, cpu_type=a.cpu_type)
    t0 = time.perf_counter()
    c.run(first_trial=a.first_trial)
    dt = time.perf_counter() - t0
    if rank == 0:
        s = c.summary()
        s.update(seconds=dt, trials_per_s=s["trials"] / dt, num_gpus=world)
        print(json.dumps(s), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def main(argv=None):
    a = parse(argv)
    try:
        import m5  # noqa: F401  (present only when run by gem5.opt)
        in_gem5 = True
    except ImportError:
        in_gem5 = False
    (run_gem5 if in_gem5 else run_ctypes)(a)


if __name__ == "__main__" or __name__ == "__m5_main__":
    main()
