"""One fault-injection trial inside a real gem5 (re-validation harness).

Run by gem5.opt built with EXTRAS=src/gem5ext, one process per site:

  gem5.opt -d OUT configs/fi_gem5_trial.py --workload crc32.elf --cmd crc32 \\
      --inst 1234 --target 10 --mask 0x20 [--addr A] --max-insts 130236

(no --target: the golden run).  SE mode, RISC-V AtomicSimpleCPU with its
ports on the memory bus and no caches, the configuration the engine models
(the reference's tests/gem5/stdlib/configs/simple_binary_run.py with
NoCache()).  The FaultInjector (src/gem5ext/FaultInjector.py) applies the
site at the top of the first tick with numInst >= inst.  The simulated
process's stdout/stderr go to OUT/stdout and OUT/stderr; the last line
printed is a JSON record {cause, code}; committed instructions are in
OUT/stats.txt.  tools/gem5_revalidate.py drives it and classifies.

--cpu timing --tick T: the tick-domain trial (the engine's fi_run_tick_sites)
on the reference run script's own board (tests/gem5/se_mode/hello_se/configs/
simple_binary_run.py: SimpleBoard at 3 GHz, NoCache, SingleChannelDDR3_1600,
a TimingSimpleCPU); the FaultInjector flips at tick T before every other
event of that tick.
"""
import argparse
import json
import os

import m5
from m5.objects import (AddrRange, FaultInjector, MemCtrl, DDR4_2400_8x8, Process, Root, RiscvAtomicSimpleCPU,
                        SEWorkload, SrcClockDomain, System, SystemXBar, VoltageDomain)

ap = argparse.ArgumentParser()
ap.add_argument("--workload", required=True)
ap.add_argument("--cmd", default="", help="comma-separated argv (argv[0] defaults to the workload path)")
ap.add_argument("--env", default="")
ap.add_argument("--inst", type=int, default=0)
ap.add_argument("--target", type=int, default=0, help="1..31 x-reg, 32 pc, 33 memory word; 0 = golden run")
ap.add_argument("--mask", type=lambda s: int(s, 0), default=0)
ap.add_argument("--addr", type=lambda s: int(s, 0), default=0)
ap.add_argument("--max-insts", type=int, default=0, help="hang cap (golden numInst * 2 + 1000)")
ap.add_argument("--clock", default="2GHz", help="CPU clock: clock_gettime sees curTick (engine: fi_set_clock)")
ap.add_argument("--cpu", default="atomic", choices=["atomic", "timing"])
ap.add_argument("--tick", type=int, default=0, help="--cpu timing: the fault's tick (fi_tick_site.tick)")
a = ap.parse_args()
cmd = [x for x in a.cmd.split(",") if x] or [a.workload]
out_dir = m5.options.outdir

if a.cpu == "timing":
    from gem5.components.boards.simple_board import SimpleBoard
    from gem5.components.cachehierarchies.classic.no_cache import NoCache
    from gem5.components.memory import SingleChannelDDR3_1600
    from gem5.components.processors.cpu_types import CPUTypes
    from gem5.components.processors.simple_processor import SimpleProcessor
    from gem5.isas import ISA
    from gem5.resources.resource import BinaryResource
    from gem5.simulate.simulator import Simulator

    board = SimpleBoard(clk_freq="3GHz", processor=SimpleProcessor(cpu_type=CPUTypes.TIMING, isa=ISA.RISCV,
                                                                   num_cores=1),
                        memory=SingleChannelDDR3_1600(), cache_hierarchy=NoCache())
    board.set_se_binary_workload(BinaryResource(local_path=a.workload), arguments=cmd[1:])
    core = board.get_processor().get_cores()[0].core
    for proc in core.workload:
        proc.output = os.path.join(out_dir, "stdout")
        proc.errout = os.path.join(out_dir, "stderr")
    if a.max_insts:
        core.max_insts_any_thread = a.max_insts
    if a.target:
        board.injector = FaultInjector(cpu=core, inst=0, tick=a.tick, target=a.target, mask=a.mask)
    sim = Simulator(board=board)
    sim.run()
    m5.stats.dump()
    print(json.dumps({"cause": sim.get_last_exit_event_cause(), "code": 0, "tick": sim.get_current_tick()}),
          flush=True)
    raise SystemExit(0)

system = System()
system.clk_domain = SrcClockDomain(clock=a.clock, voltage_domain=VoltageDomain())
system.mem_mode = "atomic"
system.mem_ranges = [AddrRange("3GiB")]
system.cpu = RiscvAtomicSimpleCPU()
system.membus = SystemXBar()
system.cpu.icache_port = system.membus.cpu_side_ports
system.cpu.dcache_port = system.membus.cpu_side_ports
system.cpu.createInterruptController()
system.mem_ctrl = MemCtrl(dram=DDR4_2400_8x8(range=system.mem_ranges[0]))
system.mem_ctrl.port = system.membus.mem_side_ports
system.system_port = system.membus.cpu_side_ports
system.workload = SEWorkload.init_compatible(a.workload)
system.cpu.workload = Process(cmd=cmd, executable=a.workload, env=[x for x in a.env.split(",") if x],
                              output=os.path.join(out_dir, "stdout"), errout=os.path.join(out_dir, "stderr"))
system.cpu.createThreads()
if a.max_insts:
    system.cpu.max_insts_any_thread = a.max_insts
if a.target:
    system.injector = FaultInjector(cpu=system.cpu, inst=a.inst, target=a.target, mask=a.mask, addr=a.addr)
root = Root(full_system=False, system=system)
m5.instantiate()
ev = m5.simulate()
m5.stats.dump()
print(json.dumps({"cause": ev.getCause(), "code": ev.getCode()}), flush=True)
