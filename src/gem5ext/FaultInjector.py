# FaultInjector SimObject -- the gem5-side half of the re-validation harness
# (INTEGRATION.md §5): flips one fault site inside a real gem5 run, so that a
# site list sampled by the MI355X engine (fi_sample_sites) can be replayed one
# gem5 process per site (configs/fi_gem5_trial.py, tools/gem5_revalidate.py)
# and compared with the engine's fi_run_sites outcomes.
#
# The flip is an instruction-count event on the CPU's thread
# (ThreadContext::scheduleInstCountEvent, src/cpu/thread_context.hh:174, the
# mechanism of BaseCPU::scheduleInstStop, src/cpu/base.cc:764-770), which
# AtomicSimpleCPU services at the top of the first tick with numInst >= inst
# (src/cpu/simple/base.cc:321-325) -- the engine's injection point.
# Tick mode (tick > 0; a TimingSimpleCPU on the reference SE board, the
# engine's fi_run_tick_sites): the flip is an event on the main queue at that
# tick with the lowest priority value, so it precedes every other event of the
# tick -- the state it sees is the one after all events of earlier ticks,
# which is what the engine's map to the instruction in flight assumes.
from m5.params import *
from m5.proxy import *
from m5.SimObject import SimObject


class FaultInjector(SimObject):
    type = "FaultInjector"
    cxx_header = "gem5ext/fault_injector.hh"
    cxx_class = "gem5::FaultInjector"

    cpu = Param.BaseCPU("the CPU whose thread 0 is faulted")
    inst = Param.UInt64("numInst at whose tick the flip is applied (fi_site.inst)")
    target = Param.UInt32("1..31 = x1..x31, 32 = pc, 33 = 8-byte memory word (fi_site.target)")
    mask = Param.UInt64("xor mask (fi_site.mask)")
    addr = Param.Addr(0, "memory sites: 8-byte aligned guest virtual address (fi_site.addr)")
    tick = Param.UInt64(
        0, "tick mode: the flip happens before every event of this tick (fi_tick_site.tick); 0 = at inst")
