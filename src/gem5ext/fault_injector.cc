#include "gem5ext/fault_injector.hh"

#include "arch/riscv/pcstate.hh"
#include "arch/riscv/regs/int.hh"
#include "base/logging.hh"
#include "cpu/thread_context.hh"
#include "mem/page_table.hh"
#include "mem/se_translating_port_proxy.hh"
#include "sim/process.hh"

namespace gem5 {

FaultInjector::FaultInjector(const Params &p)
    : SimObject(p), cpu(p.cpu), event([this] { inject(); }, name() + ".inject"),
      tick_event([this] { inject(); }, name() + ".inject_tick", false, Event::Minimum_Pri)
{
    if (p.target < 1 || p.target > 33)
        fatal("FaultInjector %s: target %u is not x1..x31, pc or memory", name(), p.target);
    if (p.tick && p.target == 33)
        fatal("FaultInjector %s: memory words have no tick mode", name());
}

void
FaultInjector::startup()
{
    SimObject::startup();
    if (params().tick) {
        // tick mode: before every other event of the tick (the flip lands in
        // whatever the TimingSimpleCPU has in flight: its fetch or data access)
        schedule(tick_event, params().tick);
        return;
    }
    // fires at the top of the first tick with numInst >= inst (the engine's
    // injection point; site.inst < golden numInst, so it is always reached)
    cpu->getContext(0)->scheduleInstCountEvent(&event, params().inst);
}

void
FaultInjector::inject()
{
    ThreadContext *tc = cpu->getContext(0);
    const uint64_t m = params().mask;
    const uint32_t t = params().target;
    if (t <= 31) {
        const RegId r = RiscvISA::intRegClass[t];
        tc->setReg(r, tc->getReg(r) ^ m);
    } else if (t == 32) {
        RiscvISA::PCState pc = tc->pcState().as<RiscvISA::PCState>();
        pc.set(pc.pc() ^ m);
        tc->pcState(pc);
    } else {
        // a word in a page that is not mapped at t: nothing to flip (the
        // engine ends such a trial as the golden run, fi_outcome.flags bit 1)
        Process *proc = tc->getProcessPtr();
        const Addr a = params().addr;
        if (!proc->pTable->lookup(a) || !proc->pTable->lookup(a + 7)) {
            warn("FaultInjector: %#x unmapped at numInst %llu", a, (unsigned long long)params().inst);
            return;
        }
        SETranslatingPortProxy proxy(tc);
        uint64_t v = 0;
        proxy.readBlob(a, &v, sizeof v);
        v ^= m;
        proxy.writeBlob(a, &v, sizeof v);
    }
}

} // namespace gem5
