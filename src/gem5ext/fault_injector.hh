// FaultInjector SimObject (gem5 side of the re-validation harness).  Compiled
// only inside a gem5 build (EXTRAS=src/gem5ext).  Applies one fi_site to
// thread 0 of a CPU at an instruction count.
#ifndef __GEM5EXT_FAULT_INJECTOR_HH__
#define __GEM5EXT_FAULT_INJECTOR_HH__

#include <cstdint>

#include "cpu/base.hh"
#include "params/FaultInjector.hh"
#include "sim/eventq.hh"
#include "sim/sim_object.hh"

namespace gem5 {

class FaultInjector : public SimObject
{
  public:
    PARAMS(FaultInjector);
    explicit FaultInjector(const Params &p);

    // schedules the flip on the thread's committed-instruction queue
    void startup() override;

  private:
    void inject();

    BaseCPU *cpu;
    EventFunctionWrapper event;       // instruction-count mode
    EventFunctionWrapper tick_event;  // tick mode: Minimum_Pri, ahead of every event of its tick
};

} // namespace gem5

#endif // __GEM5EXT_FAULT_INJECTOR_HH__
