// FaultCampaign SimObject (gem5 side).  Compiled only inside a gem5 build
// (EXTRAS=src/gem5ext); everything it does is in shrewd::Campaign
// (src/campaign/campaign.hh), which is built and tested without gem5.
#ifndef __GEM5EXT_FAULT_CAMPAIGN_HH__
#define __GEM5EXT_FAULT_CAMPAIGN_HH__

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "params/FaultCampaign.hh"
#include "sim/sim_object.hh"

namespace shrewd {
class Campaign;
}

namespace gem5 {

class FaultCampaign : public SimObject
{
  public:
    PARAMS(FaultCampaign);
    explicit FaultCampaign(const Params &p);
    ~FaultCampaign() override;

    // SimObject lifecycle (src/sim/sim_object.hh:194,218,280): the engine is
    // created in init() so that a config error surfaces at m5.instantiate().
    void init() override;

    // Python-callable (cxx_exports)
    void run();
    std::string summaryJson() const;
    void setProtectMask(uint64_t mask);
    void setProtectOpClasses(std::vector<std::string> opclasses);
    uint64_t trialsRun() const;
    // the outcome histogram: the fi_histogram counters, flattened in
    // declaration order (include/fi_engine.h)
    std::vector<uint64_t> histogram() const;

  private:
    std::unique_ptr<shrewd::Campaign> campaign;
};

} // namespace gem5

#endif // __GEM5EXT_FAULT_CAMPAIGN_HH__
