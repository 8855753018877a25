#include "gem5ext/fault_campaign.hh"

#include <stdexcept>

#include "base/logging.hh"
#include "campaign/campaign.hh"

namespace gem5 {

FaultCampaign::FaultCampaign(const Params &p) : SimObject(p) {}

FaultCampaign::~FaultCampaign() = default;

void
FaultCampaign::init()
{
    SimObject::init();
    shrewd::CampaignParams cp;
    cp.workload = params().workload;
    cp.checkpoint = params().checkpoint;
    cp.cmd = params().cmd;
    cp.env = params().env;
    cp.executable = params().executable;
    cp.input = params().input;
    cp.trials = params().trials;
    cp.first_trial = params().first_trial;
    cp.seed = params().seed;
    cp.structures = params().structures;
    cp.burst = params().burst;
    cp.bits = params().bits;
    cp.protect_mask = params().protect_mask;
    cp.protect_opclasses = params().protect_opclasses;
    cp.shadow_fu_model = params().shadow_fu_model;
    cp.priority_to_shadow = params().priority_to_shadow;
    cp.issue_width = params().issue_width;
    cp.cpu_type = params().cpu_type;
    cp.load_latency = params().load_latency;
    cp.num_gpus = params().num_gpus;
    cp.first_device = params().first_gpu;
    cp.max_insts_factor = params().max_insts_factor;
    cp.private_pages = params().private_pages;
    cp.output = params().output;
    try {
        campaign = std::make_unique<shrewd::Campaign>(cp);
    } catch (const std::exception &e) {
        // gem5 reports configuration/user errors with fatal() (base/logging.hh)
        fatal("FaultCampaign %s: %s", name(), e.what());
    }
}

void
FaultCampaign::run()
{
    try {
        campaign->run();
    } catch (const std::exception &e) {
        fatal("FaultCampaign %s: %s", name(), e.what());
    }
}

std::string
FaultCampaign::summaryJson() const
{
    return campaign->summaryJson();
}

void
FaultCampaign::setProtectMask(uint64_t mask)
{
    campaign->setProtectMask(mask);
}

void
FaultCampaign::setProtectOpClasses(std::vector<std::string> opclasses)
{
    campaign->setProtectOpClasses(opclasses);
}

uint64_t
FaultCampaign::trialsRun() const
{
    return campaign->histogram().trials;
}

std::vector<uint64_t>
FaultCampaign::histogram() const
{
    // the fi_histogram counters in declaration order (include/fi_engine.h)
    const fi_histogram &h = campaign->histogram();
    const uint64_t *p = reinterpret_cast<const uint64_t *>(&h);
    return std::vector<uint64_t>(p, p + sizeof(h) / sizeof(uint64_t));
}

} // namespace gem5
