// campaign.hh -- native fault-injection campaign driver over the fi_* C ABI.
//
// The gem5-independent core of the FaultCampaign SimObject
// (src/gem5ext/fault_campaign.{hh,cc}) and of the `fi_campaign` command-line
// driver.  Parameters mirror the SimObject's (src/gem5ext/FaultCampaign.py),
// which follow SURVEY.md §8(b): workload/cmd/env as gem5's Process
// (src/sim/Process.py:61-67), the campaign spec, the SHREWD protection mask
// (the setEnableShrewd analogue, src/cpu/BaseCPU.py:68-77) and the GPU count.
//
// Multi-GPU inside one process (gem5 is single-process): one host thread and
// one engine per device; trial ids split in contiguous blocks
// [g*T/G, (g+1)*T/G) and histograms summed on the host.  Multi-process
// (one rank per GPU, RCCL all-reduce) is the Python path in shrewd_amd/fi.py.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/fi_engine.h"

namespace shrewd {

struct CampaignParams {
    std::string workload;                 // RV64 static ELF path
    std::string checkpoint;               // gem5 SE checkpoint directory to start from ("" = process start)
    std::vector<std::string> cmd;         // argv; empty -> {workload}
    std::vector<std::string> env;
    std::string executable;               // Process.executable: /proc/self/exe resolves to its realpath
                                          // ("" = the workload path, as gem5's se configs set it)
    std::string input = "cin";            // Process.input (src/sim/Process.py:44): "cin"/"stdin" = the host's
                                          // stdin (reads of fd 0 escape); else a file fd 0 reads
    uint64_t trials = 1000;
    uint64_t first_trial = 0;
    uint64_t seed = 0x5EED0001ULL;
    std::vector<std::string> structures{"int_reg"};
    uint32_t burst = 1;
    std::string bits;                     // eligible lowest flipped bits: "0-63" (all), "0-31,63", or a number
    uint64_t protect_mask = 0;
    std::vector<std::string> protect_opclasses;   // SHREWD replication set (gem5 OpClass names)
    bool shadow_fu_model = false;         // SHREWD FU contention for result faults (fi_set_issue_model)
    bool priority_to_shadow = false;      // BaseO3CPU.priorityToShadow (src/cpu/o3/BaseO3CPU.py:227)
    uint32_t issue_width = 8;             // BaseO3CPU.issueWidth
    uint32_t load_latency = 2;            // issue model: cycles from a load's issue to its value
    uint32_t num_gpus = 1;
    uint32_t first_device = 0;
    std::vector<int32_t> devices;         // explicit HIP device per engine (overrides num_gpus/first_device;
                                          // a device may repeat: several engines share it)
    double max_insts_factor = 2.0;        // hang cap = golden * f + 1000
    uint32_t private_pages = 16;
    std::string output;                   // prefix: <output>.outcomes.bin + <output>.json
    std::string cpu_type = "atomic";      // "atomic": sites at a numInst; "timing": at a tick of a
                                          // TimingSimpleCPU run on the reference board (fi_set_cpu_model)
};

// 'int_reg' (x1..x31), 'pc', 'mem', 'xN' or ABI register names -> bitmask
// (bit r = x_r, bit 32 = pc, bit 33 = memory word).  Throws on unknown names.
uint64_t structures_mask(const std::vector<std::string> &names);
// `bits` spec ("", "0-63", "0-31,63", "0xffff") -> mask of eligible positions
uint64_t bits_mask(const std::string &spec);
// gem5 OpClass names ("IntAlu", "IntMultOp", ...) or enum values -> bitmask
uint64_t opclass_mask(const std::vector<std::string> &names);

struct GoldenSummary {
    uint64_t ninst = 0, ncycles = 0;
    uint32_t exit_code = 0;
    std::string stdout_bytes;
};

class Campaign {
  public:
    explicit Campaign(const CampaignParams &p);
    ~Campaign();
    Campaign(const Campaign &) = delete;
    Campaign &operator=(const Campaign &) = delete;

    // Runs all trials; outcomes in trial-id order.  Throws std::runtime_error
    // on engine errors (the SimObject turns these into fatal()).
    void run();
    void setProtectMask(uint64_t mask);
    void setProtectOpClasses(const std::vector<std::string> &opclasses);

    const fi_histogram &histogram() const { return hist_; }
    const std::vector<fi_outcome> &outcomes() const { return out_; }
    const GoldenSummary &golden() const { return golden_; }
    double seconds() const { return seconds_; }
    std::string summaryJson() const;
    void writeOutput() const;

  private:
    CampaignParams p_;
    std::vector<fi_engine *> engines_;
    GoldenSummary golden_;
    fi_histogram hist_{};
    std::vector<fi_outcome> out_;
    double seconds_ = 0;
};

}  // namespace shrewd
