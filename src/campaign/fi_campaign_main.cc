// fi_campaign -- command-line campaign driver (native host path above the
// fi_* C ABI; same parameters as the FaultCampaign SimObject).
//
//   fi_campaign --workload crc32.elf [--cmd crc32[,arg...]] [--env K=V,...]
//               [--trials N] [--first-trial F] [--seed S] [--structures int_reg,pc,mem]
//               [--burst K] [--bits 0-31,63] [--protect-mask M] [--protect-opclasses IntAlu,IntMult] [--num-gpus G] [--device D]
//               [--max-insts-factor F] [--private-pages P] [--output PREFIX]
//               [--executable PATH] [--input FILE|cin] [--devices 0,0,1]
//
// Prints one JSON summary line; with --output also writes PREFIX.outcomes.bin
// (fi_outcome records in trial order), PREFIX.hist.bin and PREFIX.json.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "campaign.hh"

static std::vector<std::string> split(const std::string &s) {
    std::vector<std::string> v;
    size_t a = 0;
    while (a <= s.size()) {
        size_t b = s.find(',', a);
        if (b == std::string::npos) b = s.size();
        if (b > a) v.push_back(s.substr(a, b - a));
        a = b + 1;
    }
    return v;
}

int main(int argc, char **argv) {
    shrewd::CampaignParams p;
    for (int i = 1; i < argc; i++) {
        std::string k = argv[i];
        if (i + 1 >= argc) { fprintf(stderr, "missing value for %s\n", k.c_str()); return 2; }
        std::string v = argv[++i];
        if (k == "--workload") p.workload = v;
        else if (k == "--cmd") p.cmd = split(v);
        else if (k == "--checkpoint") p.checkpoint = v;
        else if (k == "--env") p.env = split(v);
        else if (k == "--executable") p.executable = v;
        else if (k == "--input") p.input = v;
        else if (k == "--devices") {
            p.devices.clear();
            for (auto &d : split(v)) p.devices.push_back((int32_t)strtol(d.c_str(), nullptr, 0));
        }
        else if (k == "--trials") p.trials = strtoull(v.c_str(), nullptr, 0);
        else if (k == "--first-trial") p.first_trial = strtoull(v.c_str(), nullptr, 0);
        else if (k == "--seed") p.seed = strtoull(v.c_str(), nullptr, 0);
        else if (k == "--structures") p.structures = split(v);
        else if (k == "--burst") p.burst = (uint32_t)strtoul(v.c_str(), nullptr, 0);
        else if (k == "--bits") p.bits = v;
        else if (k == "--protect-mask") p.protect_mask = strtoull(v.c_str(), nullptr, 0);
        else if (k == "--protect-opclasses") p.protect_opclasses = split(v);
        else if (k == "--shadow-fu-model") p.shadow_fu_model = strtoul(v.c_str(), nullptr, 0) != 0;
        else if (k == "--priority-to-shadow") p.priority_to_shadow = strtoul(v.c_str(), nullptr, 0) != 0;
        else if (k == "--issue-width") p.issue_width = (uint32_t)strtoul(v.c_str(), nullptr, 0);
        else if (k == "--cpu-type") p.cpu_type = v;
        else if (k == "--load-latency") p.load_latency = (uint32_t)strtoul(v.c_str(), nullptr, 0);
        else if (k == "--num-gpus") p.num_gpus = (uint32_t)strtoul(v.c_str(), nullptr, 0);
        else if (k == "--device") p.first_device = (uint32_t)strtoul(v.c_str(), nullptr, 0);
        else if (k == "--max-insts-factor") p.max_insts_factor = strtod(v.c_str(), nullptr);
        else if (k == "--private-pages") p.private_pages = (uint32_t)strtoul(v.c_str(), nullptr, 0);
        else if (k == "--output") p.output = v;
        else { fprintf(stderr, "unknown option %s\n", k.c_str()); return 2; }
    }
    if (p.workload.empty()) { fprintf(stderr, "--workload is required\n"); return 2; }
    try {
        shrewd::Campaign c(p);
        c.run();
        printf("%s\n", c.summaryJson().c_str());
    } catch (const std::exception &e) {
        fprintf(stderr, "fi_campaign: %s\n", e.what());
        return 1;
    }
    return 0;
}
