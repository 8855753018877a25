// fi_checkpoint.h -- host-side reader of gem5 SE checkpoints (fi_checkpoint.cpp).
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <utility>
#include <vector>

namespace fi {

// What a campaign start needs from a gem5 SE checkpoint.
struct CptImage {
    uint64_t regs[32] = {};                // x0..x31 (x0 forced 0)
    uint64_t pc = 0;
    uint64_t fregs[32] = {};               // f0..f31 (regs.floating_point)
    uint32_t fflags = 0, frm = 0;          // MISCREG_FFLAGS / MISCREG_FRM of the ISA's miscRegFile
    bool fp_state = false;                 // any of them nonzero
    uint64_t tick0 = 0;                    // [Globals] curTick
    uint64_t brk = 0, stack_base = 0, stack_size = 0, max_stack = 0, stack_min = 0, mmap_end = 0;
    std::vector<std::string> vma_names;
    std::vector<std::pair<uint64_t, uint64_t>> vmas;
    std::map<uint64_t, std::vector<uint8_t>> pages;   // vpn -> 4 KiB
};

// Reads dir/m5.cpt and its memory store; "" on success, else the reason.
std::string read_gem5_checkpoint(const std::string &dir, CptImage &img);

}  // namespace fi
