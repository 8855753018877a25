// Tick-domain injection under TimingSimpleCPU (include/fi_engine.h,
// "Tick-domain injection"): the golden run's fetch-execute attempts as
// requests for the timing model (fi_timing.cpp), and the map from a fault at
// tick t to the numInst site the trial kernels run.  Host code.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "fi_engine.h"
#include "fi_types.h"

namespace fi {

// One fetch-execute attempt of the golden run, as the site map needs it.
struct TickAttempt {
    uint64_t pc = 0, next_pc = 0;   // its pc; the next attempt's pc
    uint64_t n = 0;                 // numInst before it
    int64_t imm = 0;                // branch / jal offset
    uint8_t len = 4, nfetch = 1;
    bool commits = false;           // numInst counts it (an ecall or a page-fault retry does not)
    bool ecall = false, pgfault = false, end = false;
    uint8_t ctl = 0;                // kCtl*
    uint8_t rd = 0, rs1 = 0, rs2 = 0;
    bool macro = false;             // AMO / LR / SC: a macro-op (formats/amo.isa)
    uint8_t done_rd = 0;            // the x register its completeAcc writes (int loads, AMO, LR, SC); 0 none
};
enum : uint8_t { kCtlNone = 0, kCtlBranch = 1, kCtlJal = 2, kCtlJalr = 3, kCtlAuipc = 4 };

struct TickGoldenIn {
    const std::vector<uint32_t> *trace;   // per committed instruction and ecall: halfword | bit 31 ecall
    const std::vector<PreInst> *pre;
    uint64_t text_lo;
    const std::vector<MemEv> *mev;        // data accesses (CPU requests; syscall ones carry kMemEvProxy)
    const std::vector<uint64_t> *alloc;   // process-start pages in allocation order (image, then argsInit)
    uint64_t stack_min0, svma_lo, svma_hi, stack_base, max_stack;
    uint64_t golden_ninst, golden_ncycles;
};

// "" on success; else why the golden run has no tick model (the request
// list cannot be rebuilt exactly: unsupported ops, inconsistent records).
std::string build_tick_attempts(const TickGoldenIn &in, std::vector<fi_timing_op> &ops,
                                std::vector<TickAttempt> &att);

// The site map: disposition 0 run `site`, 1 golden-equal, 2 escape (reason).
struct TickMapped {
    int disp = 0;
    uint32_t reason = 0;
    fi_site site{};
    uint64_t attempt = 0;
};
TickMapped map_tick_site(const std::vector<TickAttempt> &att, const std::vector<fi_timing_ticks> &ticks,
                         uint64_t golden_ninst, uint64_t t, uint32_t target, uint64_t mask, uint32_t trial);

}  // namespace fi
