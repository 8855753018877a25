// fi_types.h -- structures shared by the host engine (fi_engine.cpp) and the
// CDNA4 kernels (hip/fi_kernels.hip).  Internal; the public ABI is
// include/fi_engine.h.
#pragma once
#include <stdint.h>

#include "../../include/fi_engine.h"

namespace fi {

constexpr uint64_t kPage = 4096;
// RiscvProcess64 constants, src/arch/riscv/process.cc:73-80
constexpr uint64_t kStackBase = 0x7FFFFFFFFFFFFFFFULL;
constexpr uint64_t kMaxStack = 8ULL * 1024 * 1024;
constexpr uint64_t kStackTopVpn = kStackBase >> 12;
// default Process params, src/sim/Process.py:61-67
constexpr uint64_t kPid = 100, kPpid = 0, kUid = 100, kGid = 100;

// Pre-decoded instruction, one per halfword of the golden text.  Filled on the
// device by fi_predecode_kernel with the same decoder the slow path uses.
struct PreInst {
    uint32_t raw;
    uint8_t op, rd, rs1, rs2;   // rd/rs1/rs2 = 0 when unused (x0 semantics)
    int32_t imm;
    uint8_t len;                // 2 or 4
    uint8_t flags;              // kPreValid | kPreStraddle | kPreRs1 | kPreRs2 | kPreRd
    uint16_t aux;               // csr index (SYSTEM) / funct3
};
static_assert(sizeof(PreInst) == 16, "PreInst must stay 16 bytes (one s_load_dwordx4)");
constexpr uint8_t kPreValid = 1, kPreStraddle = 2, kPreRs1 = 4, kPreRs2 = 8, kPreRd = 16;

// Everything one launch of the trial kernel needs.  Passed by value as the
// kernel argument (lives in the kernarg segment -> scalar loads).
struct DevCtx {
    // golden text, pre-decoded
    const PreInst *pre;
    uint64_t text_lo, text_hi;       // page-aligned executable range
    // base (process-start) image: sorted vpns -> frame index into frames
    const uint64_t *base_vpn;
    const uint32_t *base_frame;
    const uint8_t *frames;
    const uint8_t *zero_page;
    uint32_t n_base;
    uint32_t record;                 // 1 = golden run: record output instead of comparing
    // process start state
    uint64_t entry, sp0, stack_min0, stack_vma_lo, stack_vma_hi;
    // golden reference output (or record buffers in golden mode)
    const uint8_t *gout, *gerr;
    uint64_t gout_len, gerr_len;
    uint8_t *rec_out, *rec_err;
    uint64_t rec_cap;
    uint32_t gexit;
    uint32_t priv_pages;             // P
    uint64_t hang_cap;
    uint64_t protect_mask;
    // per-trial private (copy-on-write) pages: frames [slot][P][4096], vpns [P][n]
    uint8_t *priv_frames;
    uint64_t *priv_vpn;
    // the work
    const fi_site *sites;            // in trial order
    const uint32_t *perm;            // launch slot -> index into sites/out (sorted by site.inst)
    fi_outcome *out;
    uint64_t n;                      // trials in this launch
    unsigned long long *stats;       // [0] fetch B [1] data B [2] pages [3..5] golden ncycles/out/err
                                     // [6] loop iterations [7] lane-insts [8] slow fetches [9] min-PC [10] max iter/wave
};

struct SampleCtx {
    uint64_t seed, structures, golden_ninst, first;
    uint32_t burst, n_struct;
    const uint64_t *mem_pages;
    uint64_t n_mem_pages;
};

}  // namespace fi
