// Tick-domain injection: the golden request list and the tick -> numInst site
// map (fi_tick.h; include/fi_engine.h "Tick-domain injection").
//
// The golden request list.  TimingSimpleCPU runs the same instructions as
// AtomicSimpleCPU; what it adds is a fetch-execute *attempt* per atomic tick
// with requests to memory (src/cpu/simple/timing.cc:677-1077): the 4-byte
// fetch of (pc & ~3) + fetchOffset (base.cc:304-318; a 32-bit instruction at
// pc % 4 == 2 fetches twice, decoder.cc:63-116), then the data request(s) of
// a load / store / AMO, split at 64-byte lines (timing.cc:451-586).  Two
// kinds of attempt do not commit: an ecall (the syscall runs in the fault's
// invoke) and a data access to a page SE has not allocated yet (the
// GenericPageTableFault's fixupFault allocates it and the instruction runs
// again, sim/faults.cc:95-105, sim/mem_state.cc:387-447).  Physical
// addresses: SE hands out frames in allocation order from the bottom of
// memory (Process::allocateMem -> MemPool, sim/process.cc:318-343,
// sim/mem_pool.cc:96-102): the image as initState writes it, argsInit's
// stack, then each page a fault or a syscall write fixes up.
//
// The site map.  A flip at tick t happens before every event of tick t; the
// attempt in flight is the first whose last event is at or after t.  Before
// it executes (its fetch outstanding) a register flip is a numInst injection
// at its numInst; while its data access is outstanding the sources are read,
// so the flip takes effect from the next instruction on -- unless the
// completion writes that register (TimingSimpleCPU::completeDataAccess ->
// completeAcc).  A pc flip while the fetch is outstanding leaves the
// instruction fetched from the old word: executed at the new pc (decode sets
// npc, decoder.cc:135-173), its effect is the golden instruction's with the
// next pc, a link or a branch target moved by the difference -- one numInst
// site after it; a pc flip during the data access goes through
// PCState::set, npc = pc + 4, which advancePC then takes.  The cases that are
// not one numInst site are FI_ESC_TIMING (FI_TK_*).
#include "fi_tick.h"

#include <algorithm>
#include <unordered_map>

#include "rv64_isa.h"

namespace fi {
namespace {

bool is_int_load(uint8_t op) {
    switch (op) {
    case OP_lb: case OP_lh: case OP_lw: case OP_ld: case OP_lbu: case OP_lhu: case OP_lwu:
    case OP_c_lw: case OP_c_ld: case OP_c_lbu: case OP_c_lhu: case OP_c_lh: case OP_c_lwsp: case OP_c_ldsp:
        return true;
    default:
        return false;
    }
}
bool is_fp_load(uint8_t op) {
    return op == OP_flh || op == OP_flw || op == OP_fld || op == OP_c_fld || op == OP_c_fldsp;
}
bool is_store(uint8_t op) {
    switch (op) {
    case OP_sb: case OP_sh: case OP_sw: case OP_sd: case OP_c_sb: case OP_c_sh: case OP_c_sw: case OP_c_sd:
    case OP_c_swsp: case OP_c_sdsp: case OP_fsh: case OP_fsw: case OP_fsd: case OP_c_fsd: case OP_c_fsdsp:
        return true;
    default:
        return false;
    }
}
bool is_amo(uint8_t op) { return op >= OP_amoadd_w && op <= OP_amomaxu_d; }
bool is_lr(uint8_t op) { return op == OP_lr_w || op == OP_lr_d; }
bool is_sc(uint8_t op) { return op == OP_sc_w || op == OP_sc_d; }

uint8_t ctl_of(uint8_t op) {
    switch (op) {
    case OP_beq: case OP_bne: case OP_blt: case OP_bge: case OP_bltu: case OP_bgeu: case OP_c_beqz: case OP_c_bnez:
        return kCtlBranch;
    case OP_jal: case OP_c_j: return kCtlJal;
    case OP_jalr: case OP_c_jr: case OP_c_jalr: return kCtlJalr;
    case OP_auipc: return kCtlAuipc;
    default: return kCtlNone;
    }
}

// SE physical frames and the stack's growth (MemState::fixupFault)
struct Frames {
    std::unordered_map<uint64_t, uint64_t> of;   // vpn -> frame
    uint64_t next = 0;
    uint64_t stack_min = 0;
    const TickGoldenIn *in = nullptr;
    bool has(uint64_t vpn) const { return of.count(vpn) != 0; }
    void alloc(uint64_t vpn) {
        if (!has(vpn)) of[vpn] = next++;
    }
    void fixup(uint64_t va) {
        const uint64_t pg = va & ~(kPage - 1);
        if ((va >= in->svma_lo && va < in->svma_hi) || (va >= stack_min && va < in->stack_base)) {
            alloc(pg >> 12);
        } else if (va < stack_min && va >= in->stack_base - in->max_stack) {
            while (va < stack_min) {
                stack_min -= kPage;
                alloc(stack_min >> 12);
            }
        } else {
            alloc(pg >> 12);   // a heap / mmap VMA page (those lie outside the stack's window)
        }
    }
    uint64_t paddr(uint64_t va) const { return (of.at(va >> 12) << 12) | (va & (kPage - 1)); }
};

}  // namespace

std::string build_tick_attempts(const TickGoldenIn &in, std::vector<fi_timing_op> &ops,
                                std::vector<TickAttempt> &att) {
    ops.clear();
    att.clear();
    const std::vector<uint32_t> &trace = *in.trace;
    const std::vector<PreInst> &pre = *in.pre;
    const std::vector<MemEv> &mev = *in.mev;
    if (trace.empty()) return "the golden trace is unavailable";
    Frames fr;
    fr.in = &in;
    fr.stack_min = in.stack_min0;
    for (uint64_t vpn : *in.alloc) fr.alloc(vpn);
    size_t k = 0;          // next data-access event
    uint64_t n = 0;        // numInst
    uint64_t cycles = 0;   // AtomicSimpleCPU ticks, against the golden count
    ops.reserve(trace.size() + 8);
    att.reserve(trace.size() + 8);
    auto emit = [&](const TickAttempt &a, const fi_timing_op &o) {
        if (!att.empty()) att.back().next_pc = a.pc;
        att.push_back(a);
        ops.push_back(o);
    };
    for (size_t i = 0; i < trace.size(); i++) {
        const uint32_t h = trace[i] & 0x7FFFFFFFu;
        const bool ecall = (trace[i] >> 31) != 0;
        if (h >= pre.size() || !(pre[h].flags & kPreValid)) return "a golden pc outside the pre-decoded text";
        const PreInst &p = pre[h];
        const uint64_t pc = in.text_lo + 2ULL * h;
        const bool last = i + 1 == trace.size();
        TickAttempt a;
        a.pc = pc; a.n = n; a.len = p.len; a.imm = p.imm;
        a.nfetch = ((pc & 3) == 2 && p.len == 4) ? 2 : 1;
        a.rd = p.rd; a.rs1 = p.rs1; a.rs2 = p.rs2;
        a.ctl = ctl_of(p.op);
        a.macro = is_amo(p.op) || is_lr(p.op) || is_sc(p.op);
        fi_timing_op o{};
        o.nfetch = a.nfetch;
        o.fetch[0] = fr.paddr(pc & ~3ULL);
        if (a.nfetch == 2) o.fetch[1] = fr.paddr((pc & ~3ULL) + 4);
        if (p.op == OP_vec || p.op == OP_vset) return "a vector op in the golden run";
        if (p.op == OP_prefetch_i || p.op == OP_prefetch_r || p.op == OP_prefetch_w)
            return "a prefetch (a PREFETCH request) in the golden run";
        if (p.op == OP_cbo && p.imm != 4) return "a cache-block management op in the golden run";
        if (ecall) {
            // the syscall's own accesses are functional (a port proxy): no
            // requests, but a write allocates the pages it touches
            while (k < mev.size() && (mev[k].t & kMemEvProxy) && (mev[k].t & ~kMemEvProxy) == n) {
                const uint64_t len = mev[k].len_kind & ((1u << 30) - 1), kind = mev[k].len_kind >> 30;
                if (kind & 2)
                    for (uint64_t v = mev[k].addr >> 12; v <= (mev[k].addr + len - 1) >> 12; v++)
                        if (!fr.has(v)) fr.fixup(std::max(v << 12, mev[k].addr));
                k++;
            }
            a.ecall = true; a.end = last;
            o.kind = last ? FI_TOP_END : FI_TOP_FAULT;
            emit(a, o);
            cycles += a.nfetch;
            continue;
        }
        const bool mem = is_int_load(p.op) || is_fp_load(p.op) || is_store(p.op) || a.macro || p.op == OP_cbo;
        if (mem) {
            while (k < mev.size() && (mev[k].t & kMemEvProxy)) {   // (an M5 op's reads, say)
                if ((mev[k].t & ~kMemEvProxy) > n) break;
                k++;
            }
            if (k >= mev.size() || mev[k].t != n) {
                if (is_sc(p.op)) return "the golden run has a failed SC";
                return "a golden memory access without its record";
            }
            const uint64_t addr = mev[k].addr, size = mev[k].len_kind & ((1u << 30) - 1);
            k++;
            // fragments at 64-byte lines; a fragment on a page SE has not
            // allocated faults the attempt (the first such fragment), the fixup
            // allocates it and the instruction runs again
            uint64_t fa[2], fs[2];
            int nf = 0;
            for (uint64_t x = addr; x < addr + size && nf < 3;) {
                const uint64_t e = std::min(addr + size, (x | 63) + 1);
                if (nf == 2) return "an access of more than two fragments";
                fa[nf] = x; fs[nf] = e - x; nf++;
                x = e;
            }
            for (;;) {
                int miss = -1;
                for (int q = 0; q < nf && miss < 0; q++)
                    if (!fr.has(fa[q] >> 12)) miss = q;
                if (miss < 0) break;
                TickAttempt r = a;
                r.pgfault = true;
                fi_timing_op ro = o;
                ro.kind = FI_TOP_FAULT;
                emit(r, ro);
                cycles += a.nfetch;
                fr.fixup(fa[miss]);
            }
            o.nfrag = (uint8_t)nf;
            for (int q = 0; q < nf; q++) { o.addr[q] = fr.paddr(fa[q]); o.size[q] = (uint16_t)fs[q]; }
            o.cmd = is_store(p.op) || p.op == OP_cbo ? FI_TCMD_WRITE
                  : is_amo(p.op) ? FI_TCMD_SWAP : is_lr(p.op) ? FI_TCMD_LL : is_sc(p.op) ? FI_TCMD_SC : FI_TCMD_READ;
            if (is_int_load(p.op) || a.macro) a.done_rd = p.rd;
        }
        a.commits = true; a.end = last;
        o.kind = last ? FI_TOP_END : FI_TOP_EXEC;
        if (last) o.nfrag = 0;   // (an M5 exit op: the run ends at its execute)
        emit(a, o);
        cycles += a.nfetch + (a.macro ? ((p.raw >> 25) & 1) + ((p.raw >> 26) & 1) : 0);
        n++;
    }
    while (k < mev.size() && (mev[k].t & kMemEvProxy)) k++;
    if (k != mev.size()) return "golden data-access records left over";
    if (n != in.golden_ninst) return "the trace's instruction count differs from the golden run's";
    if (cycles != in.golden_ncycles) return "the rebuilt attempts miss golden ticks (an unmodelled fault retry)";
    return "";
}

TickMapped map_tick_site(const std::vector<TickAttempt> &att, const std::vector<fi_timing_ticks> &ticks,
                         uint64_t golden_ninst, uint64_t t, uint32_t target, uint64_t mask, uint32_t trial) {
    TickMapped r;
    // the attempt in flight: the first whose last event is at or after t
    const auto it = std::lower_bound(ticks.begin(), ticks.end(), t,
                                     [](const fi_timing_ticks &x, uint64_t v) { return x.done < v; });
    const uint64_t j = (uint64_t)(it - ticks.begin());
    r.attempt = j;
    const TickAttempt &A = att[j];
    const fi_timing_ticks &T = ticks[j];
    enum { FETCH1, FETCH2, DATA } ph = (A.nfetch == 2 && t <= T.fetch_done[0]) ? FETCH1
                                     : t <= T.exec ? (A.nfetch == 2 ? FETCH2 : FETCH1) : DATA;
    uint64_t g = j;   // the attempts since the last commit (ecalls, page-fault retries)
    while (g > 0 && !att[g - 1].commits) g--;
    auto site = [&](uint32_t tg, uint64_t m, uint64_t inst) {
        r.disp = 0;
        r.site.inst = inst; r.site.mask = m; r.site.addr = 0; r.site.target = tg; r.site.trial = trial;
        if (inst > golden_ninst) r.disp = 1;   // after the run's last commit: the golden run
        return r;
    };
    auto golden = [&]() { r.disp = 1; return r; };
    auto escape = [&](uint32_t why) { r.disp = 2; r.reason = why; return r; };
    if (target == FI_T_RESULT) return site(FI_T_RESULT, mask, A.n);   // the first commit at or after t
    if (target >= 1 && target <= 31) {
        if (ph == DATA) return A.done_rd == target ? golden() : site(target, mask, A.n + 1);
        for (uint64_t q = g; q < j; q++) {   // the flip lands after these: it must commute with them
            const TickAttempt &Q = att[q];
            if (Q.ecall && target >= 10 && target <= 17) return escape(FI_TK_NONCOUNT);
            if (Q.pgfault && (target == Q.rs1 || target == Q.rs2)) return escape(FI_TK_NONCOUNT);
        }
        return site(target, mask, A.n);
    }
    // the pc
    if (g != j) return escape(FI_TK_NONCOUNT);
    const uint64_t pc = A.pc, np = pc ^ mask;
    const bool same_word = ((pc ^ np) & ~3ULL) == 0;
    if (ph == DATA) return A.macro ? escape(FI_TK_MACRO) : site(FI_T_PC, (pc + A.len) ^ (np + 4), A.n + 1);
    if (!A.commits || A.end) return (ph == FETCH1 && same_word) ? site(FI_T_PC, mask, A.n) : escape(FI_TK_FAULTOP);
    if (ph == FETCH1) {
        if (same_word) return site(FI_T_PC, mask, A.n);
        if (A.nfetch == 2) return escape(FI_TK_STRADDLE1);
        if ((pc & 3) != (np & 3)) return escape(FI_TK_ALIGN);
    } else if ((np & 3) == 0) {
        return escape(FI_TK_STRADDLE2);
    }
    // the golden instruction executed at np: its effect, moved by np - pc
    switch (A.ctl) {
    case kCtlAuipc: return escape(FI_TK_TWO);
    case kCtlJal:
        if (A.rd) return escape(FI_TK_TWO);
        return site(FI_T_PC, (pc + (uint64_t)A.imm) ^ (np + (uint64_t)A.imm), A.n + 1);
    case kCtlJalr:
        if (!A.rd) return golden();   // the target comes from rs1
        return site(A.rd, (pc + A.len) ^ (np + A.len), A.n + 1);
    case kCtlBranch: {
        const uint64_t x = A.next_pc != pc + A.len ? (uint64_t)A.imm : A.len;
        return site(FI_T_PC, (pc + x) ^ (np + x), A.n + 1);
    }
    default: return site(FI_T_PC, (pc + A.len) ^ (np + A.len), A.n + 1);
    }
}

}  // namespace fi
