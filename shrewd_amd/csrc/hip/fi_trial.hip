// fi_trial.hip -- the batched RV64 interpreter of the fault-injection campaign
// (CDNA4 / gfx950).  One trial per lane; a 64-lane wave runs 64 trials that
// are sorted by inject time.  The loop body is AtomicSimpleCPU::tick
// (src/cpu/simple/atomic.cc:611-739) with the golden-trace comparator and the
// outcome classifier folded into the syscall/exit path.
//
//   * Golden snapshots: a wave starts at the golden snapshot at
//     or before the earliest inject time of its lanes instead of at process
//     start, and a lane whose whole architectural state (pc, x1..x31, output
//     positions, stack limit, every mapped page) equals the golden state at a
//     later snapshot is classified masked on the spot: the machine is
//     deterministic, so its future is the golden future.  Both are exact; the
//     oracle (oracle/rv64se.c) runs every trial from process start.
//   * Registers live in LDS as R[row][lane] (row 32 = write sink for
//     instructions without a destination, so the write is unconditional).
//   * Guest memory: read-only snapshot frames shared by the whole launch +
//     per-trial copy-on-write pages; a 4-entry per-lane TLB in VGPRs in front
//     of the lane's private-page list and the snapshot's page table.
//   * Fast path: while a group of lanes is converged on the pre-decoded golden
//     text, the guest PC lives in SGPRs and each instruction is one scalar
//     dispatch; the pre-decoded entries of both successors are prefetched with
//     scalar loads while the current instruction executes.
#include "fi_rtc.h"
#include "fi_types.h"
#include "fi_device.h"
#include "rv64_isa.h"
#include "gem5_opclass_table.h"
#include "fi_softfp.h"
#include "fi_crypto.h"
#ifndef __HIPCC_RTC__
#include "fi_debug.h"   // (the static library's test hooks)
#endif

namespace fi {

// Lanes per wave.  Every kernel below is instantiated twice from the same
// source: the campaign kernel runs 64 trials per wave (kNL = 64); the solo
// kernel runs one trial per single-lane wave (kNL = 1), for the diverged
// survivors of resumed epochs.  In the solo instantiation the lane index is
// the constant 0, so every per-trial value is wave-uniform: the compiler keeps
// the trial state in SGPRs, VGPR use drops, and many more waves share a SIMD
// to hide the memory latency of serial trials.  Same semantics, same code.
template <uint32_t kNL> __device__ __forceinline__ uint32_t lane_id() {
    return kNL == 1 ? 0u : (uint32_t)threadIdx.x;
}
template <uint32_t kNL> __device__ __forceinline__ uint64_t wmin64(uint64_t v) {
    return kNL == 1 ? v : wave_min64(v);
}
template <uint32_t kNL> __device__ __forceinline__ uint64_t wsum64(uint64_t v) {
    return kNL == 1 ? v : wave_sum64(v);
}
template <uint32_t kNL> __device__ __forceinline__ uint64_t rdl64(uint64_t v, int l) {
    return kNL == 1 ? v : readlane64(v, l);
}
template <uint32_t kNL> __device__ __forceinline__ uint32_t rdl32(uint32_t v, int l) {
    return kNL == 1 ? v : (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
template <uint32_t kNL> __device__ __forceinline__ uint64_t wballot(bool x) {
    return kNL == 1 ? (uint64_t)x : (uint64_t)__ballot(x);
}

constexpr uint64_t kNone = ~0ULL;
// The solo kernels (kNL = 1: one trial per wave) run kSoloLanes identical
// lanes (fi_types.h); side effects that must happen once (atomics) are taken
// by thread 0 (kSoloOnce), page copies split over the lanes.  kSoloLanes is 1:
// with 64 lanes the compiler can no longer treat the trial state as uniform
// (the kernel's stack objects become per-lane memory) and the solo kernel
// spilled 16x more (84 -> 1,343 scratch instructions).
#define kSoloOnce (kNL > 1 || threadIdx.x == 0)
constexpr uint64_t kSoloPrioInsts = 32768;   // a solo wave past this many instructions raises its priority
constexpr uint32_t kSinkRow = 32;
constexpr uint32_t kRows = 33;

// The launch context is read through an opaque pointer into the kernarg
// segment (constant address space -> scalar loads) at each use instead of
// being held in SGPRs for the whole kernel: the interpreter's hot loop needs
// those SGPRs, and spilling them forced a wait on every prefetch.
typedef __attribute__((address_space(4))) const DevCtx KCtx;
__device__ __forceinline__ KCtx *opq(KCtx *p) {
    asm volatile("" : "+s"(p));
    return p;
}

// ------------------------------------------------------------------ semantics
// Integer helpers of the generated StaticInst::execute bodies
// (src/arch/riscv/isa/decoder.isa; div/rem edge cases src/arch/riscv/utility.hh:
// 191-231), shared by the general path below and the translated blocks.
__device__ __forceinline__ uint64_t orc_b(uint64_t a) {
    uint64_t v = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) if ((a >> (8 * i)) & 0xFF) v |= 0xFFULL << (8 * i);
    return v;
}
__device__ __forceinline__ uint64_t clmul(uint64_t a, uint64_t b) {
    uint64_t v = 0;
    for (int i = 0; i < 64; i++) if ((b >> i) & 1) v ^= a << i;
    return v;
}
__device__ __forceinline__ uint64_t clmulr(uint64_t a, uint64_t b) {
    uint64_t v = 0;
    for (int i = 0; i < 64; i++) if ((b >> i) & 1) v ^= a >> (63 - i);
    return v;
}
__device__ __forceinline__ uint64_t clmulh(uint64_t a, uint64_t b) {
    uint64_t v = 0;
    for (int i = 1; i < 64; i++) if ((b >> i) & 1) v ^= a >> (64 - i);
    return v;
}
__device__ __forceinline__ uint64_t div64(uint64_t a, uint64_t b) {
    const int64_t x = (int64_t)a, y = (int64_t)b;
    return y == 0 ? ~0ULL : (x == INT64_MIN && y == -1) ? (uint64_t)x : (uint64_t)(x / y);
}
__device__ __forceinline__ uint64_t rem64(uint64_t a, uint64_t b) {
    const int64_t x = (int64_t)a, y = (int64_t)b;
    return y == 0 ? a : (x == INT64_MIN && y == -1) ? 0 : (uint64_t)(x % y);
}
__device__ __forceinline__ uint64_t divw(uint64_t a, uint64_t b) {
    const int32_t x = (int32_t)a, y = (int32_t)b;
    const int32_t q = y == 0 ? -1 : (x == INT32_MIN && y == -1) ? x : x / y;
    return (uint64_t)(int64_t)q;
}
__device__ __forceinline__ uint64_t remw(uint64_t a, uint64_t b) {
    const int32_t x = (int32_t)a, y = (int32_t)b;
    const int32_t r = y == 0 ? x : (x == INT32_MIN && y == -1) ? 0 : x % y;
    return (uint64_t)(int64_t)r;
}
__device__ __forceinline__ uint64_t rolw(uint64_t a, uint64_t b) {
    const uint32_t x = (uint32_t)a;
    const int sh = (int)(b & 31);
    return sx32((x << sh) | (x >> ((32 - sh) & 31)));
}
__device__ __forceinline__ uint64_t rorw(uint64_t a, uint64_t b) {
    const uint32_t x = (uint32_t)a;
    const int sh = (int)(b & 31);
    return sx32((x >> sh) | (x << ((32 - sh) & 31)));
}

// ------------------------------------------------------------------ memory
struct LaneMem {
    uint64_t stack_min;
    uint64_t tv0, tv1, tv2, tv3;   // TLB vpns (kNone = empty)
    uint64_t tp0, tp1, tp2, tp3;   // page address | 1 if the page is the lane's private copy
    uint32_t tnext;
    uint32_t n_priv;
    uint64_t req_vpn;              // pending copy-on-write, kNone = none
    const uint8_t *req_src;
    bool code_dirty;
    uint64_t dlo, dhi;             // bounding range of the code bytes the lane rewrote (valid if code_dirty)
    // LR/SC: the ISA's load reservation (isa.cc:1006-1064) and this context's
    // lock record in memory (abstract_mem.cc:258-345), as virtual addresses
    // (the SE mapping is a per-page bijection); kNone = none.  A lane holding a
    // lock record stays on the general path, whose stores erase it.
    uint64_t resv, lock;
    bool vm;                       // VmState of the slot is live (the trial made a VM syscall)
    uint32_t vcfg;                 // vector configuration (vtype, vl) as oracle/rv64se.c vcfg_of; 0 = process start
    uint32_t nmiss;                // diagnostics: full page-table lookups (TLB misses)
    uint32_t *dl;                  // solo kernel: LDS copy of the slot's rewritten-code map (else NULL)
};
// solo_fast_run reads the TLB as tv0..tv3 then tp0..tp3, 8-byte aligned
static_assert(__builtin_offsetof(LaneMem, tv0) % 8 == 0 &&
              __builtin_offsetof(LaneMem, tp0) == __builtin_offsetof(LaneMem, tv0) + 32, "LaneMem TLB layout");

// Rewritten code, exactly: DevCtx::dmap holds per slot one bit per
// 2^dmap_shift-byte granule of [code_lo, code_hi) the lane stored into
// (zeroed at its first such store); [dlo, dhi) bounds them.  The solo kernel
// keeps an LDS copy (LaneMem::dl) and asks the map; the 64-lane kernel asks
// the bounding range only (conservative).
// (out of line: called only for a lane whose bounding range meets [lo, hi),
// and the translated bodies check at every block)
// (word-wise: granules g0..g1, the end words masked)
template <typename P>
__device__ __forceinline__ bool dmap_bits(P dl, uint32_t g0, uint32_t g1) {
    const uint32_t w0 = g0 >> 5, w1 = g1 >> 5;
    for (uint32_t wi = w0; wi <= w1; wi++) {
        uint32_t b = dl[wi];
        if (wi == w0) b &= ~0u << (g0 & 31);
        if (wi == w1) b &= ~0u >> (31 - (g1 & 31));
        if (b) return true;
    }
    return false;
}
__device__ __noinline__ bool dmap_test(KCtx *c, const uint32_t *dl, uint64_t lo, uint64_t hi) {
    const uint64_t a = lo > c->code_lo ? lo : c->code_lo, b = hi < c->code_hi ? hi : c->code_hi;
    if (a >= b) return false;
    const uint32_t sh = c->dmap_shift;
    return dmap_bits(dl, (uint32_t)((a - c->code_lo) >> sh), (uint32_t)((b - 1 - c->code_lo) >> sh));
}
// The same test inline, on the solo kernel's LDS copy of the map (at most a
// few granules: an instruction's 6 bytes, or one translated block).
__device__ __forceinline__ bool dmap_any(const __attribute__((address_space(3))) uint32_t *dl, uint64_t clo,
                                         uint64_t chi, uint32_t sh, uint64_t lo, uint64_t hi) {
    const uint64_t a = lo > clo ? lo : clo, b = hi < chi ? hi : chi;
    if (a >= b) return false;
    return dmap_bits(dl, (uint32_t)((a - clo) >> sh), (uint32_t)((b - 1 - clo) >> sh));
}
__device__ __forceinline__ bool dirty_range(KCtx *c, const LaneMem &m, uint64_t lo, uint64_t hi) {
    if (!m.code_dirty || lo >= m.dhi || hi <= m.dlo) return false;
    return !m.dl || dmap_test(c, m.dl, lo, hi);
}
// The golden pre-decode of the instruction at pc is stale for this lane only if
// the lane rewrote one of its bytes (conservatively [pc & ~3, pc + 6)).
__device__ __forceinline__ bool dirty_at(KCtx *c, const LaneMem &m, uint64_t pc) {
    return m.code_dirty && dirty_range(c, m, pc & ~3ULL, pc + 6);
}
// Does the lane's rewritten range come within kTxNear bytes after pc?  A
// translated block that would meet it exits there (an entry and an exit for a
// few instructions), so such lanes stay in the pre-decoded path instead.
constexpr uint64_t kTxNear = 256;
__device__ __forceinline__ bool dirty_near(const LaneMem &m, uint64_t pc) {
    return m.code_dirty && (pc & ~3ULL) < m.dhi && pc + kTxNear > m.dlo;
}
__device__ __noinline__ void dmap_mark(KCtx *c, uint32_t *dl, uint64_t slot, uint64_t lo, uint64_t hi, bool fresh) {
    uint32_t *g = c->dmap + slot * c->dmap_words;
    if (fresh)
        for (uint32_t i = 0; i < c->dmap_words; i++) g[i] = 0;   // (the solo kernel's LDS copy starts zeroed)
    const uint64_t a = lo > c->code_lo ? lo : c->code_lo, b = hi < c->code_hi ? hi : c->code_hi;
    if (a >= b) return;
    const uint32_t sh = c->dmap_shift;
    for (uint32_t q = (uint32_t)((a - c->code_lo) >> sh); q <= (uint32_t)((b - 1 - c->code_lo) >> sh); q++) {
        g[q >> 5] |= 1u << (q & 31);
        if (dl) dl[q >> 5] |= 1u << (q & 31);
    }
}
__device__ __forceinline__ void mark_dirty(KCtx *c, LaneMem &m, uint64_t slot, uint64_t lo, uint64_t hi) {
    const bool fresh = !m.code_dirty;
    m.dlo = fresh ? lo : (lo < m.dlo ? lo : m.dlo);
    m.dhi = fresh ? hi : (hi > m.dhi ? hi : m.dhi);
    m.code_dirty = true;
    if (c->dmap) dmap_mark(c, m.dl, slot, lo, hi, fresh);
}
// A translated solo store into the code range (at most 8 bytes): the bounding
// range and the LDS map only -- the solo kernel's map lives in LDS (copied to
// the slot's global map when the lane suspends), which it zeroes at a fresh
// start, so nothing needs clearing here.
__device__ __forceinline__ void mark_dirty_solo(KCtx *c, LaneMem &m, uint64_t lo, uint64_t hi) {
    const bool fresh = !m.code_dirty;
    m.dlo = fresh ? lo : (lo < m.dlo ? lo : m.dlo);
    m.dhi = fresh ? hi : (hi > m.dhi ? hi : m.dhi);
    m.code_dirty = true;
    if (!m.dl) return;
    const uint64_t a = lo > c->code_lo ? lo : c->code_lo, b = hi < c->code_hi ? hi : c->code_hi;
    if (a >= b) return;
    const uint32_t q0 = (uint32_t)((a - c->code_lo) >> c->dmap_shift), q1 = (uint32_t)((b - 1 - c->code_lo) >> c->dmap_shift);
    for (uint32_t q = q0; q <= q1; q++) m.dl[q >> 5] |= 1u << (q & 31);   // (at most 8 granules)
}

// The lane's start-snapshot page table (uniform in a fresh launch; per lane
// after a resume).
struct WaveMem {
    const PageEnt *tab;
    uint32_t tab_n;
};

// Private entry i of a slot: the first P in the slot's own frames and SoA
// vpn table, the rest in its overflow block (DevCtx::ov_*; priv_room hands
// the block out when entry P is needed).
__device__ __noinline__ uint8_t *ov_frame(KCtx *c, uint64_t slot, uint32_t i) {
    return c->ov_frames + (((uint64_t)c->ov_of[slot] * c->ov_pages + (i - c->priv_pages)) << 12);
}
__device__ __noinline__ uint64_t *ov_ent(KCtx *c, uint64_t slot, uint32_t i) {
    return c->ov_vpn + (uint64_t)c->ov_of[slot] * c->ov_pages + (i - c->priv_pages);
}
__device__ __forceinline__ uint8_t *priv_frame(KCtx *c, uint64_t slot, uint32_t i) {
    if (i < c->priv_pages) return c->priv_frames + ((slot * c->priv_pages + i) << 12);
    return ov_frame(c, slot, i);   // (rare: out of line)
}
__device__ __forceinline__ uint64_t &priv_ent(KCtx *c, uint64_t slot, uint32_t i) {
    if (i < c->priv_pages) return c->priv_vpn[(uint64_t)i * c->n_slots + slot];
    return *ov_ent(c, slot, i);
}
// May the slot take private entry i (= its n_priv)?  Past P it needs its
// overflow block, taken from the pool at entry P; none left (or no pool): no.
__device__ __noinline__ bool priv_room_ool(KCtx *c, uint64_t slot, uint32_t i) {
    if (!c->ov_blocks || i >= c->priv_pages + c->ov_pages) return false;
    if (c->ov_of[slot] == 0xFFFFFFFFu) {
        if (i != c->priv_pages) return false;
        const uint32_t b = atomicAdd(c->ov_next, 1u);
        if (b >= c->ov_blocks) return false;
        c->ov_of[slot] = b;
        atomicAdd(&c->stats[61], 1ull);   // (blocks taken: diagnostics)
    }
    return true;
}
__device__ __forceinline__ bool priv_room(KCtx *c, uint64_t slot, uint32_t i) {
    return i < c->priv_pages || priv_room_ool(c, slot, i);
}

__device__ __forceinline__ uint64_t tlb_find(const LaneMem &m, uint64_t vpn) {
    uint64_t r = 0;
    r = m.tv0 == vpn ? m.tp0 : r;
    r = m.tv1 == vpn ? m.tp1 : r;
    r = m.tv2 == vpn ? m.tp2 : r;
    r = m.tv3 == vpn ? m.tp3 : r;
    return r;
}
__device__ __forceinline__ void tlb_flush(LaneMem &m) { m.tv0 = m.tv1 = m.tv2 = m.tv3 = kNone; }
__device__ __forceinline__ void tlb_insert(LaneMem &m, uint64_t vpn, uint64_t p) {
    const uint32_t k = m.tnext & 3;
    m.tv0 = k == 0 ? vpn : m.tv0; m.tp0 = k == 0 ? p : m.tp0;
    m.tv1 = k == 1 ? vpn : m.tv1; m.tp1 = k == 1 ? p : m.tp1;
    m.tv2 = k == 2 ? vpn : m.tv2; m.tp2 = k == 2 ? p : m.tp2;
    m.tv3 = k == 3 ? vpn : m.tv3; m.tp3 = k == 3 ? p : m.tp3;
    m.tnext++;
}

// Binary search of a snapshot page table (sorted by vpn): frame or -1.
__device__ __forceinline__ int64_t tab_find(const PageEnt *t, uint32_t n, uint64_t vpn) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (t[mid].vpn < vpn) lo = mid + 1; else hi = mid;
    }
    return (lo < n && t[lo].vpn == vpn) ? (int64_t)t[lo].frame : -1;
}

// SE translation = EmulationPageTable::translate (src/mem/page_table.cc:143-153)
// over the lane's page set: its private pages, then the start snapshot's
// pages, then the stack pages [stack_min, top] that MemState::fixupFault
// (src/sim/mem_state.cc:387-447) has mapped and nobody has written (zero).
// The newest private entry of a vpn decides it; a tombstone entry (vpn |
// kTomb, left by munmap / brk shrink) means unmapped.
// Returns the page address | 1 for a private (writable) page, 0 if unmapped.
__device__ uint64_t lookup_full(KCtx *c, const WaveMem &w, LaneMem &m, uint64_t slot, uint64_t vpn) {
    m.nmiss++;
    uint64_t p = 0;
    bool dec = false;
    for (uint32_t i = m.n_priv; i-- > 0;) {
        const uint64_t e = priv_ent(c, slot, i);
        if ((e & ~kTomb) == vpn) { dec = true; if (!(e & kTomb)) p = (uint64_t)priv_frame(c, slot, i) | 1; break; }
    }
    if (!dec) {
        const int64_t f = tab_find(w.tab, w.tab_n, vpn);
        if (f >= 0) p = (uint64_t)(c->pool + ((uint64_t)f << 12));
        else if (vpn >= (m.stack_min >> 12) && vpn <= kStackTopVpn) p = (uint64_t)c->zero_page;
    }
    if (p) tlb_insert(m, vpn, p);
    return p;
}
__device__ __forceinline__ uint64_t lookup(KCtx *c, const WaveMem &w, LaneMem &m, uint64_t slot,
                                           uint64_t vpn) {
    const uint64_t p = tlb_find(m, vpn);
    return p ? p : lookup_full(c, w, m, slot, vpn);
}
__device__ __forceinline__ const uint8_t *page_of(uint64_t p) { return (const uint8_t *)(p & ~1ULL); }

// ------------------------------------------------------------------ SE memory map
// (syscall and fault paths only: one lane at a time, serial)
// The private entry that decides vpn (newest first), or -1.
__device__ int priv_decider(KCtx *c, const LaneMem &m, uint64_t slot, uint64_t vpn) {
    for (uint32_t i = m.n_priv; i-- > 0;)
        if ((priv_ent(c, slot, i) & ~kTomb) == vpn) return (int)i;
    return -1;
}
// Process::allocateMem of one page for this trial: a new private entry filled
// from src (the zero page, or the current page for a proxy write).  nullptr if
// the trial has no free private page (resource escape).
__device__ uint8_t *priv_new(KCtx *c, LaneMem &m, uint64_t slot, uint64_t vpn, const uint8_t *src) {
    if (!priv_room(c, slot, m.n_priv)) return nullptr;
    uint4 *d = (uint4 *)priv_frame(c, slot, m.n_priv);
    const uint4 *q = (const uint4 *)src;
    for (int k = 0; k < 256; k++) d[k] = q[k];
    priv_ent(c, slot, m.n_priv) = vpn;
    m.n_priv++;
    tlb_flush(m);
    return (uint8_t *)d;
}
// The trial's VM state, materialised from the start one on first use: the
// checkpoint's (vm0) or the process-start one.
__device__ VmState *vm_of(KCtx *c, LaneMem &m, uint64_t slot) {
    VmState *v = c->vm + slot;
    if (!m.vm) {
        if (c->vm0) {
            const VmState *z = c->vm0;
            v->brk = z->brk; v->mmap_end = z->mmap_end; v->ctid = z->ctid; v->rnd_pos = z->rnd_pos;
            v->nvma = z->nvma; v->fdc = z->fdc;
            for (uint32_t i = 0; i < z->nvma; i++) { v->vma[i][0] = z->vma[i][0]; v->vma[i][1] = z->vma[i][1]; }
        } else {
            v->brk = c->brk0; v->mmap_end = 0x4000000000000000ULL; v->ctid = 0;   // RiscvProcess64 (process.cc:79)
            v->rnd_pos = 0;
            v->nvma = 1; v->fdc = 0;
            v->vma[0][0] = c->svma_lo; v->vma[0][1] = c->svma_hi;                 // argsInit's "stack" VMA
        }
        m.vm = true;
        if (c->record) c->stats[22] = 1;   // the golden VM state is not in the snapshots
    }
    return v;
}
__device__ bool in_vma(KCtx *c, const LaneMem &m, uint64_t slot, uint64_t a) {
    if (!m.vm && !c->vm0) return a >= c->svma_lo && a < c->svma_hi;
    const VmState *v = m.vm ? c->vm + slot : c->vm0;
    for (uint32_t i = 0; i < v->nvma; i++)
        if (a >= v->vma[i][0] && a < v->vma[i][1]) return true;
    return false;
}
// MemState::fixupFault (mem_state.cc:387-447): 1 handled, 0 not (panic),
// -1 fatal "Maximum stack size exceeded", -2 no free private page.
__device__ int fixup_fault(KCtx *c, LaneMem &m, uint64_t slot, uint64_t fva) {
    if (in_vma(c, m, slot, fva) || (fva >= m.stack_min && fva < kStackBase))
        return priv_new(c, m, slot, fva >> 12, c->zero_page) ? 1 : -2;
    if (fva < m.stack_min && fva >= kStackBase - kMaxStack) {
        const uint64_t nm = fva & ~4095ULL;
        if (kStackBase - nm > kMaxStack) return -1;
        m.stack_min = nm;   // [nm, old stack_min) are zero pages of the trial's set
        return 1;
    }
    return 0;
}
// Calls f(vpn, decider) for every page of the trial's set in vpns [lo, hi)
// until f returns false.
template <typename F>
__device__ __forceinline__ void for_mapped(KCtx *c, const WaveMem &w, const LaneMem &m, uint64_t slot, uint64_t lo,
                                           uint64_t hi, F f) {
    for (uint32_t i = m.n_priv; i-- > 0;) {
        const uint64_t e = priv_ent(c, slot, i);
        if ((e & kTomb) || e < lo || e >= hi || priv_decider(c, m, slot, e) != (int)i) continue;
        if (!f(e, (int)i)) return;
    }
    uint32_t a = 0, b = w.tab_n;
    while (a < b) {
        const uint32_t mid = (a + b) >> 1;
        if (w.tab[mid].vpn < lo) a = mid + 1; else b = mid;
    }
    for (; a < w.tab_n && w.tab[a].vpn < hi; a++)
        if (priv_decider(c, m, slot, w.tab[a].vpn) < 0 && !f(w.tab[a].vpn, -1)) return;
    for (uint64_t v = lo > (m.stack_min >> 12) ? lo : (m.stack_min >> 12); v < hi && v <= kStackTopVpn; v++)
        if (tab_find(w.tab, w.tab_n, v) < 0 && priv_decider(c, m, slot, v) < 0 && !f(v, -1)) return;
}
// MemState::isUnmapped (mem_state.cc:82-104): 1 unmapped, 0 a VMA intersects,
// -1 panic (a page is mapped without a VMA)
__device__ int vm_is_unmapped(KCtx *c, const WaveMem &w, LaneMem &m, uint64_t slot, uint64_t lo, uint64_t len) {
    const VmState *v = c->vm + slot;
    const uint64_t hi = lo + len;
    for (uint32_t i = 0; i < v->nvma; i++)
        if (v->vma[i][0] < hi && lo < v->vma[i][1]) return 0;
    bool any = false;
    for_mapped(c, w, m, slot, lo >> 12, (hi + 4095) >> 12, [&](uint64_t, int) { any = true; return false; });
    return any ? -1 : 1;
}
// A resource escape's exit code: 0 = the trial ran out of private pages (the
// redo pass runs it again with more, fi_kernels.hip fi_redo_collect_kernel),
// kEscTable = a table both the engine and the oracle bound (the VMA list, the
// precomputed getrandom stream): more pages would not change it.
constexpr int kEscTable = 1;
// MemState::mapRegion (mem_state.cc:172-189); false = the list is full
__device__ bool vm_add(VmState *v, uint64_t lo, uint64_t hi) {
    if (lo >= hi) return true;
    if (v->nvma == kMaxVma) return false;
    v->vma[v->nvma][0] = lo; v->vma[v->nvma][1] = hi; v->nvma++;
    return true;
}
// MemState::unmapRegion (mem_state.cc:191-276) + Process::deallocateMem
// (process.cc:348-382): the VMAs lose [lo, hi), the mapped pages in it leave
// the trial's set (a private entry turns into a tombstone, a snapshot or zero
// stack page gets one).  0 ok, 1 no private page left, 2 the VMA list is full
// (resource escapes; exit code kEscTable for the latter, vm_esc).
__device__ int vm_unmap(KCtx *c, const WaveMem &w, LaneMem &m, uint64_t slot, VmState *v, uint64_t lo, uint64_t hi) {
    if (c->record) c->stats[62] = 1;   // frames freed: the tick model's frame order no longer holds
    const uint32_t n = v->nvma;
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t a = v->vma[i][0], b = v->vma[i][1];
        if (!(a < hi && lo < b)) continue;
        if (a < lo && b > hi) {
            v->vma[i][1] = lo;
            if (!vm_add(v, hi, b)) return 2;
        } else if (a >= lo && b <= hi) {
            v->vma[i][0] = v->vma[i][1] = 0;
        } else if (a < lo) {
            v->vma[i][1] = lo;
        } else {
            v->vma[i][0] = hi;
        }
    }
    uint32_t k = 0;
    for (uint32_t i = 0; i < v->nvma; i++)
        if (v->vma[i][0] < v->vma[i][1]) { v->vma[k][0] = v->vma[i][0]; v->vma[k][1] = v->vma[i][1]; k++; }
    v->nvma = k;
    bool full = false;
    for_mapped(c, w, m, slot, lo >> 12, hi >> 12, [&](uint64_t vpn, int d) {
        if (d >= 0) {
            priv_ent(c, slot, (uint32_t)d) = vpn | kTomb;
        } else if (priv_room(c, slot, m.n_priv)) {
            priv_ent(c, slot, m.n_priv) = vpn | kTomb;
            m.n_priv++;
        } else {
            full = true;
            return false;
        }
        return true;
    });
    tlb_flush(m);
    if (lo < c->code_hi && hi > c->code_lo) mark_dirty(c, m, slot, lo, hi);   // the pre-decoded text no longer applies
    return full ? 1 : 0;
}
// Readable through SETranslatingPortProxy (no fixups on reads)
__device__ bool proxy_readable(KCtx *c, const WaveMem &w, LaneMem &m, uint64_t slot, uint64_t a, uint64_t n) {
    if (!n) return true;
    const uint64_t last = a + n - 1;
    if (last < a) return false;
    for (uint64_t v = a >> 12; v <= (last >> 12); v++)
        if (!lookup(c, w, m, slot, v)) return false;
    return true;
}
__device__ uint8_t proxy_byte(KCtx *c, const WaveMem &w, LaneMem &m, uint64_t slot, uint64_t a) {
    return page_of(lookup(c, w, m, slot, a >> 12))[a & 4095];
}
// A write through the proxy (NextPage: fixupFault for each missing page):
// 1 ok, 0 fatal, -1 stack limit, -2 no free private page
__device__ int proxy_writable(KCtx *c, const WaveMem &w, LaneMem &m, uint64_t slot, uint64_t a, uint64_t n) {
    if (!n) return 1;
    const uint64_t last = a + n - 1;
    if (last < a) return 0;
    for (uint64_t v = a >> 12; v <= (last >> 12); v++) {
        if (lookup(c, w, m, slot, v)) continue;
        const int h = fixup_fault(c, m, slot, (v << 12) > a ? (v << 12) : a);
        if (h != 1) return h;
    }
    return 1;
}
// Store bytes through the proxy (every page mapped): copy-on-write as needed.
// false = no free private page.
__device__ bool proxy_write(KCtx *c, const WaveMem &w, LaneMem &m, uint64_t slot, uint64_t a, const char *src,
                            uint64_t n) {
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t x = a + i;
        uint64_t p = lookup(c, w, m, slot, x >> 12);
        if (!(p & 1)) {
            uint8_t *q = priv_new(c, m, slot, x >> 12, page_of(p));
            if (!q) return false;
            p = (uint64_t)q | 1;
        }
        const_cast<uint8_t *>(page_of(p))[x & 4095] = (uint8_t)src[i];
    }
    if (a < c->code_hi && a + n > c->code_lo) mark_dirty(c, m, slot, a, a + n);
    return true;
}

enum { F_NONE = 0, F_SYSCALL, F_BREAK, F_ILLEGAL, F_UNKNOWN, F_ESCAPE, F_ESCCSR, F_PGFAULT, F_NEEDPAGE, F_DETECT,
       F_AMOLINE, F_SCLINE, F_M5PANIC, F_UNDEF, F_VSEW, F_TKCLOCK };

// AtomicSimpleCPU::readMem/writeMem (atomic.cc:331-544): the access is split
// at 64-byte line boundaries, each fragment translated on its own; faults are
// raised in fragment order.  Writes to a shared page request a copy-on-write
// page first (not a gem5 event: the tick is retried).  llsc: 1 = LR (each
// fragment read sets the reservation and the lock record), 2 = SC (val in:
// data, out: 1 if the store was performed), 3 = AMO.  Plain stores erase the
// lock record of their fragment's 16-byte granule (abstract_mem.cc:290-345);
// AMOs do not.
__device__ int mem_access(KCtx *c, const WaveMem &w, LaneMem &m, uint64_t slot, uint64_t ea,
                          uint32_t size, bool wr, uint64_t &val, uint64_t &fva, int llsc) {
    uint32_t n1 = 64 - (uint32_t)(ea & 63);
    if (n1 > size) n1 = size;
    if (ea + n1 - 1 < ea) { fva = ea; return F_PGFAULT; }
    const uint64_t p1 = lookup(c, w, m, slot, ea >> 12);
    if (!p1) { fva = ea; return F_PGFAULT; }
    const uint64_t ea2 = ea + n1;
    const uint32_t off = (uint32_t)(ea & 4095);
    if (llsc == 2) {
        // SC (atomic.cc:437-544, ISA::handleLockedWrite isa.cc:1015-1060):
        // the ISA check after translation clears the reservation either way;
        // memory performs a passing store only if this context's lock record
        // is the fragment's granule, then erases it.  A second fragment trips
        // assert(curr_frag_id == 0) after its translation.
        if (!(p1 & 1)) { m.req_vpn = ea >> 12; m.req_src = page_of(p1); return F_NEEDPAGE; }
        const bool pass = m.resv != kNone && (m.resv & ~63ULL) == (ea & ~63ULL);
        m.resv = kNone;
        const bool ok = pass && m.lock == (ea & ~0xFULL);
        if (ok) {
            uint8_t *w1 = const_cast<uint8_t *>(page_of(p1));
            for (uint32_t i = 0; i < n1; i++) w1[off + i] = (uint8_t)(val >> (8 * i));
            if (ea < c->code_hi && ea + n1 > c->code_lo) mark_dirty(c, m, slot, ea, ea + n1);
            m.lock = kNone;
        }
        val = ok ? 1 : 0;
        if (n1 < size) {
            if (ea2 + (size - n1) - 1 < ea2 || !lookup(c, w, m, slot, ea2 >> 12)) { fva = ea2; return F_PGFAULT; }
            return F_SCLINE;
        }
        return F_NONE;
    }
    uint64_t p2 = p1;
    if (n1 < size) {
        if (ea2 + (size - n1) - 1 < ea2) { fva = ea2; if (llsc) { m.resv = ea; m.lock = ea & ~0xFULL; } return F_PGFAULT; }
        p2 = lookup(c, w, m, slot, ea2 >> 12);
        if (!p2) { fva = ea2; if (llsc) { m.resv = ea; m.lock = ea & ~0xFULL; } return F_PGFAULT; }
    }
    if (wr) {
        if (!(p1 & 1)) { m.req_vpn = ea >> 12; m.req_src = page_of(p1); return F_NEEDPAGE; }
        if (!(p2 & 1)) { m.req_vpn = ea2 >> 12; m.req_src = page_of(p2); return F_NEEDPAGE; }
        if (ea < c->code_hi && ea + size > c->code_lo) mark_dirty(c, m, slot, ea, ea + size);   // the lane rewrote its code
        uint8_t *w1 = const_cast<uint8_t *>(page_of(p1));
        if (n1 == size && (off & (size - 1)) == 0) {
            switch (size) {
            case 1: w1[off] = (uint8_t)val; break;
            case 2: *(uint16_t *)(w1 + off) = (uint16_t)val; break;
            case 4: *(uint32_t *)(w1 + off) = (uint32_t)val; break;
            case 64:   // cbo.zero: the 64-byte line (val is 0)
                for (int k = 0; k < 8; k++) *(uint64_t *)(w1 + off + 8 * k) = 0;
                break;
            default: *(uint64_t *)(w1 + off) = val; break;
            }
        } else {
            uint8_t *w2 = const_cast<uint8_t *>(page_of(p2));
            for (uint32_t i = 0; i < size; i++) (i < n1 ? w1 : w2)[(ea + i) & 4095] = (uint8_t)(val >> (8 * i));
        }
        // (an AMO's write, llsc == 3, leaves the lock records alone: atomic.cc:546-608)
        if (llsc != 3 && (m.lock == (ea & ~0xFULL) || (n1 < size && m.lock == (ea2 & ~0xFULL)))) m.lock = kNone;
    } else {
        const uint8_t *r1 = page_of(p1);
        uint64_t v = 0;
        if (n1 == size && (off & (size - 1)) == 0) {
            switch (size) {
            case 1: v = r1[off]; break;
            case 2: v = *(const uint16_t *)(r1 + off); break;
            case 4: v = *(const uint32_t *)(r1 + off); break;
            default: v = *(const uint64_t *)(r1 + off); break;
            }
        } else {
            const uint8_t *r2 = page_of(p2);
            for (uint32_t i = 0; i < size; i++) v |= (uint64_t)(i < n1 ? r1 : r2)[(ea + i) & 4095] << (8 * i);
        }
        val = v;
        if (llsc) {   // LR: the last fragment read holds the reservation (ISA::handleLockedRead, trackLoadLocked)
            m.resv = n1 < size ? ea2 : ea;
            m.lock = m.resv & ~0xFULL;
        }
    }
    return F_NONE;
}

// Slow-path fetch of one lane: Decoder::moreBytes + setupFetchRequest
// (src/arch/riscv/decoder.cc:63-116, src/cpu/simple/base.cc:304-318).
// Returns 0 ok, or F_PGFAULT with the faulting fetch address and the number of
// ticks consumed (1 if the first word faulted, 2 if the second did).
__device__ int fetch_lane(KCtx *c, const WaveMem &w, LaneMem &m, uint64_t slot, uint64_t pc, uint32_t &raw,
                          uint32_t &ticks, uint64_t &fva) {
    const uint64_t w0 = pc & ~3ULL;
    ticks = 1;
    const uint64_t p0 = lookup(c, w, m, slot, w0 >> 12);
    if (!p0) { fva = w0; return F_PGFAULT; }
    const uint32_t word = *(const uint32_t *)(page_of(p0) + (w0 & 4095));
    if ((pc & 3) == 0) {
        raw = ((word & 3) != 3) ? (word & 0xFFFF) : word;
        return F_NONE;
    }
    const uint32_t half = word >> 16;
    if ((half & 3) != 3) { raw = half; return F_NONE; }
    ticks = 2;
    const uint64_t w1 = w0 + 4;
    const uint64_t p1 = lookup(c, w, m, slot, w1 >> 12);
    if (!p1) { fva = w1; return F_PGFAULT; }
    const uint32_t word2 = *(const uint32_t *)(page_of(p1) + (w1 & 4095));
    raw = half | ((word2 & 0xFFFF) << 16);
    return F_NONE;
}

// ------------------------------------------------------------------ syscalls
// RV64 Linux SE syscall table classification (src/arch/riscv/linux/
// se_workload.cc:529-895); 0 absent, 1 unimplemented, 2 ignore, 3 escape,
// 4 modelled.
__device__ int sys_class(int num) {
    switch (num) {   // modelled (oracle/rv64se.c:sys_modelled)
    case 29: case 57: case 63: case 64: case 66: case 78: case 93: case 94: case 96: case 113: case 160: case 163:
    case 214: case 215: case 222: case 258: case 261: case 278: case 1058:
        return 4;
    default:
        if (num >= 172 && num <= 178) return 4;
    }
    const bool present = (num >= 0 && num <= 64) || (num >= 66 && num <= 243) || num == 258 ||
                         (num >= 260 && num <= 287) || (num >= 424 && num <= 450) ||
                         (num >= 1024 && num <= 1079) || num == 2011;
    if (!present) return 0;
    if (num == 99 || num == 100 || num == 101 || num == 124 || (num >= 133 && num <= 139) || num == 146 ||
        num == 164 || (num >= 226 && num <= 233) || num == 235)
        return 2;
    switch (num) {   // gem5 handlers not modelled on the device (escape)
    case 17: case 23: case 25: case 29: case 33: case 34: case 35: case 38: case 43: case 44: case 45: case 46:
    case 47: case 48: case 49: case 52: case 55: case 56: case 57: case 59: case 61: case 62: case 63: case 66:
    case 67: case 68: case 78: case 79: case 80: case 96: case 98: case 113: case 114: case 121: case 123:
    case 131: case 153: case 154: case 160: case 163: case 165: case 166: case 168: case 169: case 179:
    case 198: case 199: case 200: case 201: case 202: case 203: case 204: case 205: case 206: case 207:
    case 208: case 209: case 210: case 211: case 212: case 214: case 215: case 216: case 220: case 221:
    case 222: case 258: case 260: case 261: case 278: case 435:
    case 1024: case 1025: case 1026: case 1027: case 1028: case 1029: case 1030: case 1031: case 1033:
    case 1034: case 1035: case 1036: case 1037: case 1038: case 1039: case 1040: case 1041: case 1044:
    case 1047: case 1048: case 1049: case 1050: case 1051: case 1052: case 1054: case 1055: case 1056:
    case 1057: case 1058: case 1060: case 1062: case 1065: case 1067: case 1068:
        return 3;
    default:
        return 1;
    }
}

// U-mode CSR reachability (CSRExecute, src/arch/riscv/isa/formats/standard.isa:
// 325-447 and the CSRData map, src/arch/riscv/regs/misc.hh:604-1241).
__device__ __forceinline__ bool csr_u_accessible(uint32_t csr) {
    if ((csr >> 8) & 3) return false;
    return (csr >= 0x001 && csr <= 0x003) || (csr >= 0x008 && csr <= 0x00A) || csr == 0x00F || csr == 0x017 ||
           (csr >= 0xC00 && csr <= 0xC1F) || (csr >= 0xC20 && csr <= 0xC22);
}

struct Lane {
    uint64_t pc, ninst, ncyc;
    uint64_t out_pos, err_pos;
    uint64_t fetch_b, data_b;
    uint64_t next_chk;            // next snapshot boundary to compare at (kNone = none)
    uint32_t nfail;               // failed comparisons (back-off)
    int watch;
    bool out_bad, done;
    bool fp;                      // FP registers materialised (else all zero, as at process start)
    uint8_t fflags, frm;          // MISCREG_FFLAGS / MISCREG_FRM (zero at process start)
    uint8_t injected;             // 0 pending, 1 applied, 2 nothing to flip, 3 result fault armed
    fi_outcome res;
};

// gem5 OpClass of an executed op (generated from the reference's ISA
// description; tests/golden/opclass_rv64.json)
__device__ __forceinline__ uint32_t op_class(uint32_t op) {
    switch (op) {
#define FI_OPC(n, c) case OP_##n: return c;
        FI_GEM5_OPCLASS(FI_OPC)
#undef FI_OPC
    default: return 0;
    }
}
// SHREWD shadow execution: FUPool::getUnit(cap, is_shadow) (src/cpu/o3/
// fu_pool.cc:177-301) has a shadow unit only for IntAlu, IntMult, IntDiv and
// FloatAdd..FloatSqrt.  Without the issue model a protected class among them
// is always replicated; with it (fi_set_issue_model) only if the k-th golden
// instruction's shadow found a free unit (oracle/rv64se.c:replicated).  The
// target of a result fault is the golden instruction numInst = k: the trial
// equals the golden run up to its commit.
__device__ __forceinline__ bool replicated(KCtx *CX, uint32_t cls, uint64_t k) {
    if (!(cls >= FI_OPC_INTALU && cls <= FI_OPC_FLOATSQRT && ((CX->protect_opc >> cls) & 1))) return false;
    const uint32_t *sb = CX->shadow_bits;
    return !sb || k >= CX->gninst || ((sb[k >> 5] >> (k & 31)) & 1u);
}

// ------------------------------------------------------------------ F/D/Zfh + A
// FP registers live in HBM, [32][n_slots] (lane-coalesced), touched only by the
// FP data-movement ops of the general path; a lane that never wrote one reads
// zeros (RegFile is zeroed at process start).  NaN-boxing follows
// src/arch/riscv/regs/float.hh:72-107 (default NaNs 0x7e00 / 0x7fc00000).
__device__ __forceinline__ uint64_t fp_unbox32(uint64_t v) {
    return (v >> 32) == 0xFFFFFFFFULL ? (v & 0xFFFFFFFFULL) : 0x7FC00000ULL;
}
__device__ __forceinline__ uint64_t fp_unbox16(uint64_t v) {
    return (v >> 16) == 0xFFFFFFFFFFFFULL ? (v & 0xFFFF) : 0x7E00ULL;
}
// f16/f32/f64_classify (ext/softfloat/f32_classify.c, same shape per width)
__device__ __forceinline__ uint64_t fp_classify(uint64_t ui, int eb, int fb) {
    const uint64_t emax = (1ULL << eb) - 1, e = (ui >> fb) & emax, fr = ui & ((1ULL << fb) - 1);
    const bool sg = (ui >> (eb + fb)) & 1, infnan = e == emax, subz = e == 0, fz = fr == 0;
    const bool nan = infnan && !fz, snan = nan && !((fr >> (fb - 1)) & 1);
    int k;
    if (nan) k = snan ? 8 : 9;
    else if (infnan) k = sg ? 0 : 7;
    else if (subz) k = fz ? (sg ? 3 : 4) : (sg ? 2 : 5);
    else k = sg ? 1 : 6;
    return 1ULL << k;
}
// AtomicMemOp read-modify-write bodies (decoder.isa:2067-2283), op = 0 add,
// 1 swap, 2 xor, 3 or, 4 and, 5 min, 6 max, 7 minu, 8 maxu
__device__ __forceinline__ uint64_t amo_apply(int op, uint64_t mem, uint64_t src, bool w) {
    if (w) { mem &= 0xFFFFFFFFULL; src &= 0xFFFFFFFFULL; }
    const int64_t sm = w ? (int64_t)(int32_t)(uint32_t)mem : (int64_t)mem;
    const int64_t ss = w ? (int64_t)(int32_t)(uint32_t)src : (int64_t)src;
    switch (op) {
    case 0: return mem + src;
    case 1: return src;
    case 2: return mem ^ src;
    case 3: return mem | src;
    case 4: return mem & src;
    case 5: return ss < sm ? src : mem;
    case 6: return ss > sm ? src : mem;
    case 7: return src < mem ? src : mem;
    default: return src > mem ? src : mem;
    }
}

// F/D/Zfh arithmetic of one instruction (oracle/rv64se.c execute, FP cases):
// FloatExecute (formats/fp.isa:34-56) with RM_REQUIRED (fp_inst.hh:37-44),
// operands unboxed per format (float.hh), results boxed, except fminm/fmaxm's
// non-NaN result, which gem5 writes unboxed.  Out of line: rare, and big.
struct FpRes { uint64_t v; uint32_t fl, kind; };   // kind: 0 FP rd, 1 integer rd, 2 IllegalInst
__device__ __noinline__ FpRes fp_exec(uint32_t op, uint32_t imm, uint32_t rs2, uint64_t r1, uint64_t r2, uint64_t r3,
                                      uint64_t ia, uint32_t frm) {
    namespace sf = fi::sf;
    FpRes o;
    o.v = 0; o.fl = 0; o.kind = 0;
    const int fmt = (int)((imm >> 3) & 3), sub = (int)((imm >> 5) & 7);
    const uint64_t sgn = fmt == 0 ? 0x8000ULL : fmt == 1 ? 0x80000000ULL : 0x8000000000000000ULL;
    const uint64_t qnan = fmt == 0 ? 0x7E00ULL : fmt == 1 ? 0x7FC00000ULL : 0x7FF8000000000000ULL;
    const uint64_t inf = fmt == 0 ? 0x7C00ULL : fmt == 1 ? 0x7F800000ULL : 0x7FF0000000000000ULL;
    auto unbox = [](int f, uint64_t x) { return f == 0 ? fp_unbox16(x) : f == 1 ? fp_unbox32(x) : x; };
    auto box = [](int f, uint64_t x) {
        return f == 0 ? (0xFFFFFFFFFFFF0000ULL | x) : f == 1 ? (0xFFFFFFFF00000000ULL | x) : x;
    };
    const bool rounds = !(op == OP_fmin || op == OP_fmax || op == OP_feq || op == OP_flt || op == OP_fle ||
                          op == OP_fli);
    if (op == OP_fsqrt && rs2 != 0) { o.kind = 2; return o; }   // "source reg x1"
    int rm = (int)(imm & 7);
    if (rounds) {
        if (rm == 7) rm = (int)frm;
        if (rm > 4) { o.kind = 2; return o; }                   // "RM fault"
    }
    const uint64_t x = unbox(op == OP_fcvt_f2f ? sub : fmt, r1), y = unbox(fmt, r2), z = unbox(fmt, r3);
    uint32_t fl = 0;
    uint64_t r = 0;
    switch (op) {
    case OP_fadd: r = sf::op(sf::OP_ADD, fmt, rm, x, y, 0, fl); break;
    case OP_fsub: r = sf::op(sf::OP_SUB, fmt, rm, x, y, 0, fl); break;
    case OP_fmul: r = sf::op(sf::OP_MUL, fmt, rm, x, y, 0, fl); break;
    case OP_fdiv: r = sf::op(sf::OP_DIV, fmt, rm, x, y, 0, fl); break;
    case OP_fsqrt: r = sf::op(sf::OP_SQRT, fmt, rm, x, 0, 0, fl); break;
    case OP_fmadd: r = sf::op(sf::OP_FMA, fmt, rm, x, y, z, fl); break;
    case OP_fmsub: r = sf::op(sf::OP_FMA, fmt, rm, x, y, z ^ sgn, fl); break;
    case OP_fnmsub: r = sf::op(sf::OP_FMA, fmt, rm, x ^ sgn, y, z, fl); break;
    case OP_fnmadd: r = sf::op(sf::OP_FMA, fmt, rm, x ^ sgn, y, z ^ sgn, fl); break;
    case OP_fmin: case OP_fmax: {   // lt_quiet, then eq (decoder.isa:2944-3120)
        const bool mx = op == OP_fmax;
        const uint64_t p = mx ? y : x, q = mx ? x : y;
        bool pick = sf::op(sf::OP_LTQ, fmt, rm, p, q, 0, fl) != 0;
        if (!pick) pick = sf::op(sf::OP_EQ, fmt, rm, p, q, 0, fl) != 0 && (p & sgn);
        const bool nx = (x & ~sgn) > inf, ny = (y & ~sgn) > inf;
        if (sub) {
            o.fl = fl;
            o.v = (nx || ny) ? box(fmt, qnan) : (pick ? x : y);   // unboxed (Fd_bits = fs.v)
            return o;
        }
        r = (nx && ny) ? qnan : ((pick || ny) ? x : y);
        break;
    }
    case OP_feq: o.v = sf::op(sf::OP_EQ, fmt, rm, x, y, 0, fl); o.kind = 1; break;
    case OP_flt: o.v = sf::op(sub ? sf::OP_LTQ : sf::OP_LT, fmt, rm, x, y, 0, fl); o.kind = 1; break;
    case OP_fle: o.v = sf::op(sub ? sf::OP_LEQ : sf::OP_LE, fmt, rm, x, y, 0, fl); o.kind = 1; break;
    case OP_fcvt_f2i:   // w / wu sign-extended from 32 bits (decoder.isa:3273-3420)
        o.v = sf::op(sf::OP_TO_I32 + sub, fmt, rm, x, 0, 0, fl);
        if (sub <= 1) o.v = sx32(o.v);
        o.kind = 1;
        break;
    case OP_fcvt_i2f: r = sf::op(sf::OP_FROM_I32 + sub, fmt, rm, ia, 0, 0, fl); break;
    case OP_fli: {   // Zfa fli: table index in imm >> 8, no flags
        const uint32_t i = (imm >> 8) & 31;
        r = fmt == 0 ? sf::fli<sf::H>(i) : fmt == 1 ? sf::fli<sf::S>(i) : sf::fli<sf::D>(i);
        break;
    }
    case OP_fround: r = sf::op((sub & 1) ? sf::OP_RINTX : sf::OP_RINT, fmt, rm, x, 0, 0, fl); break;
    case OP_fcvtmod: o.v = sf::fcvtmod_w_d(x, fl); o.kind = 1; break;
    default: r = sf::op(sf::OP_TO_H + fmt, sub, rm, x, 0, 0, fl); break;   // between formats
    }
    o.fl = fl;
    if (o.kind == 0) o.v = box(fmt, r);
    return o;
}

__device__ __forceinline__ void finish(Lane &L, int cls, int sub, int code, uint32_t detail) {
    L.done = true;
    L.res.cls = (uint8_t)cls; L.res.sub = (uint8_t)sub; L.res.exit_code = (uint8_t)code;
    L.res.flags = (uint8_t)((L.injected ? 1 : 0) | (L.injected == 2 ? 2 : 0));
    L.res.detail = detail;
    L.res.ninst = L.ninst;
}

// Record mode: one data access of the golden run (the host builds the memory
// liveness index from them).  Not in the load-time build: the golden run is
// over before it exists.
__device__ __forceinline__ void rec_mem(KCtx *c, uint64_t a, uint64_t n, uint64_t t, uint32_t kind) {
#ifndef FI_TX
    while (n && kind) {
        const uint64_t k = n < (1u << 29) ? n : (1u << 29);
        const unsigned long long i = atomicAdd(&c->stats[25], 1ull);
        if (i < c->rec_mem_cap) {
            MemEv ev;
            ev.addr = a; ev.t = (uint32_t)t; ev.len_kind = (uint32_t)k | (kind << 30);
            c->rec_mem[i] = ev;
        }
        a += k; n -= k;
    }
#endif
}

// A memory fault (8-byte word at addr, xor mask, at numInst t) is dead when
// the golden run from t on never reads a flipped byte before writing it: the
// trial then executes exactly the golden run (a machine that differs only in
// bytes no instruction or syscall reads behaves identically), so its outcome
// is the golden one.  Instruction bytes are never dead (fetches are not in the
// index).
__device__ __noinline__ bool mem_dead(const KCtx *c, uint64_t addr, uint64_t mask, uint64_t t) {
    if (addr < c->text_hi && addr + 8 > c->text_lo) return false;
    uint32_t fb = 0;
    for (int b = 0; b < 8; b++) fb |= ((mask >> (8 * b)) & 0xFF) ? (1u << b) : 0u;
    uint32_t lo = 0, hi = c->mw_n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (c->mw_addr[mid] < addr) lo = mid + 1; else hi = mid;
    }
    if (lo == c->mw_n || c->mw_addr[lo] != addr) return true;   // never accessed again... or at all
    uint32_t a = c->mw_off[lo], b = c->mw_off[lo + 1];
    while (a < b) {   // first event at numInst >= t
        const uint32_t mid = (a + b) >> 1;
        if ((c->mw_ev[mid] >> 16) < t) a = mid + 1; else b = mid;
    }
    for (const uint32_t e = c->mw_off[lo + 1]; a < e; a++) {
        const uint64_t ev = c->mw_ev[a];
        if ((ev >> 8) & fb & 0xFF) return false;   // read while flipped
        fb &= ~(uint32_t)ev & 0xFF;                // overwritten: the golden value again
        if (!fb) return true;
    }
    return true;
}

#define RREG(r) R[(uint32_t)(r) * kNL + lane]

// The syscall path of one lane: EmuLinux::syscall (se_workload.cc:95-106)
// with the golden-output comparator folded into write()/writev().  Returns
// true if the trial's code mapping or bytes may have changed (the solo
// kernel's decode cache is dropped).
constexpr uint64_t kVmMaxLen = 1ULL << 43;   // == oracle/rv64se.c VM_MAX_LEN
template <uint32_t kNL>
__device__ __noinline__ bool do_syscall(KCtx *c, WaveMem w, Lane &L, LaneMem &m, uint64_t slot, uint64_t *R,
                                        uint32_t lane) {
    const int num = (int)(uint32_t)RREG(17);
    const int cls = sys_class(num);
    const uint32_t pc32 = (uint32_t)L.pc;
    if (cls == 0) { finish(L, FI_CRASH, FI_CRASH_SYSCALL_RANGE, 1, (uint32_t)num); return false; }
    if (cls == 1) { finish(L, FI_CRASH, FI_CRASH_SYSCALL_UNIMPL, 1, (uint32_t)num); return false; }
    if (cls == 3) { finish(L, FI_ESCAPE, FI_ESC_SYSCALL, 0, (uint32_t)num); return false; }
    if (cls == 2) { RREG(10) = 0; return false; }
    const uint64_t a0 = RREG(10), a1 = RREG(11), a2 = RREG(12), a3 = RREG(13), a4 = RREG(14), a5 = RREG(15);
    const uint32_t fdc = m.vm ? c->vm[slot].fdc : 0u;
    // the bytes [buf, buf + n) (all mapped) appended to stream fd (1 or 2)
    auto emit = [&](int fd, uint64_t buf, uint64_t n) {
        uint64_t &pos = fd == 1 ? L.out_pos : L.err_pos;
        const uint8_t *gold = fd == 1 ? c->gout : c->gerr;
        const uint64_t glen = fd == 1 ? c->gout_len : c->gerr_len;
        uint8_t *rec = fd == 1 ? c->rec_out : c->rec_err;
        uint64_t cur_vpn = kNone;
        const uint8_t *pg = nullptr;
        if (c->record) rec_mem(c, buf, n, L.ninst | kMemEvProxy, 1u);
        for (uint64_t i = 0; i < n; i++) {
            const uint64_t a = buf + i;
            if ((a >> 12) != cur_vpn) { cur_vpn = a >> 12; pg = page_of(lookup(c, w, m, slot, cur_vpn)); }
            const uint8_t ch = pg[a & 4095];
            const uint64_t p = pos + i;
            if (c->record) {
                if (p < c->rec_cap) rec[p] = ch;
            } else if (p >= glen || gold[p] != ch) {
                L.out_bad = true;
            }
        }
        pos += n;
    };
    auto rd64 = [&](uint64_t a) {
        if (c->record) rec_mem(c, a, 8, L.ninst | kMemEvProxy, 1u);
        uint64_t v = 0;
        for (int k = 0; k < 8; k++) v |= (uint64_t)proxy_byte(c, w, m, slot, a + k) << (8 * k);
        return v;
    };
    auto set_ret = [&](int64_t v) { RREG(10) = (uint64_t)v; };
    auto pwrite = [&](uint64_t a, const char *src, uint64_t n) {
        if (c->record) rec_mem(c, a, n, L.ninst | kMemEvProxy, 2u);
        return proxy_write(c, w, m, slot, a, src, n);
    };
    switch (num) {
    case 93: case 94: {  // exitImpl -> exitSimLoop(status & 0xff), sim/syscall_emul.cc:120-248
        const int code = (int)(uint32_t)a0 & 0xff;
        if (m.vm && c->vm[slot].ctid) {   // exitFutexWake: *childClearTID = 0 through the proxy (:106-117)
            const int h = proxy_writable(c, w, m, slot, c->vm[slot].ctid, 8);
            if (h == 0) { finish(L, FI_CRASH, FI_CRASH_PROXY, 1, pc32); return false; }
            if (h == -1) { finish(L, FI_CRASH, FI_CRASH_STACK_LIMIT, 1, pc32); return false; }
            if (h == -2) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, pc32); return false; }
        }
        if (c->record) {
            finish(L, FI_MASKED, 0, code, pc32);
            return false;
        }
        // masked: the golden run's output and exit code, ended the way it ended
        // (an exit syscall, not m5_exit / m5_fail: INTEGRATION.md, outcome classes)
        const bool same = !L.out_bad && L.out_pos == c->gout_len && L.err_pos == c->gerr_len && code == (int)c->gexit &&
                          c->gsub == FI_END_EXIT;
        finish(L, same ? FI_MASKED : FI_SDC, 0, code, pc32);
        return false;
    }
    case 172: case 178: set_ret(kPid); return false;
    case 173: set_ret(kPpid); return false;
    case 174: case 175: set_ret(kUid); return false;
    case 176: case 177: set_ret(kGid); return false;
    case 96:   // setTidAddressFunc (syscall_emul.cc:292-299)
        vm_of(c, m, slot)->ctid = a0;
        set_ret(kPid);
        return false;
    case 57: {   // closeFunc -> FDArray::closeFDEntry (fd_array.cc:334-352)
        const int fd = (int)(uint32_t)a0;
        if (fd < 0 || fd >= 1024) { set_ret(-9); return false; }
        if (fd <= 2) vm_of(c, m, slot)->fdc |= 1u << fd;
        set_ret(0);
        return false;
    }
    case 29: {   // ioctlFunc (syscall_emul.hh:743-813)
        const int fd = (int)(uint32_t)a0;
        const uint32_t req = (uint32_t)a1;
        if (!(req == 0x5401 || req == 0x5405 || req == 0x5407 || req == 0x541B) && (fd < 0 || fd >= 1024)) {
            finish(L, FI_CRASH, FI_CRASH_FD_ASSERT, 134, pc32);
            return false;
        }
        set_ret(-25);   // -ENOTTY
        return false;
    }
    case 214: {   // brkFunc (syscall_emul.cc:268-289), MemState::updateBrkRegion (mem_state.cc:107-170)
        VmState *v = vm_of(c, m, slot);
        const uint64_t nb = a0, ob = v->brk;
        if (nb == 0 || nb == ob) { set_ret((int64_t)ob); return false; }
        const uint64_t na = (nb + 4095) & ~4095ULL, oa = (ob + 4095) & ~4095ULL;
        if ((na > oa ? na - oa : oa - na) > kVmMaxLen) { finish(L, FI_ESCAPE, FI_ESC_SYSCALL, 0, 214u); return false; }
        if (nb < ob) {
            const int r = oa != na ? vm_unmap(c, w, m, slot, v, na, oa) : 0;
            if (r) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, r == 2 ? kEscTable : 0, pc32); return false; }
            v->brk = nb;
            set_ret((int64_t)nb);
            return true;
        }
        if (na > oa) {
            const int u = vm_is_unmapped(c, w, m, slot, oa, na - oa);
            if (u < 0) { finish(L, FI_CRASH, FI_CRASH_SE_PANIC, 134, pc32); return false; }
            if (!u) { set_ret((int64_t)ob); return false; }
            if (!vm_add(v, oa, na)) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, kEscTable, pc32); return false; }
        }
        v->brk = nb;
        set_ret((int64_t)nb);
        return false;
    }
    case 222: case 1058: {   // mmapFunc (syscall_emul.hh:2002-2126), anonymous mappings; MemState::extendMmap
        uint64_t start = a0, len = a1;
        const int flags = (int)(uint32_t)a3, fd = (int)(uint32_t)a4;
        if ((start & 4095) || (a5 & 4095) || ((flags & 2) && (flags & 1)) || (!(flags & 2) && !(flags & 1)) || !len) {
            set_ret(-22);
            return false;
        }
        if (len > kVmMaxLen) { finish(L, FI_ESCAPE, FI_ESC_SYSCALL, 0, 222u); return false; }
        len = (len + 4095) & ~4095ULL;
        if (!(flags & 0x20)) {
            if (fd < 0 || fd >= 1024) { finish(L, FI_CRASH, FI_CRASH_FD_ASSERT, 134, pc32); return false; }
            if (fd > 2 || ((fdc >> fd) & 1)) { set_ret(-9); return false; }
            finish(L, FI_ESCAPE, FI_ESC_HOST, 0, pc32);   // a host file mapping
            return false;
        }
        if (start + len < start) { finish(L, FI_ESCAPE, FI_ESC_SYSCALL, 0, 222u); return false; }
        VmState *v = vm_of(c, m, slot);
        bool changed = false;
        if (!(flags & 0x10)) {
            int u = 0;
            if (start) {
                u = vm_is_unmapped(c, w, m, slot, start, len);
                if (u < 0) { finish(L, FI_CRASH, FI_CRASH_SE_PANIC, 134, pc32); return false; }
            }
            if (!u) {
                uint64_t s2 = v->mmap_end - len;
                for (;;) {
                    if (s2 > v->mmap_end) { finish(L, FI_ESCAPE, FI_ESC_SYSCALL, 0, 222u); return false; }
                    int hit = -1;
                    for (uint32_t i = 0; i < v->nvma && hit < 0; i++)
                        if (v->vma[i][0] < s2 + len && s2 < v->vma[i][1]) hit = (int)i;
                    if (hit < 0) break;
                    s2 = v->vma[hit][0] - len;   // the page-by-page scan lands right below it
                }
                if (vm_is_unmapped(c, w, m, slot, s2, len) < 0) { finish(L, FI_CRASH, FI_CRASH_SE_PANIC, 134, pc32); return false; }
                v->mmap_end = s2;
                start = s2;
            }
        } else {
            const int r = vm_unmap(c, w, m, slot, v, start, start + len);
            if (r) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, r == 2 ? kEscTable : 0, pc32); return false; }
            changed = true;
        }
        if (!vm_add(v, start, start + len)) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, kEscTable, pc32); return false; }
        set_ret((int64_t)start);
        return changed;
    }
    case 215: {   // munmapFunc (syscall_emul.hh:3140-3156)
        if (a0 & 4095) { set_ret(-22); return false; }
        if (a1 > kVmMaxLen) { finish(L, FI_ESCAPE, FI_ESC_SYSCALL, 0, 215u); return false; }
        const uint64_t len = (a1 + 4095) & ~4095ULL;
        if (a0 + len < a0) { finish(L, FI_ESCAPE, FI_ESC_SYSCALL, 0, 215u); return false; }
        const int r = vm_unmap(c, w, m, slot, vm_of(c, m, slot), a0, a0 + len);
        if (r) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, r == 2 ? kEscTable : 0, pc32); return false; }
        set_ret(0);
        return true;
    }
    case 163: case 261: {   // getrlimitFunc / prlimitFunc (syscall_emul.hh:2197-2264)
        const uint64_t rlp = num == 163 ? a1 : a3;
        if (rlp && !proxy_readable(c, w, m, slot, rlp, 16)) { finish(L, FI_CRASH, FI_CRASH_PROXY, 1, pc32); return false; }
        if (num == 261 && (int)(uint32_t)a0 != 0) { set_ret(-1); return false; }   // -EPERM
        if (num == 261 && !rlp) { set_ret(0); return false; }
        const int64_t res = num == 163 ? (int64_t)(uint32_t)a0 : (int64_t)(int32_t)(uint32_t)a1;
        uint64_t lim;
        if (res == 3) lim = 8ULL << 20;
        else if (res == 2) lim = 256ULL << 20;
        else if (res == 6 && num == 163) lim = 1;   // RLIMIT_NPROC: the system's thread contexts
        else { set_ret(-22); return false; }
        if (!rlp) { finish(L, FI_CRASH, FI_CRASH_SE_PANIC, 134, pc32); return false; }   // null ProxyPtr
        char b[16];
        for (int k = 0; k < 8; k++) b[k] = b[8 + k] = (char)(lim >> (8 * k));
        if (!pwrite(rlp, b, 16)) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, pc32); return false; }
        set_ret(0);
        return rlp < c->code_hi && rlp + 16 > c->code_lo;
    }
    case 278: {   // getrandomFunc (syscall_emul.hh:3222-3236): count bytes of mt19937_64() % 255
        VmState *v = vm_of(c, m, slot);
        if (a1 > (1ULL << 31)) { finish(L, FI_ESCAPE, FI_ESC_HOST, 0, pc32); return false; }
        if (v->rnd_pos + a1 > c->rnd_len) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, kEscTable, pc32); return false; }
        const int h = proxy_writable(c, w, m, slot, a0, a1);
        if (h == 0) { finish(L, FI_CRASH, FI_CRASH_PROXY, 1, pc32); return false; }
        if (h == -1) { finish(L, FI_CRASH, FI_CRASH_STACK_LIMIT, 1, pc32); return false; }
        if (h == -2) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, pc32); return false; }
        if (!pwrite(a0, (const char *)(c->rnd_tab + v->rnd_pos), a1)) {
            finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, pc32);
            return false;
        }
        v->rnd_pos += a1;
        set_ret((int64_t)a1);
        return a0 < c->code_hi && a0 + a1 > c->code_lo;
    }
    case 113: {   // clock_gettimeFunc (syscall_emul.hh:2266-2278): curTick() in ns + 1e9 s
        if (c->clk_esc) { finish(L, FI_ESCAPE, FI_ESC_TIMING, FI_TK_CLOCK, pc32); return false; }
        if (!a1) { finish(L, FI_CRASH, FI_CRASH_SE_PANIC, 134, pc32); return false; }
        if (!proxy_readable(c, w, m, slot, a1, 16)) { finish(L, FI_CRASH, FI_CRASH_PROXY, 1, pc32); return false; }
        const uint64_t ns = (c->tick0 + (L.ncyc - 1) * c->clk_period) / 1000;
        if (c->record) c->stats[52] = L.ninst + 1;   // the golden future reads curTick up to here
        const uint64_t sec = ns / 1000000000ULL + 1000000000ULL, nsec = ns % 1000000000ULL;
        char b[16];
        for (int k = 0; k < 8; k++) { b[k] = (char)(sec >> (8 * k)); b[8 + k] = (char)(nsec >> (8 * k)); }
        if (!pwrite(a1, b, 16)) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, pc32); return false; }
        set_ret(0);
        return a1 < c->code_hi && a1 + 16 > c->code_lo;
    }
    case 160: {   // unameFunc64 (arch/riscv/linux/se_workload.cc:109-122): 5 fields of 65 chars
        if (!a0) { finish(L, FI_CRASH, FI_CRASH_SE_PANIC, 134, pc32); return false; }
        if (!proxy_readable(c, w, m, slot, a0, 325)) { finish(L, FI_CRASH, FI_CRASH_PROXY, 1, pc32); return false; }
        const char *f0 = "Linux", *f1 = "sim.gem5.org", *f2 = "5.1.0", *f3 = "#1 Mon Aug 18 11:32:15 EDT 2003",
                   *f4 = "riscv64";
        const char *f[5] = {f0, f1, f2, f3, f4};
        for (int k = 0; k < 5; k++) {
            uint64_t n = 0;
            while (f[k][n]) n++;
            if (!pwrite(a0 + 65 * k, f[k], n + 1)) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, pc32); return false; }
        }
        set_ret(0);
        return a0 < c->code_hi && a0 + 325 > c->code_lo;
    }
    case 66: {   // writevFunc (syscall_emul.hh:1964-1996)
        const int fd = (int)(uint32_t)a0;
        if (fd < 0 || fd >= 1024) { finish(L, FI_CRASH, FI_CRASH_FD_ASSERT, 134, pc32); return false; }
        if (fd > 2 || ((fdc >> fd) & 1)) { set_ret(-9); return false; }
        if ((fd == 0 && !c->stdin_data) || a2 > (1u << 20)) { finish(L, FI_ESCAPE, FI_ESC_HOST, 0, pc32); return false; }
        uint64_t total = 0;
        for (uint64_t i = 0; i < a2; i++) {
            const uint64_t e = a1 + 16 * i;
            if (e < a1 || !proxy_readable(c, w, m, slot, e, 16)) { finish(L, FI_CRASH, FI_CRASH_PROXY, 1, pc32); return false; }
            const uint64_t base = rd64(e), n = rd64(e + 8);
            if (n > (1ULL << 31)) { finish(L, FI_ESCAPE, FI_ESC_HOST, 0, pc32); return false; }
            if (!proxy_readable(c, w, m, slot, base, n)) { finish(L, FI_CRASH, FI_CRASH_PROXY, 1, pc32); return false; }
            total += n;
        }
        if (fd == 0) { set_ret(-9); return false; }       // the input file (O_RDONLY): EBADF before IOV_MAX
        if (a2 > 1024) { set_ret(-22); return false; }   // host writev: IOV_MAX
        if (total > (1ULL << 31)) { finish(L, FI_ESCAPE, FI_ESC_HOST, 0, pc32); return false; }
        for (uint64_t i = 0; i < a2; i++) {
            const uint64_t e = a1 + 16 * i;
            emit(fd, rd64(e), rd64(e + 8));
        }
        set_ret((int64_t)total);
        return false;
    }
    case 63: {   // readFunc (syscall_emul.hh:2798-2822): (*fds)[fd] asserts the range; no host-backed
                 // entry -> -EBADF; the open stdio entries read the host's files
        const int fd = (int)(uint32_t)a0;
        if (fd < 0 || fd >= 1024) { finish(L, FI_CRASH, FI_CRASH_FD_ASSERT, 134, pc32); return false; }
        if (fd > 2 || ((fdc >> fd) & 1)) { set_ret(-9); return false; }
        if (fd != 0 || !c->stdin_data) { finish(L, FI_ESCAPE, FI_ESC_HOST, 0, pc32); return false; }
        // Process.input is a file (fd_array.cc:69-75): poll() on a regular file
        // is ready; read() takes min(n, left) bytes at the file offset, and the
        // zero-filled BufferArg (syscall_emul_buf.hh:55-85) copies all n bytes
        // out when the read returned any
        if (a2 > (1ULL << 31)) { finish(L, FI_ESCAPE, FI_ESC_HOST, 0, pc32); return false; }
        uint64_t &pos = c->in_pos[slot];
        const uint64_t left = c->stdin_len - pos, k = a2 < left ? a2 : left;
        if (k) {
            const int h = proxy_writable(c, w, m, slot, a1, a2);
            if (h == 0) { finish(L, FI_CRASH, FI_CRASH_PROXY, 1, pc32); return false; }
            if (h == -1) { finish(L, FI_CRASH, FI_CRASH_STACK_LIMIT, 1, pc32); return false; }
            if (h == -2) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, pc32); return false; }
            if (!pwrite(a1, (const char *)(c->stdin_data + pos), k)) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, pc32); return false; }
            const char zero[16] = {};
            for (uint64_t i = k; i < a2; i += 16) {
                if (!pwrite(a1 + i, zero, a2 - i < 16 ? a2 - i : 16)) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, pc32); return false; }
            }
        }
        pos += k;
        set_ret((int64_t)k);
        return k && a1 < c->code_hi && a1 + a2 > c->code_lo;
    }
    case 78: {   // readlinkatFunc (syscall_emul.hh:1066-1129; oracle/rv64se.c sys_readlinkat)
        const int dirfd = (int)(uint32_t)a0;
        const char *want = "/proc/self/exe";
        bool exe = true;
        uint8_t first = 0;
        uint64_t n = 0;
        for (;; n++) {   // the path string through the proxy: -EFAULT at an unmapped byte
            if (n == 4096) { finish(L, FI_ESCAPE, FI_ESC_HOST, 0, pc32); return false; }
            if (a1 + n < a1 || !proxy_readable(c, w, m, slot, a1 + n, 1)) { set_ret(-14); return false; }
            const uint8_t ch = proxy_byte(c, w, m, slot, a1 + n);
            if (c->record) rec_mem(c, a1 + n, 1, L.ninst | kMemEvProxy, 1u);
            if (n == 0) first = ch;
            if (n < 15) exe = exe && ch == (uint8_t)want[n];
            if (!ch) break;
        }
        if (first != '/' && dirfd != -100) {   // atSyscallPath (:356-374)
            if (dirfd < 0 || dirfd >= 1024) { finish(L, FI_CRASH, FI_CRASH_FD_ASSERT, 134, pc32); return false; }
            if (dirfd > 2 || ((fdc >> dirfd) & 1)) { set_ret(-9); return false; }
            finish(L, FI_ESCAPE, FI_ESC_HOST, 0, pc32);
            return false;
        }
        if (!exe || n != 14 || !c->exe_len || a3 > (1ULL << 20)) { finish(L, FI_ESCAPE, FI_ESC_HOST, 0, pc32); return false; }
        const int h = proxy_writable(c, w, m, slot, a2, a3);
        if (h == 0) { finish(L, FI_CRASH, FI_CRASH_PROXY, 1, pc32); return false; }
        if (h == -1) { finish(L, FI_CRASH, FI_CRASH_STACK_LIMIT, 1, pc32); return false; }
        if (h == -2) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, pc32); return false; }
        const uint64_t k = c->exe_len < a3 ? c->exe_len : a3;   // strncpy: the path, then NULs to bufsiz
        if (k && !pwrite(a2, (const char *)c->exe_path, k)) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, pc32); return false; }
        const char zero[16] = {};
        for (uint64_t i = k; i < a3; i += 16) {
            if (!pwrite(a2 + i, zero, a3 - i < 16 ? a3 - i : 16)) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, pc32); return false; }
        }
        set_ret((int64_t)k);
        return a2 < c->code_hi && a2 + a3 > c->code_lo;
    }
    case 258: {   // riscvHWProbeFunc (arch/riscv/linux/se_workload.cc:221-527; oracle/rv64se.c sys_hwprobe)
        const uint64_t pairs = a0, count = a1, cpus_user = a3;
        uint64_t cpusetsize = a2;
        const uint32_t flags = (uint32_t)a4;
        if (count > (1ULL << 16)) { finish(L, FI_ESCAPE, FI_ESC_HOST, 0, pc32); return false; }
        const uint64_t psz = 16 * count;
        auto pw8 = [&](uint64_t a, uint64_t v) {
            char b[8];
            for (int q = 0; q < 8; q++) b[q] = (char)(v >> (8 * q));
            return pwrite(a, b, 8);
        };
        auto copy_out_ok = [&](uint64_t a, uint64_t n) {
            const int h = proxy_writable(c, w, m, slot, a, n);
            if (h == 0) { finish(L, FI_CRASH, FI_CRASH_PROXY, 1, pc32); return false; }
            if (h == -1) { finish(L, FI_CRASH, FI_CRASH_STACK_LIMIT, 1, pc32); return false; }
            if (h == -2) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, pc32); return false; }
            return true;
        };
        auto one = [&](int64_t &key) -> uint64_t {
            switch (key) {
            case 0: case 1: case 2: return 0;
            case 3: return 1;
            case 4: return (1ULL << 0) | (1ULL << 1) | (1ULL << 2) | (0x3FFFULL << 3) | (1ULL << 28) | (1ULL << 29) |
                           (1ULL << 31) | (1ULL << 32) | (1ULL << 33) | (1ULL << 36) | (1ULL << 42) | (1ULL << 45) |
                           (1ULL << 46) | (1ULL << 47);
            case 5: case 9: return 2;
            case 6: return 64;
            case 7: return m.vm ? c->vm[slot].mmap_end : c->vm0 ? c->vm0->mmap_end : 0x4000000000000000ULL;   // MemState::getMmapEnd()
            default: key = -1; return 0;
            }
        };
        if (flags & 1) {   // hwprobe_get_cpus
            if (flags != 1 || cpusetsize == 0 || !cpus_user) { set_ret(-22); return false; }
            if (cpusetsize > 8) cpusetsize = 8;
            const uint64_t usz = cpusetsize;
            if (!proxy_readable(c, w, m, slot, cpus_user, usz)) { finish(L, FI_CRASH, FI_CRASH_PROXY, 1, pc32); return false; }
            uint64_t ub = 0;
            for (uint64_t q = 0; q < usz; q++) ub |= (uint64_t)proxy_byte(c, w, m, slot, cpus_user + q) << (8 * q);
            if (c->record) rec_mem(c, cpus_user, usz, L.ninst | kMemEvProxy, 1u);
            uint64_t cpus = ub ? ub : 1;
            if (!ub) cpusetsize = 8;
            cpus &= 1;
            if (psz && !proxy_readable(c, w, m, slot, pairs, psz)) { finish(L, FI_CRASH, FI_CRASH_PROXY, 1, pc32); return false; }
            if (c->record) rec_mem(c, pairs, psz, L.ninst | kMemEvProxy, 1u);
            int64_t bad = -1;   // the first invalid key's index
            for (uint64_t i = 0; i < count; i++) {
                const int64_t key = (int64_t)rd64(pairs + 16 * i);
                const uint64_t val = rd64(pairs + 16 * i + 8);
                if (key < 0 || key > 9) {
                    if (cpusetsize > usz) { finish(L, FI_ESCAPE, FI_ESC_UNDEF, 0, pc32); return false; }
                    bad = (int64_t)i;
                    ub = 0;
                    break;
                }
                if (cpusetsize > 1) { finish(L, FI_ESCAPE, FI_ESC_UNDEF, 0, pc32); return false; }
                if (cpus & 1) {
                    int64_t k2 = key;
                    const uint64_t v2 = one(k2);
                    const bool bitmask = key == 3 || key == 4 || key == 5;
                    if (!(k2 == key && (bitmask ? (v2 & val) == val : v2 == val))) cpus &= ~1ULL;
                }
            }
            if (!copy_out_ok(pairs, psz)) return false;
            if (bad >= 0 && (!pw8(pairs + 16 * bad, ~0ULL) || !pw8(pairs + 16 * bad + 8, 0))) {
                finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, pc32);
                return false;
            }
            if (!copy_out_ok(cpus_user, usz)) return false;
            char b[8];
            for (int q = 0; q < 8; q++) b[q] = (char)(ub >> (8 * q));
            if (!pwrite(cpus_user, b, usz)) { finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, pc32); return false; }
            set_ret(0);
            return (pairs < c->code_hi && pairs + psz > c->code_lo) || (cpus_user < c->code_hi && cpus_user + usz > c->code_lo);
        }
        if (flags != 0) { set_ret(-22); return false; }   // hwprobe_get_values
        if (cpusetsize > 8) cpusetsize = 8;
        if (!(cpusetsize == 0 && !cpus_user)) {
            if (!proxy_readable(c, w, m, slot, cpus_user, cpusetsize)) { finish(L, FI_CRASH, FI_CRASH_PROXY, 1, pc32); return false; }
            if (c->record) rec_mem(c, cpus_user, cpusetsize, L.ninst | kMemEvProxy, 1u);
            if (cpusetsize < 8 || !(proxy_byte(c, w, m, slot, cpus_user) & 1)) { set_ret(-22); return false; }
        }
        if (psz && !proxy_readable(c, w, m, slot, pairs, psz)) { finish(L, FI_CRASH, FI_CRASH_PROXY, 1, pc32); return false; }
        if (c->record) rec_mem(c, pairs, psz, L.ninst | kMemEvProxy, 1u);
        if (!copy_out_ok(pairs, psz)) return false;
        for (uint64_t i = 0; i < count; i++) {
            int64_t key = (int64_t)rd64(pairs + 16 * i);
            const uint64_t val = one(key);
            if (!pw8(pairs + 16 * i, (uint64_t)key) || !pw8(pairs + 16 * i + 8, val)) {
                finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, pc32);
                return false;
            }
        }
        set_ret(0);
        return pairs < c->code_hi && pairs + psz > c->code_lo;
    }
    default: break;   // 64: write
    }
    // writeFunc (src/sim/syscall_emul.hh:2826-2860): int fd, buffer copied in
    // through a non-allocating proxy (fatal on an unmapped byte), then compared
    // with the golden stream at the current position.
    const int fd = (int)(uint32_t)a0;
    const uint64_t buf = a1, n = a2;
    if (fd < 0 || fd >= 1024) { finish(L, FI_CRASH, FI_CRASH_FD_ASSERT, 134, pc32); return false; }
    if (fd > 2 || ((fdc >> fd) & 1)) { set_ret(-9); return false; }   // no fd entry: -EBADF
    if (fd == 0 && !c->stdin_data) { finish(L, FI_ESCAPE, FI_ESC_HOST, 0, pc32); return false; }
    if (n > (1ULL << 31)) { finish(L, FI_ESCAPE, FI_ESC_HOST, 0, pc32); return false; }
    if (n) {
        if (!proxy_readable(c, w, m, slot, buf, n)) { finish(L, FI_CRASH, FI_CRASH_PROXY, 1, pc32); return false; }
        if (fd == 0) {   // the input file, opened O_RDONLY (fd_array.cc:69-75): host write() -> EBADF
            if (c->record) rec_mem(c, buf, n, L.ninst | kMemEvProxy, 1u);
        } else {
            emit(fd, buf, n);
        }
    }
    if (fd == 0) { set_ret(-9); return false; }
    RREG(10) = n;
    return false;
}

// ------------------------------------------------------------------ snapshots
// Wave-cooperative 4 KiB comparison (all 64 lanes active): each lane compares
// 64 bytes.
template <uint32_t kNL>
__device__ __forceinline__ bool page_eq(const uint8_t *a, const uint8_t *b, uint32_t lane) {
    if (a == b) return true;
    const uint4 *x = (const uint4 *)a, *y = (const uint4 *)b;
    bool eq = true;
#pragma unroll 4
    for (uint32_t k = lane; k < 256; k += kNL) {
        const uint4 u = x[k], v = y[k];
        eq = eq && u.x == v.x && u.y == v.y && u.z == v.z && u.w == v.w;
    }
    return wballot<kNL>(!eq) == 0;
}
// Copy one 4 KiB page, the wave cooperating (the solo kernel's 64 lanes all
// run the one trial: they split the copy by thread index).
template <uint32_t kNL>
__device__ __forceinline__ void page_copy(uint4 *dst, const uint4 *src, uint32_t lane) {
    const uint32_t l0 = kNL == 1 ? (uint32_t)threadIdx.x : lane, step = kNL == 1 ? kSoloLanes : kNL;
#pragma unroll 4
    for (uint32_t k = l0; k < 256; k += step) dst[k] = src[k];
}

// Is lane l's memory equal to the golden memory of snapshot S?  (wave-uniform
// arguments, all lanes active).  The lane's page set is its private pages
// over the start snapshot's table over zero stack pages; the golden one is
// S's table over zero stack pages.  Called only once pc, registers, output
// positions and stack limit already match, so the stack ranges agree.
template <uint32_t kNL>
__device__ bool lane_mem_equal(KCtx *c, const WaveMem &w, uint64_t lslot, uint32_t np, const SnapState *S,
                               uint32_t lane) {
    const PageEnt *tk = c->snap_tab + S->tab_off;
    const uint32_t nk = S->tab_n;
    const uint64_t smin = S->stack_min >> 12;
    for (uint32_t i = 0; i < np; i++) {   // every page the lane has written
        const uint64_t v = uni64(priv_ent(c, lslot, i));
        const int64_t f = tab_find(tk, nk, v);
        const uint8_t *g = f >= 0 ? c->pool + ((uint64_t)f << 12)
                                  : ((v >= smin && v <= kStackTopVpn) ? c->zero_page : nullptr);
        if (!g) return false;
        if (!page_eq<kNL>(priv_frame(c, lslot, i), g, lane)) return false;
    }
    for (uint32_t e = 0; e < nk; e++) {   // golden pages the lane still sees through its start snapshot
        const uint64_t v = uni64(tk[e].vpn);
        const uint32_t f = uni32(tk[e].frame);
        bool priv = false;
        for (uint32_t i = 0; i < np; i++) priv = priv || priv_ent(c, lslot, i) == v;
        if (priv) continue;
        const int64_t fj = tab_find(w.tab, w.tab_n, v);
        const uint8_t *lv = fj >= 0 ? c->pool + ((uint64_t)fj << 12)
                                    : ((v >= smin && v <= kStackTopVpn) ? c->zero_page : nullptr);
        if (!lv) return false;
        if (!page_eq<kNL>(lv, c->pool + ((uint64_t)f << 12), lane)) return false;
    }
    return true;
}

// Guest memory through the global address space (global_load/store, not flat),
// byte-aligned: a misaligned access inside one page is one unaligned memory
// instruction (the HSA runtime runs the GPU in unaligned-access mode; the
// compiler still emits global_load_dword[x2] for these types).
typedef __attribute__((address_space(1))) uint8_t g_u8;
typedef __attribute__((address_space(1), aligned(1))) uint16_t g_u16;
typedef __attribute__((address_space(1), aligned(1))) uint32_t g_u32;
typedef __attribute__((address_space(1), aligned(1))) uint64_t g_u64;
// Translated code: the wave mask of a lane predicate (no int round trip), and
// a value pinned in a VGPR so that `mine ? v : X` stays a select (a select on
// a load's result is otherwise turned into a divergent branch around the load,
// which makes the whole region divergent).
#define TXB(x) (kNL == 1 ? (uint64_t)(bool)(x) : (uint64_t)__builtin_amdgcn_ballot_w64(x))
#define TXSET(r, e)                                         \
    do {                                                    \
        uint64_t t_ = (uint64_t)(e);                        \
        if (kNL > 1) __asm__ volatile("" : "+v"(t_));       \
        X##r = mine ? t_ : X##r;                            \
    } while (0)

// Solo translated code: the trial's guest registers are uniform in a
// one-lane wave and the compiler keeps them in SGPRs.  (Pinning them in VGPRs
// instead -- an asm barrier on every write, conditions and jump targets made
// uniform again -- traded SGPR spills for VALU work and lost: crc32 3.2-3.7M
// against 7.06M trials/s, profiles/r02j_solo_ab.txt.)
#define SCOND(x) (x)
#define SPRIV(x) (x)   // a translated load from the trial's own page (the clean body may hint it)
#define SUNI(x) (x)
#define SUNI32(x) (x)
#define SX(r, e) X##r = (uint64_t)(e)
// the translated bodies' temporaries, at function scope (fi_translate.cpp:
// no block-scope variables in the generated text)
#define TX_TEMPS()                                                                       \
    uint8_t *p_;                                                                         \
    bool pv_, ok_, c_, chg_;                                                             \
    uint64_t v_, ea_, vp_, e_, t_, t0_, tk_, off_;                                       \
    uint32_t cs_, mm_;                                                                   \
    (void)p_; (void)pv_; (void)ok_; (void)c_; (void)chg_; (void)v_; (void)ea_; (void)vp_; \
    (void)e_; (void)t_; (void)t0_; (void)tk_; (void)off_; (void)cs_; (void)mm_
// cycle headers: the pending-route flag as an opaque scalar (fi_translate.cpp)
#define ETGT_OPAQUE() __asm__ volatile("" : "+s"(eon))

// The pre-decoded text (uniform): table, text range, exact code range.
struct TextRef { const PreInst *pre; uint32_t lo, hi, bytes; uint64_t clo, chi; };

// Translated-code memory access: the page must be in the lane's TLB (and be
// its private copy for a store) and the access inside that page (misaligned
// is fine); anything else leaves the translated code before the instruction
// (the interpreter handles misses, copy-on-write, faults and page-crossing).
// Solo translated stores: as tx_probe, but a store into the code range is
// taken too (1 = ok, 3 = ok and it rewrites code: the block marks the bytes
// dirty and leaves if they are still ahead of it; 0 = leave before it).
__device__ __forceinline__ uint32_t tx_probe_st(const LaneMem &m, uint64_t ea, uint32_t size, uint8_t *&p,
                                               const TextRef &t) {
    const uint64_t e = tlb_find(m, ea >> 12);
    p = const_cast<uint8_t *>(page_of(e)) + (ea & 4095);
    const bool ok = (e & 1) != 0 && (uint32_t)(ea & 4095) + size <= 4096u;
    const bool code = !((ea >= t.chi) | (ea + size <= t.clo));
    return ok ? (code ? 3u : 1u) : 0u;
}
typedef __attribute__((address_space(4))) const uint32_t const_u32;

// Solo translated loads: a page the trial has not copied (a shared snapshot
// frame or the zero page -- nothing writes those during a launch) is read
// through the scalar data cache (tx_sload), its own copies with vector loads.
__device__ __forceinline__ bool tx_probe_ld(const LaneMem &m, uint64_t ea, uint32_t size, uint8_t *&p, bool &priv) {
    const uint64_t e = tlb_find(m, ea >> 12);
    p = const_cast<uint8_t *>(page_of(e)) + (ea & 4095);
    priv = (e & 1) != 0;
    return (e != 0) & ((uint32_t)(ea & 4095) + size <= 4096u);
}
// `size` bytes at p (any alignment), zero-extended, by scalar loads of the
// dwords that hold them (may read up to 11 bytes past the access: the shared
// frame pool and the zero page carry 64 bytes of padding, fi_engine.cpp).
__device__ __forceinline__ uint64_t tx_sload(const uint8_t *p, uint32_t size) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    const const_u32 *q = (const const_u32 *)(uintptr_t)(a & ~3ULL);
    const uint32_t sh = (uint32_t)(a & 3) * 8;
    uint64_t v = ((uint64_t)q[1] << 32) | q[0];
    if (size == 8) {
        if (sh) v = (v >> sh) | ((uint64_t)q[2] << (64 - sh));
        return v;
    }
    v >>= sh;
    return v & ((1ULL << (8 * size)) - 1);
}
// The same given the TLB entry e of ea's page (the clean body's site caches).
__device__ __forceinline__ bool tx_probe_e(uint64_t e, uint64_t ea, uint32_t size, uint8_t *&p, bool &priv) {
    p = const_cast<uint8_t *>(page_of(e)) + (ea & 4095);
    priv = (e & 1) != 0;
    return (e != 0) & ((uint32_t)(ea & 4095) + size <= 4096u);
}
__device__ __forceinline__ bool tx_probe_st_e(uint64_t e, uint64_t ea, uint32_t size, uint8_t *&p, const TextRef &t) {
    p = const_cast<uint8_t *>(page_of(e)) + (ea & 4095);
    const bool code_ok = (ea >= t.chi) | (ea + size <= t.clo);
    return ((e & 1) != 0) & code_ok & ((uint32_t)(ea & 4095) + size <= 4096u);
}
__device__ __forceinline__ bool tx_probe(const LaneMem &m, uint64_t ea, uint32_t size, bool st, uint8_t *&p,
                                         const TextRef &t) {
    const uint64_t e = tlb_find(m, ea >> 12);
    p = const_cast<uint8_t *>(page_of(e)) + (ea & 4095);
    // bitwise, not short-circuit: a && here becomes a divergent branch
    const bool code_ok = (ea >= t.chi) | (ea + size <= t.clo);
    return (e != 0) & (!st | (((e & 1) != 0) & code_ok)) & ((uint32_t)(ea & 4095) + size <= 4096u);
}

// ------------------------------------------------------------------ trial kernel
// Diagnostic build only (-DFI_PROF): s_memtime stamps at the phase boundaries
// of the fast loop, summed per wave into stats[24..27] (never in the shipped
// library; a stamp waits for outstanding scalar/LDS loads, so it also shows
// which phase absorbs those waits).
#ifdef FI_PROF
#define PSTAMP(k)                                               \
    do {                                                        \
        const uint64_t _t = __builtin_amdgcn_s_memtime();       \
        pacc[k] += _t - plast;                                  \
        plast = _t;                                             \
    } while (0)
#else
#define PSTAMP(k) do { } while (0)
#endif

struct Pre4 { uint32_t x, y, z, w; };

__device__ __forceinline__ Pre4 pre_load(const PreInst *p) {
    const const_u32 *q = (const const_u32 *)(uintptr_t)p;
    Pre4 r;
    r.x = q[0]; r.y = q[1]; r.z = q[2]; r.w = q[3];
    return r;
}

// Pre-decoded entry of the instruction at pc: one unconditional scalar load,
// and a separate in-text flag, so that a prefetch is not waited for until its
// entry is used.  Odd pcs fetch like pc | 2 of their word:
// key = (pc & ~1) | ((pc & 1) << 1).  The host guarantees that the text does
// not cross a 4 GiB boundary (32-bit compares only: SALU has no 64-bit <).
struct PreRef { Pre4 e; bool in; };
__device__ __forceinline__ PreRef pre_entry(const TextRef &t, uint64_t pc) {
    const uint32_t klo = ((uint32_t)pc & ~1u) | (((uint32_t)pc & 1u) << 1);
    const uint32_t off = klo - t.lo;
    PreRef r;
    r.in = (uint32_t)(pc >> 32) == t.hi && off < t.bytes;
    r.e = pre_load(t.pre + (r.in ? (off >> 1) : 0u));
    return r;
}

// a < b for wave-uniform 64-bit values on the scalar unit (SALU compares are 32-bit)
__device__ __forceinline__ bool ult64(uint64_t a, uint64_t b) {
    const uint32_t ah = (uint32_t)(a >> 32), bh = (uint32_t)(b >> 32);
    return ah < bh || (ah == bh && (uint32_t)a < (uint32_t)b);
}

#ifndef FI_SOLO_VLOAD   // clean solo body: vector loads from shared frames too (0: scalar loads there; profiles/r06 A/B)
#define FI_SOLO_VLOAD 1
#endif
#ifndef FI_SOLO_CPB     // clean solo body: site caches hold frame - page address (0: the TLB entry)
#define FI_SOLO_CPB 1
#endif
typedef __attribute__((address_space(3))) uint64_t lds_u64;
typedef __attribute__((address_space(3))) LaneMem lds_mem;

#ifdef FI_TX
// ---- solo translated blocks, out of line.  Inlined into trial_body<1> they
// shared one register allocation with the whole interpreter: thousands of
// SGPR spills and VGPR scratch spills, some inside the hot blocks.  Here the
// allocator sees only the guest registers, the lane's TLB and the block
// counters.  The caller passes everything through LDS (its register file R,
// its LaneMem and this record); the function reads them back as uniform
// values, runs the blocks from `spc` and writes the registers and the
// counters back.
struct SoloTxIO {
    uint64_t spc;                        // in: entry pc; out: where the blocks left
    uint32_t bud, lwm, sdlo, sdhi;       // in: instruction budget, watched-register mask, rewritten range
    uint32_t st, xt, fb, db;             // out: instructions, straddle ticks, fetch / data bytes
    uint32_t cslo, cshi, schg;           // out: code bytes the blocks rewrote (offsets from text_lo)
    uint32_t hleft, hok, hang;           // in: instructions to the hang cap, proofs allowed; out: a loop that
                                         // cannot leave before the cap (a hang, or a crash on one of its loads)
    uint32_t bst;                        // out: left at a budget test (clean body: the budget may be unspent)
    // out with `hang`: the loop (fi_translate.cpp run-off blocks) -- counter |
    // compared register << 8 | (uint8) step << 16, instructions per iteration,
    // loads (0: a counted loop without memory access, a hang); per load: reg |
    // kind << 8 | size << 12 | position << 16, offset, span (loop_outcome)
    uint32_t lp_cnt, lp_m, lp_n;
    uint32_t lp_ld[4][3];
};
typedef __attribute__((address_space(3))) SoloTxIO lds_io;

template <bool kOdd>
__device__ __noinline__ void solo_tx_run(KCtx *CX, lds_u64 *R, lds_mem *mp, lds_io *io) {
    // the arguments arrive in VGPRs: make the LDS addresses (and so every
    // value read through them) uniform
    CX = (KCtx *)(uintptr_t)uni64((uint64_t)(uintptr_t)CX);
    R = (lds_u64 *)(uintptr_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)R);
    mp = (lds_mem *)(uintptr_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)mp);
    io = (lds_io *)(uintptr_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)io);
    LaneMem m = *mp;   // TLB and rewritten-code state in registers (the blocks never insert into the TLB)
    TextRef tx;
    tx.pre = CX->pre; tx.lo = (uint32_t)CX->text_lo; tx.hi = (uint32_t)(CX->text_lo >> 32);
    tx.bytes = CX->text_bytes; tx.clo = CX->code_lo; tx.chi = CX->code_hi;
    const uint64_t tlo = CX->text_lo;
    uint64_t spc = io->spc;
    const uint32_t bud = io->bud, lwm = io->lwm;
    uint32_t sdlo = io->sdlo, sdhi = io->sdhi;
    uint32_t etgt = 0xFFFFFFFFu;   // block an entry is routed to through its cycle headers
    uint32_t eon = 0;              // ... while an entry is being routed
    bool schg = false;
    uint32_t cslo = 0xFFFFFFFFu, cshi = 0u;
    uint32_t st = 0, xt = 0, fb = 0, db = 0;
#define SADD(n_) (st += (n_))
// a translated store rewrote code bytes [ea_, ea_ + sz_): later blocks see the
// grown range; the decode cache forgets them when the blocks are left
#define TXCODE(ea_, sz_)                                                                        \
    do {                                                                                        \
        const uint32_t o_ = SUNI32((uint32_t)((ea_) - tlo));                                    \
        sdlo = o_ < sdlo ? o_ : sdlo;                                                           \
        sdhi = o_ + (sz_) > sdhi ? o_ + (sz_) : sdhi;                                           \
        cslo = o_ < cslo ? o_ : cslo;                                                           \
        cshi = o_ + (sz_) > cshi ? o_ + (sz_) : cshi;                                           \
        schg = true;                                                                            \
        mark_dirty_solo(CX, m, (ea_), (ea_) + (sz_));                                           \
    } while (0)
// a block's bytes [tlo + lo_, tlo + hi_) hold code the lane rewrote (exact map)
    const __attribute__((address_space(3))) uint32_t *const dl = (const __attribute__((address_space(3))) uint32_t *)m.dl;
    const bool have_dl = m.dl != nullptr;
    const uint32_t dsh = CX->dmap_shift;
#define SDIRTY(lo_, hi_) \
    (((sdlo < (hi_)) & (sdhi > (lo_))) && (!have_dl || dmap_any(dl, tx.clo, tx.chi, dsh, tlo + (lo_), tlo + (hi_))))
#define TXR(r) uint64_t X##r = R[r];
    TXR(1) TXR(2) TXR(3) TXR(4) TXR(5) TXR(6) TXR(7) TXR(8) TXR(9) TXR(10) TXR(11) TXR(12) TXR(13)
    TXR(14) TXR(15) TXR(16) TXR(17) TXR(18) TXR(19) TXR(20) TXR(21) TXR(22) TXR(23) TXR(24) TXR(25)
    TXR(26) TXR(27) TXR(28) TXR(29) TXR(30) TXR(31)
#undef TXR
    TX_TEMPS();
#ifdef FI_TX_SOLO_ODD
    if constexpr (kOdd) {
        goto Q_dispatch;
        /*@TX_SOLO_ODD@*/
    } else
#endif
    {
        goto S_dispatch;
        /*@TX_SOLO@*/
    }
S_out:
#define TXW(r) R[r] = X##r;
    TXW(1) TXW(2) TXW(3) TXW(4) TXW(5) TXW(6) TXW(7) TXW(8) TXW(9) TXW(10) TXW(11) TXW(12) TXW(13)
    TXW(14) TXW(15) TXW(16) TXW(17) TXW(18) TXW(19) TXW(20) TXW(21) TXW(22) TXW(23) TXW(24) TXW(25)
    TXW(26) TXW(27) TXW(28) TXW(29) TXW(30) TXW(31)
#undef TXW
#undef TXCODE
#undef SDIRTY
#undef SADD
    if (schg) {   // mark_dirty_solo changed the bounding range (its LDS map bits are written already)
        mp->code_dirty = true; mp->dlo = m.dlo; mp->dhi = m.dhi;
    }
    io->spc = spc; io->st = st; io->xt = xt; io->fb = fb; io->db = db;
    io->cslo = cslo; io->cshi = cshi; io->schg = schg ? 1u : 0u; io->hang = 0u; io->bst = 0u;
}
#endif

// (loop proofs: unconditional, so the static library's test hook
// fi_debug_loop_outcome runs the same code the translated kernels do)
// A counted loop (fi_translate.cpp) whose counter x steps by c = +-1 and ends
// it at zero passes its branch n more times, x + n c = 0 (mod 2^64; 2^64 for
// x = 0), at least m instructions apart: it commits (n - 1) m of them before
// it can leave -- a hang if that reaches `left`, the instructions to the cap.
// Steps of +-2, 4, 8: a counter whose distance to zero is not a multiple of
// the step never reaches it.
__device__ __forceinline__ uint64_t loop_passes(uint64_t x, int c) {
    const uint64_t d = c < 0 ? x : 0 - x;
    const uint32_t a = (uint32_t)(c < 0 ? -c : c);
    if (d & (a - 1)) return ~0ULL;
    const uint64_t n = d / a;
    return n ? n : ~0ULL;   // (0: 2^64 / a passes)
}
__device__ __forceinline__ bool tx_hang_proof(uint64_t x, int c, uint32_t m, uint32_t left) {
    const uint64_t n = loop_passes(x, c);
    return n - 1 >= ((uint64_t)left + m - 1) / m;
}
// A region loop (fi_translate.cpp region proofs) that runs while x < l
// (unsigned), x growing by c per pass: it passes its exit test at least
// ceil((l - x) / c) more times (x >= l: it may leave at the next test).
__device__ __forceinline__ uint64_t loop_passes_u(uint64_t x, uint64_t l, int c) {
    return x < l ? (l - x - 1) / (uint64_t)c + 1 : 0;
}
__device__ __forceinline__ bool tx_hang_proof_u(uint64_t x, uint64_t l, int c, uint32_t m, uint32_t left) {
    const uint64_t n = loop_passes_u(x, l, c);
    return n != 0 && n - 1 >= ((uint64_t)left + m - 1) / m;
}

// Is vpn in the lane's page set?  (lookup_full without the TLB insert)
__device__ __forceinline__ bool page_mapped(KCtx *c, const WaveMem &w, const LaneMem &m, uint64_t slot, uint64_t vpn) {
    for (uint32_t i = m.n_priv; i-- > 0;) {
        const uint64_t e = priv_ent(c, slot, i);
        if ((e & ~kTomb) == vpn) return !(e & kTomb);
    }
    return tab_find(w.tab, w.tab_n, vpn) >= 0 || (vpn >= (m.stack_min >> 12) && vpn <= kStackTopVpn);
}

// The outcome of a run-off loop that the clean body found unable to leave
// before the hang cap (fi_translate.cpp; the registers are the ones at the
// loop's first instruction, `left` the instructions to the cap).  Iteration i
// runs the block's instruction at position p as the (i m + p)-th from here,
// if i < n (the n-th pass of the branch leaves) and i m + p < left.  Loads and
// stores (kind 2) at the counter plus a constant walk through memory, and so
// do those at another induction register (kinds 3 / 4, with its own step) --
// a store walk that could reach the code range is undecided --; bounded loads
// (a table lookup) stay inside [base + off, base + off + span + size).
//   2: a counter access first touches a page outside the lane's set that
//      MemState::fixupFault would not map (mem_state.cc:387-447) -- the
//      process dies there with GenericPageTableFault (sim/faults.cc:95-105):
//      *k instructions commit first, *fva is the address;
//   1: no load faults before the cap: a hang;
//   0: undecided (a page the fault handler would map, a table page outside
//      the set, a counter load that could straddle a line, many pages, or
//      the loop leaves before the cap): the trial runs on.
template <typename RegP, typename IoP>
__device__ __noinline__ int loop_outcome(KCtx *c, const WaveMem &w, const LaneMem &m, uint64_t slot, RegP R, IoP io,
                                         uint64_t left, uint64_t &k, uint64_t &fva) {
    const uint32_t cnt = io->lp_cnt, mm = io->lp_m, nl = io->lp_n;
    const uint32_t cr = cnt & 0xFF, tr = (cnt >> 8) & 0xFF;
    const int cs = (int)(int8_t)(uint8_t)(cnt >> 16);
    const bool rel = (cnt >> 24) & 1;   // a region loop: runs while x < R[tr] (bounded accesses only)
    if (!mm || nl > 4 || !cr || (rel && (!tr || cs <= 0))) return 0;
    const uint64_t x = R[cr], n = rel ? loop_passes_u(x, R[tr], cs) : loop_passes(x - (tr ? R[tr] : 0ULL), cs);
    if (rel && n == 0) return 0;
    uint64_t best_k = ~0ULL, best_a = 0;
    for (uint32_t j = 0; j < nl; j++) {
        const uint32_t d = io->lp_ld[j][0], br = d & 0xFF, kind = (d >> 8) & 15, size = (d >> 12) & 15, pos = d >> 16;
        const int64_t off = (int64_t)(int32_t)io->lp_ld[j][1];
        if (kind == 1 || kind == 5) {   // bounded (5: a store): every page of its range in the set
            const uint64_t lo = (br ? R[br] : 0ULL) + (uint64_t)off, hi = lo + io->lp_ld[j][2] + size - 1;
            if (hi < lo || (hi >> 12) - (lo >> 12) > 8) return 0;
            for (uint64_t v = lo >> 12; v <= (hi >> 12); v++)
                if (!page_mapped(c, w, m, slot, v)) return 0;
            if (kind == 5 && !(hi < c->code_lo || lo >= c->code_hi)) return 0;   // it could rewrite code
            continue;
        }
        if (rel) return 0;   // (region proofs pass bounded accesses only)
        // kinds 0 / 2 walk with the counter, 3 / 4 with another induction
        // register (its value at the loop's first instruction, its own step)
        const int64_t st = kind >= 3 ? (int64_t)(int32_t)io->lp_ld[j][2] : (int64_t)cs;
        if (kind > 4 || st == 0) return 0;
        const uint64_t a0 = (kind >= 3 ? (br ? R[br] : 0ULL) : x) + (uint64_t)off, ac = (uint64_t)(st < 0 ? -st : st);
        if (size > 1 && ((a0 & (size - 1)) || (ac & (size - 1)))) return 0;   // could straddle a 64-byte line
        if (pos >= left) continue;
        uint64_t ilim = (left - pos + mm - 1) / mm;   // iterations in which it runs
        if (n < ilim) ilim = n;
        if (kind == 2 || kind == 4) {   // a store walk: undecided if it could reach the code range (it would rewrite code)
            const uint64_t span = (ilim - 1) * ac;
            if (ilim > 1 && span / ac != ilim - 1) return 0;
            const uint64_t lo = st > 0 ? a0 : a0 - span, hi = (st > 0 ? a0 + span : a0) + size;
            if ((st > 0 ? hi < a0 : lo > a0) || !(hi <= c->code_lo || lo >= c->code_hi)) return 0;
        }
        uint64_t i = 0;
        for (uint32_t pg = 0; i < ilim; pg++) {
            if (pg > 512) return 0;
            const uint64_t a = a0 + i * (uint64_t)st, vpn = a >> 12;
            if (!page_mapped(c, w, m, slot, vpn)) {
                const uint64_t kj = i * mm + pos;
                if (kj < best_k) { best_k = kj; best_a = a; }
                break;
            }
            if (st > 0) {   // the first iteration past this page
                const uint64_t nx = (vpn + 1) << 12;
                if (!nx) return 0;
                i = (nx - a0 + ac - 1) / ac;
            } else {
                const uint64_t lo = vpn << 12;
                if (!lo) return 0;
                i = (a0 - lo) / ac + 1;
            }
        }
    }
    if (best_k != ~0ULL) {
        const uint64_t f = best_a;
        if (in_vma(c, m, slot, f) || (f >= m.stack_min && f < kStackBase) || (f < m.stack_min && f >= kStackBase - kMaxStack))
            return 0;
        k = best_k; fva = f;
        return 2;
    }
    return n - 1 >= (left + mm - 1) / mm ? 1 : 0;
}

#ifdef FI_TX
// The clean solo body (fi_translate.cpp): for a trial that rewrote no code and
// watches no register, blocks without those checks (a store into the code
// range leaves before itself).  Same calling convention as solo_tx_run.
__device__ __noinline__ void solo_tx_clean_run(KCtx *CX, lds_u64 *R, lds_mem *mp, lds_io *io) {
    CX = (KCtx *)(uintptr_t)uni64((uint64_t)(uintptr_t)CX);
    R = (lds_u64 *)(uintptr_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)R);
    mp = (lds_mem *)(uintptr_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)mp);
    io = (lds_io *)(uintptr_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)io);
    LaneMem m;   // the TLB only (tx_probe)
    m.tv0 = mp->tv0; m.tv1 = mp->tv1; m.tv2 = mp->tv2; m.tv3 = mp->tv3;
    m.tp0 = mp->tp0; m.tp1 = mp->tp1; m.tp2 = mp->tp2; m.tp3 = mp->tp3;
    TextRef tx;
    tx.pre = CX->pre; tx.lo = (uint32_t)CX->text_lo; tx.hi = (uint32_t)(CX->text_lo >> 32);
    tx.bytes = CX->text_bytes; tx.clo = CX->code_lo; tx.chi = CX->code_hi;
    uint64_t spc = io->spc;
    const uint32_t bud = io->bud;
    uint32_t etgt = 0xFFFFFFFFu, eon = 0;
    uint32_t st = 0, xt = 0, fb = 0, db = 0;
    // counted-loop hang proofs (fi_translate.cpp): entering such a cycle with
    // its counter this far from zero, the trial reaches the hang cap inside it
    const uint32_t hleft = io->hleft, hok = io->hok;
    uint32_t hang = 0, bst = 0;
    // instructions: counted down from the budget (brem; the body redefines
    // SADD / SOVER / SDONE, fi_translate.cpp)
    uint32_t brem = bud;
#define SADD(n_) (st += (n_))
#define SOVER(n_) (st + (n_) > bud)
#define SDONE() (st)
#define TXHANG(x_, c_, m_) (hok && tx_hang_proof((x_), (c_), (m_), hleft - SDONE()))
#define TXHANGU(x_, l_, c_, m_) (hok && tx_hang_proof_u((x_), (l_), (c_), (m_), hleft - SDONE()))
#define TXLOOP(c_, m_, n_) (io->lp_cnt = (c_), io->lp_m = (m_), io->lp_n = (n_))
#define TXLD(j_, d_, o_, s_) (io->lp_ld[j_][0] = (d_), io->lp_ld[j_][1] = (uint32_t)(o_), io->lp_ld[j_][2] = (s_))
#define TXR(r) uint64_t X##r = R[r];
    TXR(1) TXR(2) TXR(3) TXR(4) TXR(5) TXR(6) TXR(7) TXR(8) TXR(9) TXR(10) TXR(11) TXR(12) TXR(13)
    TXR(14) TXR(15) TXR(16) TXR(17) TXR(18) TXR(19) TXR(20) TXR(21) TXR(22) TXR(23) TXR(24) TXR(25)
    TXR(26) TXR(27) TXR(28) TXR(29) TXR(30) TXR(31)
#undef TXR
    // the site caches (fi_translate.cpp): the page number CV of the last page a
    // site touched and its TLB entry CP (frame | private bit) -- or, with
    // FI_SOLO_CPB, the frame minus the page's own address (a hit is one add)
    // and the private bit apart in CQ
#if FI_SOLO_CPB
#define SC_SET(i, vp, e) (CV##i = (vp), CP##i = ((e) & ~1ULL) - ((vp) << 12), CQ##i = (uint32_t)(e) & 1u)
#define SC_PTR(i, ea) ((uint8_t *)(uintptr_t)(CP##i + (ea)))
#define SC_PRIV(i) (CQ##i != 0u)
#else
#define SC_SET(i, vp, e) (CV##i = (vp), CP##i = (e))
#define SC_PTR(i, ea) ((uint8_t *)(uintptr_t)((CP##i & ~1ULL) + ((ea) & 4095u)))
#define SC_PRIV(i) ((CP##i & 1u) != 0)
#endif
#if FI_SOLO_VLOAD
    // every translated load through the vector memory path (shared frames are
    // read-only during a launch: either path reads the same bytes)
#undef SPRIV
#define SPRIV(x) ((x) || true)
#endif
    TX_TEMPS();
    goto S_entry;
    /*@TX_SOLO_CLEAN@*/
S_out:
#define TXW(r) R[r] = X##r;
    TXW(1) TXW(2) TXW(3) TXW(4) TXW(5) TXW(6) TXW(7) TXW(8) TXW(9) TXW(10) TXW(11) TXW(12) TXW(13)
    TXW(14) TXW(15) TXW(16) TXW(17) TXW(18) TXW(19) TXW(20) TXW(21) TXW(22) TXW(23) TXW(24) TXW(25)
    TXW(26) TXW(27) TXW(28) TXW(29) TXW(30) TXW(31)
#undef TXW
#undef TXHANG
#undef TXLOOP
#undef TXLD
    io->spc = spc; io->st = SDONE(); io->xt = xt; io->fb = fb; io->db = db;
#undef SADD
#undef SOVER
#undef SDONE
#ifdef SCOLD
#undef SCOLD
#endif
#undef SPRIV
#define SPRIV(x) (x)
    io->cslo = 0xFFFFFFFFu; io->cshi = 0u; io->schg = 0u; io->hang = hang; io->bst = bst;
}
#endif

// ---- dynamic loop proofs (solo kernel).  The static proofs
// (fi_translate.cpp) only see the golden run's translated blocks; the trials
// that end a campaign's tail loop where no translation reaches: in rewritten
// code, in data pages a flipped pc or return address jumped into, or through a
// return into the middle of a block.  A trial that has spent FI_LP_START
// instructions in the interpreters is single-stepped through the general path
// for one pass around its current loop, each committed instruction recorded
// (its operands and kind), and the pass is proved to repeat forever:
//   * every branch / indirect-jump operand, load and store address and
//     store datum is loop-invariant -- a constant, a register the pass never
//     writes, or computed only from invariant values -- so the next pass takes
//     the same path, reads the same addresses and writes the same data;
//   * every store in the pass was silent (wrote the bytes already there), so
//     memory, and with it every load and every fetched instruction, is the
//     same from pass to pass;
//   * no instruction with another effect (syscall, CSR, AMO, LR/SC, M5 op,
//     cache-block or vector op) is in it, and none faulted;
//   * a register the pass writes and is taken as invariant at its start holds
//     the same value at the end of the recorded pass as at its start.
// By induction every later pass equals the recorded one: the trial runs to
// the hang cap (a hang; it can neither end nor meet a golden snapshot, whose
// future terminates).  Registers 0..31 are x0..x31, 32..63 f0..f31.
#ifndef FI_LP_WINDOW
#define FI_LP_WINDOW 128   // instructions per recorded pass at most
#endif
#ifndef FI_LP_START
#define FI_LP_START 4096   // interpreted instructions before the first probe (doubling after a failed one)
#endif
struct LoopProbe {
    uint32_t on;            // recording a pass
    uint32_t n;             // entries recorded
    uint32_t tries;         // windows started in this probe
    uint32_t fp0;           // the FP file existed at the start
    uint32_t cnt, at;       // interpreted instructions since the last probe, the next probe's threshold
    uint64_t pc0;           // where the pass starts (and must return)
    uint64_t r0[32], f0[32];   // registers at the start
    uint32_t e[FI_LP_WINDOW];  // per committed instruction: lp_entry
};
typedef __attribute__((address_space(3))) LoopProbe lds_lp;
constexpr uint32_t kLpNone = 127u;                       // no register in a field
constexpr uint32_t kLpPure = 0, kLpLoad = 1, kLpStore = 2, kLpCtrl = 3, kLpConst = 4;
constexpr uint32_t kLpBad = 0xFFFFFFFFu;                 // an instruction the proof does not admit
constexpr uint32_t kLpLoud = 0xFFFFFFFEu;                // a store that changed memory

// An M5 pseudo-op without an architectural effect beyond a0 = 0, a1 = 0 (the
// general path's `default` case of OP_m5op: not rpns, sum, initparam, a
// debug break or panic, nor one that controls the simulator or host files).
__device__ __forceinline__ bool m5_no_effect(uint32_t fn) {
    switch (fn) {
    case 0x07: case 0x23: case 0x30: case 0x51: case 0x54:
    case 0x01: case 0x02: case 0x03: case 0x04: case 0x21: case 0x22: case 0x4f:
    case 0x53: case 0x5a: case 0x5b: case 0x62: case 0x70: case 0x71:
        return false;
    default: return true;   // (checkpoint 0x43 and switchcpu 0x52 included: they continue)
    }
}

// One committed instruction as {kind, destination, up to three sources}:
// s1 | s2 << 7 | s3 << 14 | dst << 21 | kind << 28 (fields 127: none; x0
// reads are constants and x0 writes vanish).  Integer operands come from the
// decode flags (the same read / write sets the liveness pass uses); FP
// register fields are taken per op (rv_refine_fp_arith / rv_refine_fp_amo).
__device__ __noinline__ uint32_t lp_entry(uint32_t op, uint32_t rd, uint32_t rs1, uint32_t rs2, uint32_t fl,
                                          int32_t imm, bool silent) {
    uint32_t s1 = kLpNone, s2 = kLpNone, s3 = kLpNone, dst = kLpNone, kind = kLpPure;
    if ((fl & kPreRs1) && rs1) s1 = rs1;
    if ((fl & kPreRs2) && rs2) s2 = rs2;
    if ((fl & kPreRd) && rd) dst = rd;
    switch (op) {
    case OP_UNKNOWN: case OP_ESC_FP: case OP_ESC_VEC: case OP_ESC_AMO: case OP_ESC_SYS: case OP_ESC_CRYPTO:
    case OP_ESC_CBO: case OP_ESC_CMP: case OP_ESC_M5: case OP_ESC_HYP: case OP_c_ebreak: case OP_ebreak:
    case OP_ecall: case OP_csr: case OP_lr_w: case OP_sc_w: case OP_lr_d: case OP_sc_d: case OP_priv:
    case OP_cbo:
        return kLpBad;
    case OP_m5op:   // (the commit records a0 = 0 and a1 = 0 for the ones without an effect)
    case OP_vset:
        return kLpBad;
    case OP_vec:    // RVV before any vset*: a no-op of one or two ticks (imm 2, 3), else a fault or escape
        if (imm != 2 && imm != 3) return kLpBad;
        break;
    case OP_c_lw: case OP_c_ld: case OP_c_lbu: case OP_c_lhu: case OP_c_lh: case OP_c_lwsp: case OP_c_ldsp:
    case OP_lb: case OP_lh: case OP_lw: case OP_ld: case OP_lbu: case OP_lhu: case OP_lwu:
        kind = kLpLoad; break;
    case OP_c_sb: case OP_c_sh: case OP_c_sw: case OP_c_sd: case OP_c_swsp: case OP_c_sdsp:
    case OP_sb: case OP_sh: case OP_sw: case OP_sd:
        if (!silent) return kLpLoud;
        kind = kLpStore; break;
    case OP_flh: case OP_flw: case OP_fld: case OP_c_fld: case OP_c_fldsp:
        kind = kLpLoad; dst = 32 + rd; break;
    case OP_fsh: case OP_fsw: case OP_fsd: case OP_c_fsd: case OP_c_fsdsp:
        if (!silent) return kLpLoud;
        kind = kLpStore; s2 = 32 + rs2; break;
    case OP_beq: case OP_bne: case OP_blt: case OP_bge: case OP_bltu: case OP_bgeu: case OP_c_beqz: case OP_c_bnez:
    case OP_jalr: case OP_c_jr: case OP_c_jalr:
        kind = kLpCtrl; break;   // (a link register gets pc + len: a constant)
    case OP_jal: case OP_c_j: case OP_auipc:
        kind = kLpConst; break;
    case OP_fmv_x_w: case OP_fmv_x_d: case OP_fmv_x_h: case OP_fclass_s: case OP_fclass_d: case OP_fclass_h:
    case OP_fcvt_f2i: case OP_fcvtmod:
        s1 = 32 + rs1; break;
    case OP_feq: case OP_flt: case OP_fle:
        s1 = 32 + rs1; s2 = 32 + rs2; break;
    case OP_fmv_w_x: case OP_fmv_d_x: case OP_fmv_h_x: case OP_fcvt_i2f:
        dst = 32 + rd; break;
    case OP_fli:
        kind = kLpConst; dst = 32 + rd; break;
    case OP_fsgnj_s: case OP_fsgnjn_s: case OP_fsgnjx_s: case OP_fsgnj_d: case OP_fsgnjn_d: case OP_fsgnjx_d:
    case OP_fsgnj_h: case OP_fsgnjn_h: case OP_fsgnjx_h: case OP_fadd: case OP_fsub: case OP_fmul: case OP_fdiv:
    case OP_fsqrt: case OP_fmin: case OP_fmax: case OP_fround: case OP_fcvt_f2f:
        s1 = 32 + rs1; s2 = 32 + rs2; dst = 32 + rd; break;   // (one-operand ops: rs2 taken too, conservatively)
    case OP_fmadd: case OP_fmsub: case OP_fnmsub: case OP_fnmadd:
        s1 = 32 + rs1; s2 = 32 + rs2; s3 = 32 + (((uint32_t)imm >> 8) & 31); dst = 32 + rd; break;
    default:   // AMOs are not in any case above: they read and write memory
        if (op >= OP_amoadd_w && op <= OP_amomaxu_d) return kLpBad;
        break;   // integer ALU / M / B / K / Zicond, fences and prefetch hints: pure
    }
    return s1 | s2 << 7 | s3 << 14 | dst << 21 | kind << 28;
}

__device__ __forceinline__ bool lp_src_ok(uint32_t e, uint64_t cur) {
    const uint32_t s1 = e & 127, s2 = (e >> 7) & 127, s3 = (e >> 14) & 127;
    return (s1 == kLpNone || ((cur >> s1) & 1)) && (s2 == kLpNone || ((cur >> s2) & 1)) &&
           (s3 == kLpNone || ((cur >> s3) & 1));
}
// The invariance of the destination after entry e, given the invariant set cur.
__device__ __forceinline__ uint64_t lp_step(uint32_t e, uint64_t cur) {
    const uint32_t dst = (e >> 21) & 127, kind = e >> 28;
    if (dst == kLpNone) return cur;
    const bool inv = kind != kLpPure || lp_src_ok(e, cur);   // loads read unchanged memory at invariant addresses
    return inv ? (cur | (1ULL << dst)) : (cur & ~(1ULL << dst));
}

// The recorded pass repeats forever (the rules above).  xe: the integer
// registers now, at the pass's end; fr: the slot's FP file (stride apart;
// zeros while it does not exist, fp false).
// The whole state again: every register equal at the pass's start and end
// (and the FP file, if any) -- with no store that changed memory in the pass,
// the next pass is the same pass (a loop whose values converge: x = x & y,
// shifts that reach zero, a pointer reset at the top).
__device__ __forceinline__ bool lp_same_state(const lds_lp *P, const uint64_t *xe, const uint64_t *fr, uint64_t stride,
                                              bool fp) {
    if ((P->fp0 != 0) != fp) return false;
    for (uint32_t r = 1; r < 32; r++)
        if (P->r0[r] != xe[r]) return false;
    if (fp)
        for (uint32_t f = 0; f < 32; f++)
            if (P->f0[f] != fr[(uint64_t)f * stride]) return false;
    return true;
}
__device__ __noinline__ bool lp_prove(const lds_lp *P, const uint64_t *xe, const uint64_t *fr, uint64_t stride,
                                      bool fp) {
    const uint32_t n = P->n;
    uint64_t W = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t dst = (P->e[i] >> 21) & 127;
        if (dst != kLpNone) W |= 1ULL << dst;
    }
    W &= ~1ULL;
    // the registers invariant at the pass's start: the least fixpoint from
    // "never written in the pass" (one written from invariant values carries
    // the same value into every later pass)
    uint64_t inv = ~W;
    for (int it = 0; it < 65; it++) {
        uint64_t cur = inv;
        for (uint32_t i = 0; i < n; i++) cur = lp_step(P->e[i], cur);
        const uint64_t nin = ~W | (W & cur);
        if (nin == inv) break;
        inv = nin;
    }
    uint64_t cur = inv;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t e = P->e[i], kind = e >> 28;
        if (kind != kLpPure && kind != kLpConst && !lp_src_ok(e, cur)) return lp_same_state(P, xe, fr, stride, fp);
        cur = lp_step(e, cur);
    }
    const uint64_t chk = W & inv;
    for (uint32_t r = 1; r < 64; r++) {
        if (!((chk >> r) & 1)) continue;
        const uint64_t a = r < 32 ? P->r0[r] : P->f0[r - 32];
        const uint64_t b = r < 32 ? xe[r] : (fp ? fr[(uint64_t)(r - 32) * stride] : 0ULL);
        if (a != b) return lp_same_state(P, xe, fr, stride, fp);
    }
    return true;
}

// The probe's bookkeeping, out of line (the trial loop's registers stay
// free): a failed probe backs off; a window starts from the registers now.
__device__ __noinline__ void lp_fail(lds_lp *P, KCtx *c) {
    P->on = 0; P->cnt = 0;
    P->at = P->at < (1u << 30) ? 2 * P->at : P->at;
    atomicAdd(&c->stats[60], 1ull);
}
__device__ __noinline__ void lp_window(lds_lp *P, KCtx *c, const lds_u64 *R, uint64_t slot, uint64_t pc, bool fp) {
    if (++P->tries > 4) { lp_fail(P, c); return; }
    P->n = 0; P->pc0 = pc; P->fp0 = fp ? 1u : 0u;
    for (int r = 0; r < 32; r++) {
        P->r0[r] = R[r];
        P->f0[r] = fp ? c->fregs[(uint64_t)r * c->n_slots + slot] : 0ULL;
    }
}
// `n` more interpreted instructions; a probe starts once they reach P->at
// (eligible: injected, no watched register, live).
__device__ __noinline__ void lp_count(lds_lp *P, KCtx *c, const lds_u64 *R, uint64_t slot, uint64_t pc, bool fp,
                                      bool eligible, uint32_t n) {
    P->cnt += n;
    if (P->cnt >= P->at && eligible && !c->record && c->hang_proof) {
        P->on = 1; P->tries = 0;
        lp_window(P, c, R, slot, pc, fp);
    }
}
// One committed instruction of a probe's pass (the general path; pc = the
// next one); at the pass's start pc again, the proof.  1 = a proved hang.
__device__ __noinline__ uint32_t lp_commit(lds_lp *P, KCtx *c, const lds_u64 *R, uint64_t slot, uint64_t pc, bool fp,
                                           uint32_t op, uint32_t rd, uint32_t rs1, uint32_t rs2, uint32_t fl, int32_t imm,
                                           bool silent) {
    uint32_t en = lp_entry(op, rd, rs1, rs2, fl, imm, silent);
    if (op == OP_m5op && m5_no_effect((uint32_t)imm) && P->n + 1 < FI_LP_WINDOW) {   // a0 = 0, a1 = 0
        P->e[P->n++] = kLpNone | kLpNone << 7 | kLpNone << 14 | 10u << 21 | kLpConst << 28;
        en = kLpNone | kLpNone << 7 | kLpNone << 14 | 11u << 21 | kLpConst << 28;
    }
    if (en == kLpBad) { lp_fail(P, c); return 0; }
    if (en == kLpLoud || P->n >= FI_LP_WINDOW) {   // memory changed, or the pass is too long: again from here
        lp_window(P, c, R, slot, pc, fp);
        return 0;
    }
    P->e[P->n++] = en;
    if (pc != P->pc0) return 0;
    if (lp_prove(P, (const uint64_t *)R, c->fregs + slot, c->n_slots, fp)) {
        P->on = 0;
        atomicAdd(&c->stats[59], 1ull);
        return 1;
    }
    lp_fail(P, c);
    return 0;
}

// ---- solo pre-decoded run, out of line: the fast path of trial_body<1>
// (one trial, every value uniform) with its own register allocation.  Same
// rules as the 64-lane fast path below: pre-decoded micro-ops from pc until
// the budget is spent, an instruction the path does not own (K_SLOW, a fault,
// a TLB miss lookup_full cannot resolve, copy-on-write, a page-crossing
// access, a watched register read), or (translated build) a block leader the
// translated blocks take over.  Rewritten code is decoded from the lane's own
// bytes through the decode cache (DCT/DCE), and stores into the code range
// mark the bytes rewritten.  Nothing commits unless the whole instruction does.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) Pre4 lds_pre4;
struct SoloPreIO {
    uint64_t spc;          // in: start pc; out: next pc
    uint64_t slot;         // in: the trial's slot
    const PageEnt *tab;    // in: start-snapshot page table
    uint32_t tab_n;
    uint32_t budget;       // in: instructions at most
    uint32_t tx_gate;      // in: leaders stop the run once steps >= tx_gate (translated build)
    int32_t watch;         // in/out: watched flipped register (-1 none)
    uint32_t fps;          // in/out: FP state: the file exists (bit 0) | fflags << 8 | frm << 16
    uint32_t steps, xticks, fbytes, dbytes;   // out
#ifdef FI_PROF
    uint64_t prof[4];      // out: s_memtime cycles per phase (diagnostic build)
#endif
};
typedef __attribute__((address_space(3))) SoloPreIO lds_pio;
constexpr uint32_t kSoloDC = 64;   // decode-cache entries (power of two)

// The F/D/Zfh ops solo_pre_run executes itself (solo_fp_op) instead of
// leaving them to the general path: data movement, sign injection, class,
// and the arithmetic of fp_exec.
__device__ __forceinline__ bool solo_fp_ok(uint32_t op) {
    return (op >= OP_flh && op <= OP_fclass_h) || (op >= OP_fadd && op <= OP_fcvt_f2f) || op == OP_fli ||
           op == OP_fround || op == OP_fcvtmod;
}
// One such op, exactly as the general path executes it (its OP_f* cases and
// the FP-state commit): 0 = not here (a fault, a page to copy, a store into
// the code range, an illegal encoding: the general path takes it, nothing
// done), 1 = committed, 2 = committed with *v for x[rd].  *msz: data bytes.
__device__ __noinline__ uint32_t solo_fp_op(KCtx *c, const WaveMem &w, LaneMem &m, uint64_t slot, const lds_u64 *R,
                                            lds_pio *io, uint32_t q1, uint32_t q2, uint64_t &v, uint32_t &msz) {
    const uint32_t op = q1 & 0xFF, rd = (q1 >> 8) & 0xFF, rs1 = (q1 >> 16) & 0xFF, rs2 = q1 >> 24;
    const int64_t imm = (int32_t)q2;
    uint32_t fps = io->fps;
    const bool fp = fps & 1;
    uint64_t *const F = c->fregs + slot;
    const uint64_t st = c->n_slots;
#define SFR(r) (fp ? F[(uint64_t)(r) * st] : 0ULL)
    uint64_t fval = 0;
    uint32_t fbox = 0, fpst = 0, ret = 1;
    msz = 0;
    switch (op) {
    case OP_flh: case OP_flw: case OP_fld: case OP_c_fld: case OP_c_fldsp: {
        msz = op == OP_flh ? 2 : op == OP_flw ? 4 : 8;
        uint64_t t = 0, fva = 0;
        if (mem_access(c, w, m, slot, R[rs1] + imm, msz, false, t, fva, 0) != F_NONE) return 0;
        fval = msz == 2 ? (0xFFFFFFFFFFFF0000ULL | t) : msz == 4 ? (0xFFFFFFFF00000000ULL | t) : t;
        fbox = 1;
        break;
    }
    case OP_fsh: case OP_fsw: case OP_fsd: case OP_c_fsd: case OP_c_fsdsp: {
        msz = op == OP_fsh ? 2 : op == OP_fsw ? 4 : 8;
        const uint64_t ea = R[rs1] + imm;
        if (ea < c->code_hi && ea + msz > c->code_lo) return 0;   // rewrites code: the general path marks it
        const uint64_t p = lookup(c, w, m, slot, ea >> 12);
        if (!(p & 1) || (ea & 4095) + msz > 4096) return 0;       // a copy-on-write or a page crossing first
        uint64_t t = SFR(rs2), fva = 0;
        if (mem_access(c, w, m, slot, ea, msz, true, t, fva, 0) != F_NONE) return 0;
        break;
    }
    case OP_fmv_x_w: v = sx32(SFR(rs1)); ret = 2; break;
    case OP_fmv_x_d: v = SFR(rs1); ret = 2; break;
    case OP_fmv_x_h: v = (uint64_t)sext64(SFR(rs1) & 0xFFFF, 16); ret = 2; break;
    case OP_fmv_w_x: fval = 0xFFFFFFFF00000000ULL | (R[rs1] & 0xFFFFFFFFULL); fbox = 1; break;
    case OP_fmv_d_x: fval = R[rs1]; fbox = 1; break;
    case OP_fmv_h_x: fval = 0xFFFFFFFFFFFF0000ULL | (R[rs1] & 0xFFFF); fbox = 1; break;
    case OP_fsgnj_s: case OP_fsgnjn_s: case OP_fsgnjx_s: {
        const uint64_t x = fp_unbox32(SFR(rs1)), y = fp_unbox32(SFR(rs2));
        const uint64_t sg = op == OP_fsgnj_s ? y : op == OP_fsgnjn_s ? ~y : (x ^ y);
        fval = 0xFFFFFFFF00000000ULL | (x & 0x7FFFFFFFULL) | (sg & 0x80000000ULL); fbox = 1;
        break;
    }
    case OP_fsgnj_d: case OP_fsgnjn_d: case OP_fsgnjx_d: {
        const uint64_t x = SFR(rs1), y = SFR(rs2);
        const uint64_t sg = op == OP_fsgnj_d ? y : op == OP_fsgnjn_d ? ~y : (x ^ y);
        fval = (x & 0x7FFFFFFFFFFFFFFFULL) | (sg & 0x8000000000000000ULL); fbox = 1;
        break;
    }
    case OP_fsgnj_h: case OP_fsgnjn_h: case OP_fsgnjx_h: {
        const uint64_t x = fp_unbox16(SFR(rs1)), y = fp_unbox16(SFR(rs2));
        const uint64_t sg = op == OP_fsgnj_h ? y : op == OP_fsgnjn_h ? ~y : (x ^ y);
        fval = 0xFFFFFFFFFFFF0000ULL | (x & 0x7FFF) | (sg & 0x8000); fbox = 1;
        break;
    }
    case OP_fclass_s: v = fp_classify(fp_unbox32(SFR(rs1)), 8, 23); ret = 2; break;
    case OP_fclass_d: v = fp_classify(SFR(rs1), 11, 52); ret = 2; break;
    case OP_fclass_h: v = fp_classify(fp_unbox16(SFR(rs1)), 5, 10); ret = 2; break;
    default: {   // fadd .. fcvt_f2f, fli, fround, fcvtmod
        const uint32_t ui = (uint32_t)imm;
        const FpRes fr = fp_exec(op, ui, rs2, SFR(rs1), SFR(rs2), SFR((ui >> 8) & 31), R[rs1], (fps >> 16) & 7);
        if (fr.kind == 2) return 0;   // IllegalInst: the general path's crash
        fpst = 0x100u | fr.fl;
        if (fr.kind == 1) { v = fr.v; ret = 2; }
        else { fval = fr.v; fbox = 1; }
        break;
    }
    }
#undef SFR
    if (fbox || fpst) {   // FP state written: the file exists from its first write on
        if (!fp) {
            for (int r = 0; r < 32; r++) F[(uint64_t)r * st] = 0;
            fps |= 1;
        }
        if (fbox) F[(uint64_t)rd * st] = fval;
        if (fpst & 0x100u) fps |= (fpst & 0x1F) << 8;   // FFLAGS_EXE: accumulate
        io->fps = fps;
    }
    return ret;
}

// ---- the solo interpreter's inner loop in CDNA4 assembly (solo_fast_run).
// The C++ loop of solo_pre_run costs ~140 machine instructions per guest
// instruction (a single wave issues one every 4 cycles: ~400 ns); most of it
// is the guest register file in LDS (address, ds_read, wait, readfirstlane
// per operand, a ds_write per result) and the compiler's compare tree on the
// micro-op kind.  Here the 31 guest registers live in lanes of two VGPRs
// (x_r = lane r of v28 lo / v29 hi; lane 32 absorbs the writes to x0), read
// with v_readlane and written with v_writelane (lane select in M0), and
// everything else is SALU -- two VGPRs instead of 64, so the call saves no
// callee-saved VGPRs (round 4 kept them in v64..v127 under VGPR index mode:
// 32 of those are callee-saved, spilled to scratch and back on every call):
// ~40 instructions for an ALU op, the kind dispatched through a jump table;
// the entries of the pcs it runs are kept in a 64-entry cache in VGPR lanes
// (v24..v27, lane (po >> 1) & 63, read with v_readlane), so a loop reads no
// LDS (rewritten code) after its first iteration.
// It runs every micro-op but K_SLOW -- add / sub / and / or / xor / slt(u) /
// shifts / mul / mulh(s)(u) / div(u) / rem(u) (also the W forms), in-page
// loads and stores through a two-entry page cache in front of the
// lane's TLB, the six branches, jal, jalr -- with the exact rules of
// solo_pre_run, and leaves to the C++ loop, before the instruction, at
// anything else (reason 1): K_SLOW, a decode-cache miss in the rewritten window, a page the TLB
// does not hold, a page crossing (misaligned accesses inside a page go byte by
// byte, as in solo_pre_run), the first store that
// changes bytes of the code range (later ones: the rewrite is marked here as
// in solo_pre_run -- bounding range, LDS map, decode and entry caches) or a
// store to a page the lane has not copied.  Outcomes are those of the C++
// loop bit for bit (every parity test runs through it).
struct alignas(16) SoloFastIO {
    uint32_t po, steps, budget, xticks;     // 0   in/out (budget in)
    uint32_t fbytes, dbytes, tby, ddlo;     // 16  counters in/out; text bytes; rewritten window lo
    uint32_t ddhi3, clo_o, csz, gate;       // 32  window hi + 3; code range (text offset, size); leader gate
    uint32_t lbe, lbo, reason, r_lds;       // 48  leader flag bits (even / odd pc); out: why it left; LDS of R
    uint32_t dct_lds, dce_lds, tlb_lds, lc_lds;// 64  LDS of the decode cache tags / entries, of LaneMem::tv0, of the entry cache
    uint64_t pre, tlo;                      // 80  pre-decoded text, text base
    uint64_t clo, cvpn;                     // 96  code range base; page cache (in/out)
    uint64_t cpg, npc;                      // 112 its page; out: the pc that left the text (reason 3)
    uint32_t dl_lds, dsh, pad0, pad1;       // 128 LDS of the rewritten-code map (0: none), its granule shift
};
static_assert(sizeof(SoloFastIO) == 144, "SoloFastIO layout");
// a store that rewrites code updates LaneMem::dlo / dhi in place (LDS, from &tv0)
static_assert(__builtin_offsetof(LaneMem, dlo) == __builtin_offsetof(LaneMem, tv0) + 96 &&
              __builtin_offsetof(LaneMem, dhi) == __builtin_offsetof(LaneMem, tv0) + 104, "LaneMem dlo / dhi");
typedef __attribute__((address_space(3))) SoloFastIO lds_fio;
// reasons: 0 budget spent, 1 the instruction at po is the C++ loop's, 2 a
// block leader stops the run, 3 a jump left the text (npc), 4 the fall-through
// left the text (po >= tby)
__device__ __noinline__ void solo_fast_run(lds_fio *io) {
    const uint32_t a = (uint32_t)(uintptr_t)io;
    asm volatile(
        // ---- state in: the io record (LDS) into SGPRs, R into lanes of v28 / v29
        "s_mov_b32 s4, m0\n"
        "v_mov_b32 v31, %[io]\n"
        "ds_read2_b64 v[0:3], v31 offset0:0 offset1:1\n"
        "ds_read2_b64 v[4:7], v31 offset0:2 offset1:3\n"
        "ds_read2_b64 v[8:11], v31 offset0:4 offset1:5\n"
        "ds_read2_b64 v[12:15], v31 offset0:6 offset1:7\n"
        "ds_read2_b64 v[16:19], v31 offset0:8 offset1:9\n"
        "ds_read2_b64 v[20:23], v31 offset0:10 offset1:11\n"
        "ds_read2_b64 v[24:27], v31 offset0:12 offset1:13\n"
        "ds_read_b64 v[28:29], v31 offset:112\n"
        "s_waitcnt lgkmcnt(0)\n"
        "v_readfirstlane_b32 s5, v0\n"      // po
        "v_readfirstlane_b32 s6, v1\n"      // steps
        "v_readfirstlane_b32 s7, v2\n"      // budget
        "v_readfirstlane_b32 s8, v3\n"      // xticks
        "v_readfirstlane_b32 s9, v4\n"      // fbytes
        "v_readfirstlane_b32 s10, v5\n"     // dbytes
        "v_readfirstlane_b32 s11, v6\n"     // tby
        "v_readfirstlane_b32 s12, v7\n"     // ddlo
        "v_readfirstlane_b32 s13, v8\n"     // ddhi + 3
        "v_readfirstlane_b32 s14, v9\n"     // clo_o
        "v_readfirstlane_b32 s15, v10\n"    // csz
        "v_readfirstlane_b32 s16, v11\n"    // gate
        "v_readfirstlane_b32 s17, v12\n"    // lbe
        "v_readfirstlane_b32 s18, v13\n"    // lbo
        "v_readfirstlane_b32 s20, v20\n"    // pre
        "v_readfirstlane_b32 s21, v21\n"
        "v_readfirstlane_b32 s22, v22\n"    // tlo
        "v_readfirstlane_b32 s23, v23\n"
        "v_readfirstlane_b32 s24, v24\n"    // clo
        "v_readfirstlane_b32 s25, v25\n"
        "v_readfirstlane_b32 s26, v26\n"    // cvpn (slot 0)
        "v_readfirstlane_b32 s27, v27\n"
        "v_readfirstlane_b32 s28, v28\n"    // cpg
        "v_readfirstlane_b32 s29, v29\n"
        // v15 = R, v16 = DCT, v17 = DCE, v18 = &tv0 (LDS addresses; v12..v14 free again)
        "s_or_b32 s79, s17, s18\n"          // leader flag bits of either parity, in place in w
        "s_lshl_b32 s79, s79, 8\n"
        "s_getpc_b64 s[80:81]\n"            // the jump table's address
        "L_gp%=:\n"
        "s_add_u32 s80, s80, L_jt%= - L_gp%=\n"
        "s_addc_u32 s81, s81, 0\n"
        "s_mov_b64 s[70:71], -1\n"          // page cache slot 1: empty
        "s_mov_b64 s[72:73], 0\n"
        // the entry cache in VGPR lanes: v24 tag (po) / v25..v27 entry words
        // y z w, lane (po >> 1) & 63; kept in LDS between calls (lc_lds: one
        // 16-byte record per lane, invalidated there by every code-changing
        // store), so a loop that hands back stays warm
        "v_readfirstlane_b32 s62, v19\n"
        "s_mov_b64 s[74:75], exec\n"
        "s_mov_b64 exec, -1\n"
        "v_mbcnt_lo_u32_b32 v30, -1, 0\n"
        "v_mbcnt_hi_u32_b32 v30, -1, v30\n"
        "v_lshl_add_u32 v30, v30, 4, s62\n"
        "ds_read_b128 v[24:27], v30\n"
        "s_mov_b64 exec, s[74:75]\n"
        // the guest registers: x_r in lane r of v28 (low word) / v29 (high
        // word), lanes 0..31 (lane 32 takes the writes to x0)
        "v_readfirstlane_b32 s62, v15\n"
        "s_mov_b64 s[74:75], exec\n"
        "s_mov_b32 exec_lo, -1\n"
        "s_mov_b32 exec_hi, 0\n"
        "v_mbcnt_lo_u32_b32 v2, -1, 0\n"
        "v_lshl_add_u32 v2, v2, 3, s62\n"
        "ds_read_b64 v[28:29], v2\n"
        "s_mov_b64 exec, s[74:75]\n"
        "s_waitcnt lgkmcnt(0)\n"
        // ================================================================ loop
        "L_top%=:\n"
        "s_cmp_ge_u32 s6, s7\n"
        "s_cbranch_scc1 L_budget%=\n"
        // ---- the entry: the VGPR-lane entry cache (a loop runs from it with
        // no memory wait), else (L_lmiss, out of line) the decode cache inside
        // the rewritten window or pre[], then filled into the lane cache
        "s_bfe_u32 s82, s5, 0x60001\n"
        "v_readlane_b32 s63, v24, s82\n"
        "s_cmp_eq_u32 s63, s5\n"
        "s_cbranch_scc0 L_lmiss%=\n"
        "v_readlane_b32 s37, v25, s82\n"
        "v_readlane_b32 s38, v26, s82\n"
        "v_readlane_b32 s39, v27, s82\n"
        "L_have%=:\n"
        // (K_SLOW leaves through the jump table)
        "s_bfe_u32 s56, s39, 0x60010\n"     // kind
        "s_and_b32 s62, s39, s79\n"         // maybe a block leader the translated code takes
        "s_cbranch_scc1 L_lead%=\n"         // (out of line)
        "L_nolead%=:\n"
        "s_and_b32 s60, s39, 0xff\n"        // len
        "s_bfe_u32 s57, s37, 0x50008\n"     // rd
        "s_bfe_u32 s58, s37, 0x50010\n"     // rs1
        "s_bfe_u32 s59, s37, 0x50018\n"     // rs2
        // a = x[rs1] (av but for U_APC), b = x[rs2]: lane rs of v28 / v29
        "v_readlane_b32 s44, v28, s58\n"
        "v_readlane_b32 s45, v29, s58\n"
        "v_readlane_b32 s42, v28, s59\n"
        "v_readlane_b32 s43, v29, s59\n"
        "s_ashr_i32 s53, s38, 31\n"         // imm, sign-extended
        "s_mov_b32 s52, s38\n"
        "s_bitcmp1_b32 s39, 25\n"           // U_APC (aux = w >> 16): av = pc (out of line)
        "s_cbranch_scc1 L_apc%=\n"
        "L_apcb%=:\n"
        "s_bitcmp1_b32 s39, 24\n"           // U_BIMM
        "s_cselect_b64 s[46:47], s[52:53], s[42:43]\n"
        // ---- dispatch on the kind (rv64_isa.h Kind): add inline (the most
        // frequent kind; it falls through into the write-back), the rest
        // through a jump table of s_branch instructions, one per kind, at
        // s[80:81] (L_disp, out of line)
        "s_cmp_lg_u32 s56, 1\n"
        "s_cbranch_scc1 L_disp%=\n"
        "L_add%=:\n"
        "s_add_u32 s48, s44, s46\n"
        "s_addc_u32 s49, s45, s47\n"
        // ---- write back x[rd] (w32: sign-extended low word), then fall through
        "L_wb%=:\n"
        "s_bitcmp1_b32 s39, 26\n"           // U_W32: sign-extend the low word (out of line)
        "s_cbranch_scc1 L_wbw%=\n"
        "L_wb64%=:\n"
        "s_cmp_eq_u32 s57, 0\n"             // x0 stays zero: its writes go to lane 32
        "s_cselect_b32 m0, 32, s57\n"
        "v_writelane_b32 v28, s48, m0\n"
        "v_writelane_b32 v29, s49, m0\n"
        "L_nowb%=:\n"
        "s_add_u32 s6, s6, 1\n"             // commit (data bytes: in the memory paths)
        "s_bfe_u32 s62, s39, 0x10009\n"     // straddle tick (kPreStraddle)
        "s_add_u32 s8, s8, s62\n"
        "s_add_u32 s9, s9, s60\n"
        "s_add_u32 s5, s5, s60\n"           // the fall-through
        "s_cmp_lt_u32 s5, s11\n"
        "s_cbranch_scc1 L_top%=\n"
        "s_mov_b32 s19, 4\n"
        "s_branch L_out%=\n"
        // ---- out of line: the entry fetch, the rewritten window, a leader,
        // the jump table
        "L_lmiss%=:\n"
        "s_add_u32 s62, s5, 6\n"
        "s_cmp_gt_u32 s62, s12\n"
        "s_cbranch_scc1 L_win%=\n"
        "L_pre%=:\n"                        // entry (po >> 1) | (po & 1), 16 bytes each
        "s_bitcmp1_b32 s5, 0\n"
        "s_cbranch_scc1 L_preo%=\n"         // (odd pc: out of line)
        "s_lshl_b32 s62, s5, 3\n"
        "L_prel%=:\n"
        "s_load_dwordx4 s[36:39], s[20:21], s62\n"
        "s_waitcnt lgkmcnt(0)\n"
        "L_fill%=:\n"                       // (lane select in M0: one SGPR operand per VALU op)
        "s_mov_b32 m0, s82\n"
        "v_writelane_b32 v24, s5, m0\n"
        "v_writelane_b32 v25, s37, m0\n"
        "v_writelane_b32 v26, s38, m0\n"
        "v_writelane_b32 v27, s39, m0\n"
        "s_branch L_have%=\n"
        "L_win%=:\n"
        "s_cmp_lt_u32 s5, s13\n"
        "s_cbranch_scc0 L_pre%=\n"
        "s_sub_u32 s62, s5, s14\n"          // in the code range?
        "s_cmp_lt_u32 s62, s15\n"
        "s_cbranch_scc0 L_slow%=\n"
        "s_bfe_u32 s62, s5, 0x60001\n"      // ci = (po >> 1) & 63
        "v_lshl_add_u32 v0, s62, 2, v16\n"
        "v_lshl_add_u32 v1, s62, 4, v17\n"
        "ds_read_b32 v2, v0\n"
        "ds_read2_b64 v[4:7], v1 offset0:0 offset1:1\n"
        "s_waitcnt lgkmcnt(0)\n"
        "v_readfirstlane_b32 s62, v2\n"     // tag
        "v_readfirstlane_b32 s37, v5\n"
        "v_readfirstlane_b32 s38, v6\n"
        "v_readfirstlane_b32 s39, v7\n"
        "s_cmp_eq_u32 s62, s5\n"
        "s_cbranch_scc0 L_slow%=\n"         // a miss: the C++ loop decodes and fills the cache
        "s_branch L_fill%=\n"
        "L_lead%=:\n"                       // a block leader the translated code takes?
        "s_bitcmp1_b32 s5, 0\n"
        "s_cselect_b32 s62, s18, s17\n"
        "s_bfe_u32 s63, s39, 0x80008\n"
        "s_and_b32 s62, s62, s63\n"
        "s_cbranch_scc0 L_nolead%=\n"
        "s_cmp_ge_u32 s6, s16\n"
        "s_cbranch_scc1 L_leader%=\n"
        "s_branch L_nolead%=\n"
        "L_preo%=:\n"
        "s_lshr_b32 s62, s5, 1\n"
        "s_or_b32 s62, s62, 1\n"
        "s_lshl_b32 s62, s62, 4\n"
        "s_branch L_prel%=\n"
        "L_wbw%=:\n"
        "s_ashr_i32 s49, s48, 31\n"
        "s_branch L_wb64%=\n"
        "L_apc%=:\n"                        // av = pc
        "s_add_u32 s44, s22, s5\n"
        "s_addc_u32 s45, s23, 0\n"
        "s_branch L_apcb%=\n"
        "L_disp%=:\n"
        "s_cmp_gt_u32 s56, 29\n"
        "s_cbranch_scc1 L_slow%=\n"
        "s_lshl_b32 s62, s56, 2\n"
        "s_add_u32 s64, s80, s62\n"
        "s_addc_u32 s65, s81, 0\n"
        "s_setpc_b64 s[64:65]\n"
        "L_jt%=:\n"
        "s_branch L_slow%=\n"               // 0 K_SLOW
        "s_branch L_add%=\n"                // 1 K_ADD
        "s_branch L_sub%=\n"
        "s_branch L_and%=\n"
        "s_branch L_or%=\n"
        "s_branch L_xor%=\n"
        "s_branch L_slt%=\n"
        "s_branch L_sltu%=\n"
        "s_branch L_sll%=\n"
        "s_branch L_srl%=\n"
        "s_branch L_sra%=\n"
        "s_branch L_mul%=\n"                // 11 K_MUL
        "s_branch L_mem%=\n"                // 12 K_LOAD
        "s_branch L_mem%=\n"                // 13 K_STORE
        "s_branch L_beq%=\n"                // 14 K_BEQ
        "s_branch L_bne%=\n"
        "s_branch L_blt%=\n"
        "s_branch L_bge%=\n"
        "s_branch L_bltu%=\n"
        "s_branch L_bgeu%=\n"               // 19 K_BGEU
        "s_branch L_jal%=\n"                // 20 K_JAL
        "s_branch L_jalr%=\n"               // 21 K_JALR
        "s_branch L_nowb%=\n"               // 22 K_NOP
        "s_branch L_mulh%=\n"               // 23 K_MULH
        "s_branch L_mulhu%=\n"
        "s_branch L_mulhsu%=\n"
        "s_branch L_div%=\n"                // 26 K_DIV
        "s_branch L_divu%=\n"
        "s_branch L_rem%=\n"
        "s_branch L_remu%=\n"               // 29 K_REMU
        // ---- ALU
        "L_sub%=:\n"
        "s_sub_u32 s48, s44, s46\n"
        "s_subb_u32 s49, s45, s47\n"
        "s_branch L_wb%=\n"
        "L_and%=:\n"
        "s_and_b64 s[48:49], s[44:45], s[46:47]\n"
        "s_branch L_wb%=\n"
        "L_or%=:\n"
        "s_or_b64 s[48:49], s[44:45], s[46:47]\n"
        "s_branch L_wb%=\n"
        "L_xor%=:\n"
        "s_xor_b64 s[48:49], s[44:45], s[46:47]\n"
        "s_branch L_wb%=\n"
        "L_slt%=:\n"                        // signed av < bv
        "s_mov_b64 s[48:49], 0\n"
        "s_cmp_lt_i32 s45, s47\n"
        "s_cbranch_scc1 L_one%=\n"
        "s_cmp_lg_u32 s45, s47\n"
        "s_cbranch_scc1 L_wb%=\n"
        "s_cmp_lt_u32 s44, s46\n"
        "s_cbranch_scc0 L_wb%=\n"
        "L_one%=:\n"
        "s_mov_b32 s48, 1\n"
        "s_branch L_wb%=\n"
        "L_sltu%=:\n"                       // unsigned av < bv
        "s_mov_b64 s[48:49], 0\n"
        "s_cmp_lt_u32 s45, s47\n"
        "s_cbranch_scc1 L_one%=\n"
        "s_cmp_lg_u32 s45, s47\n"
        "s_cbranch_scc1 L_wb%=\n"
        "s_cmp_lt_u32 s44, s46\n"
        "s_cbranch_scc1 L_one%=\n"
        "s_branch L_wb%=\n"
        "L_sll%=:\n"                        // av << (bv & shm)
        "s_bitcmp1_b32 s39, 26\n"           // U_W32: 5-bit amount
        "s_cselect_b32 s62, 31, 63\n"
        "s_and_b32 s62, s46, s62\n"
        "s_lshl_b64 s[48:49], s[44:45], s62\n"
        "s_branch L_wb%=\n"
        "L_srl%=:\n"                        // (w32 ? av & 0xffffffff : av) >> (bv & shm)
        "s_mov_b32 s64, s44\n"
        "s_bitcmp1_b32 s39, 26\n"
        "s_cselect_b32 s62, 31, 63\n"
        "s_cselect_b32 s65, 0, s45\n"
        "s_and_b32 s62, s46, s62\n"
        "s_lshr_b64 s[48:49], s[64:65], s62\n"
        "s_branch L_wb%=\n"
        "L_sra%=:\n"                        // (w32 ? (int32)av : (int64)av) >> (bv & shm)
        "s_mov_b32 s64, s44\n"
        "s_ashr_i32 s66, s44, 31\n"
        "s_bitcmp1_b32 s39, 26\n"
        "s_cselect_b32 s62, 31, 63\n"
        "s_cselect_b32 s65, s66, s45\n"
        "s_and_b32 s62, s46, s62\n"
        "s_ashr_i64 s[48:49], s[64:65], s62\n"
        "s_branch L_wb%=\n"
        "L_mul%=:\n"                        // low 64 bits of av * bv
        "s_mul_i32 s48, s44, s46\n"
        "s_mul_hi_u32 s62, s44, s46\n"
        "s_mul_i32 s64, s44, s47\n"
        "s_mul_i32 s65, s45, s46\n"
        "s_add_u32 s62, s62, s64\n"
        "s_add_u32 s49, s62, s65\n"
        "s_branch L_wb%=\n"
        // ---- M extension.  mulh*: the high word of the 128-bit product from
        // 32-bit partial products, then the signed corrections (a < 0: - b,
        // b < 0: - a).  div* / rem*: RISC-V rules (x / 0 = ~0, x % 0 = x,
        // overflow through the unsigned magnitudes); W forms on the sign- or
        // zero-extended low words (L_wb sign-extends the result).  The
        // unsigned core is the compiler's expansion of a uniform u64 divide
        // (reciprocal estimate + two refinements + two corrections), with a
        // 32-bit short path.
        "L_mulhu%=:\n"
        "s_mov_b32 s36, 0\n"
        "s_branch L_mh%=\n"
        "L_mulh%=:\n"
        "s_mov_b32 s36, 3\n"
        "s_branch L_mh%=\n"
        "L_mulhsu%=:\n"
        "s_mov_b32 s36, 1\n"
        "L_mh%=:\n"
        "s_mul_hi_u32 s62, s44, s46\n"     // hi(a0 b0)
        "s_mul_i32 s64, s44, s47\n"        // a0 b1
        "s_mul_hi_u32 s65, s44, s47\n"
        "s_mul_i32 s66, s45, s46\n"        // a1 b0
        "s_mul_hi_u32 s67, s45, s46\n"
        "s_mul_i32 s68, s45, s47\n"        // a1 b1
        "s_mul_hi_u32 s69, s45, s47\n"
        "s_add_u32 s62, s62, s64\n"        // carries out of bits 32..63
        "s_addc_u32 s65, s65, 0\n"
        "s_add_u32 s62, s62, s66\n"
        "s_addc_u32 s67, s67, 0\n"
        "s_add_u32 s48, s68, s65\n"
        "s_addc_u32 s49, s69, 0\n"
        "s_add_u32 s48, s48, s67\n"
        "s_addc_u32 s49, s49, 0\n"
        "s_bitcmp1_b32 s36, 0\n"           // signed a (mulh, mulhsu): a < 0 -> - b
        "s_cbranch_scc0 L_wb%=\n"
        "s_cmp_lt_i32 s45, 0\n"
        "s_cselect_b64 s[64:65], s[46:47], 0\n"
        "s_sub_u32 s48, s48, s64\n"
        "s_subb_u32 s49, s49, s65\n"
        "s_bitcmp1_b32 s36, 1\n"           // signed b (mulh): b < 0 -> - a
        "s_cbranch_scc0 L_wb%=\n"
        "s_cmp_lt_i32 s47, 0\n"
        "s_cselect_b64 s[64:65], s[44:45], 0\n"
        "s_sub_u32 s48, s48, s64\n"
        "s_subb_u32 s49, s49, s65\n"
        "s_branch L_wb%=\n"
        // s36: bit 0 remainder, bit 1 signed
        "L_divu%=:\n"
        "s_mov_b32 s36, 0\n"
        "s_branch L_dv%=\n"
        "L_div%=:\n"
        "s_mov_b32 s36, 2\n"
        "s_branch L_dv%=\n"
        "L_rem%=:\n"
        "s_mov_b32 s36, 3\n"
        "s_branch L_dv%=\n"
        "L_remu%=:\n"
        "s_mov_b32 s36, 1\n"
        "L_dv%=:\n"
        "s_mov_b64 s[64:65], s[44:45]\n"   // N, D
        "s_mov_b64 s[66:67], s[46:47]\n"
        "s_bitcmp1_b32 s39, 26\n"          // U_W32: the low words, sign- or zero-extended
        "s_cbranch_scc0 L_dv64%=\n"
        "s_ashr_i32 s65, s64, 31\n"
        "s_ashr_i32 s67, s66, 31\n"
        "s_bitcmp1_b32 s36, 1\n"
        "s_cbranch_scc1 L_dv64%=\n"
        "s_mov_b32 s65, 0\n"
        "s_mov_b32 s67, 0\n"
        "L_dv64%=:\n"
        "s_cmp_lg_u64 s[66:67], 0\n"
        "s_cbranch_scc1 L_dvnz%=\n"
        "s_mov_b64 s[68:69], -1\n"         // x / 0 = ~0, x % 0 = x
        "s_mov_b64 s[74:75], s[64:65]\n"
        "s_branch L_dvsel%=\n"
        "L_dvnz%=:\n"
        "s_mov_b32 s52, 0\n"               // negate the quotient / the remainder
        "s_mov_b32 s53, 0\n"
        "s_bitcmp1_b32 s36, 1\n"
        "s_cbranch_scc0 L_dvu%=\n"
        "s_cmp_lt_i32 s65, 0\n"
        "s_cbranch_scc0 L_dvpa%=\n"
        "s_sub_u32 s64, 0, s64\n"
        "s_subb_u32 s65, 0, s65\n"
        "s_mov_b32 s53, 1\n"
        "s_mov_b32 s52, 1\n"
        "L_dvpa%=:\n"
        "s_cmp_lt_i32 s67, 0\n"
        "s_cbranch_scc0 L_dvu%=\n"
        "s_sub_u32 s66, 0, s66\n"
        "s_subb_u32 s67, 0, s67\n"
        "s_xor_b32 s52, s52, 1\n"
        "L_dvu%=:\n"
        "s_mov_b64 s[44:45], s[64:65]\n"   // |N|, |D| (the core consumes its inputs)
        "s_mov_b64 s[46:47], s[66:67]\n"
        "s_or_b32 s62, s65, s67\n"
        "s_cmp_lg_u32 s62, 0\n"
        "s_cbranch_scc0 L_dv32%=\n"
        "v_cvt_f32_u32 v0, s66\n"
        "v_cvt_f32_u32 v1, s67\n"
        "s_sub_u32 s74, 0, s66\n"
        "s_subb_u32 s75, 0, s67\n"
        "v_fmamk_f32 v0, v1, 0x4f800000, v0\n"
        "v_rcp_f32 v0, v0\n"
        "s_nop 0\n"
        "v_mul_f32 v0, 0x5f7ffffc, v0\n"
        "v_mul_f32 v1, 0x2f800000, v0\n"
        "v_trunc_f32 v1, v1\n"
        "v_fmamk_f32 v0, v1, 0xcf800000, v0\n"
        "v_cvt_u32_f32 v1, v1\n"
        "v_cvt_u32_f32 v0, v0\n"
        "v_readfirstlane_b32 s76, v1\n"
        "v_readfirstlane_b32 s68, v0\n"
        "s_mul_i32 s69, s74, s76\n"
        "s_mul_hi_u32 s78, s74, s68\n"
        "s_mul_i32 s77, s75, s68\n"
        "s_add_i32 s69, s78, s69\n"
        "s_add_i32 s69, s69, s77\n"
        "s_mul_i32 s37, s74, s68\n"
        "s_mul_i32 s78, s68, s69\n"
        "s_mul_hi_u32 s38, s68, s37\n"
        "s_mul_hi_u32 s77, s68, s69\n"
        "s_add_u32 s78, s38, s78\n"
        "s_addc_u32 s77, 0, s77\n"
        "s_mul_hi_u32 s40, s76, s37\n"
        "s_mul_i32 s37, s76, s37\n"
        "s_add_u32 s78, s78, s37\n"
        "s_mul_hi_u32 s38, s76, s69\n"
        "s_addc_u32 s77, s77, s40\n"
        "s_addc_u32 s78, s38, 0\n"
        "s_mul_i32 s69, s76, s69\n"
        "s_add_u32 s69, s77, s69\n"
        "s_addc_u32 s77, 0, s78\n"
        "s_add_u32 s78, s68, s69\n"
        "s_cselect_b64 s[68:69], -1, 0\n"
        "s_cmp_lg_u64 s[68:69], 0\n"
        "s_addc_u32 s76, s76, s77\n"
        "s_mul_i32 s68, s74, s76\n"
        "s_mul_hi_u32 s69, s74, s78\n"
        "s_add_i32 s68, s69, s68\n"
        "s_mul_i32 s75, s75, s78\n"
        "s_add_i32 s68, s68, s75\n"
        "s_mul_i32 s74, s74, s78\n"
        "s_mul_hi_u32 s75, s76, s74\n"
        "s_mul_i32 s77, s76, s74\n"
        "s_mul_i32 s38, s78, s68\n"
        "s_mul_hi_u32 s74, s78, s74\n"
        "s_mul_hi_u32 s37, s78, s68\n"
        "s_add_u32 s74, s74, s38\n"
        "s_addc_u32 s37, 0, s37\n"
        "s_add_u32 s74, s74, s77\n"
        "s_mul_hi_u32 s69, s76, s68\n"
        "s_addc_u32 s74, s37, s75\n"
        "s_addc_u32 s69, s69, 0\n"
        "s_mul_i32 s68, s76, s68\n"
        "s_add_u32 s68, s74, s68\n"
        "s_addc_u32 s74, 0, s69\n"
        "s_add_u32 s75, s78, s68\n"
        "s_cselect_b64 s[68:69], -1, 0\n"
        "s_cmp_lg_u64 s[68:69], 0\n"
        "s_addc_u32 s68, s76, s74\n"
        "s_mul_i32 s74, s64, s68\n"
        "s_mul_hi_u32 s76, s64, s75\n"
        "s_mul_hi_u32 s69, s64, s68\n"
        "s_add_u32 s74, s76, s74\n"
        "s_addc_u32 s69, 0, s69\n"
        "s_mul_hi_u32 s77, s65, s75\n"
        "s_mul_i32 s75, s65, s75\n"
        "s_add_u32 s74, s74, s75\n"
        "s_mul_hi_u32 s76, s65, s68\n"
        "s_addc_u32 s69, s69, s77\n"
        "s_addc_u32 s74, s76, 0\n"
        "s_mul_i32 s68, s65, s68\n"
        "s_add_u32 s76, s69, s68\n"
        "s_addc_u32 s77, 0, s74\n"
        "s_mul_i32 s68, s66, s77\n"
        "s_mul_hi_u32 s69, s66, s76\n"
        "s_add_i32 s68, s69, s68\n"
        "s_mul_i32 s69, s67, s76\n"
        "s_add_i32 s78, s68, s69\n"
        "s_sub_i32 s74, s65, s78\n"
        "s_mul_i32 s68, s66, s76\n"
        "s_sub_u32 s37, s64, s68\n"
        "s_cselect_b64 s[68:69], -1, 0\n"
        "s_cmp_lg_u64 s[68:69], 0\n"
        "s_subb_u32 s38, s74, s67\n"
        "s_sub_u32 s40, s37, s66\n"
        "s_cselect_b64 s[74:75], -1, 0\n"
        "s_cmp_lg_u64 s[74:75], 0\n"
        "s_subb_u32 s74, s38, 0\n"
        "s_cmp_ge_u32 s74, s67\n"
        "s_cselect_b32 s75, -1, 0\n"
        "s_cmp_ge_u32 s40, s66\n"
        "s_cselect_b32 s38, -1, 0\n"
        "s_cmp_eq_u32 s74, s67\n"
        "s_cselect_b32 s74, s38, s75\n"
        "s_add_u32 s75, s76, 1\n"
        "s_addc_u32 s38, s77, 0\n"
        "s_add_u32 s40, s76, 2\n"
        "s_addc_u32 s41, s77, 0\n"
        "s_cmp_lg_u32 s74, 0\n"
        "s_cselect_b32 s74, s40, s75\n"
        "s_cselect_b32 s75, s41, s38\n"
        "s_cmp_lg_u64 s[68:69], 0\n"
        "s_subb_u32 s65, s65, s78\n"
        "s_cmp_ge_u32 s65, s67\n"
        "s_cselect_b32 s68, -1, 0\n"
        "s_cmp_ge_u32 s37, s66\n"
        "s_cselect_b32 s69, -1, 0\n"
        "s_cmp_eq_u32 s65, s67\n"
        "s_cselect_b32 s67, s69, s68\n"
        "s_cmp_lg_u32 s67, 0\n"
        "s_cselect_b32 s69, s75, s77\n"
        "s_cselect_b32 s68, s74, s76\n"
        "s_branch L_dvr%=\n"
        "L_dv32%=:\n"
        "v_cvt_f32_u32 v0, s66\n"
        "s_sub_i32 s62, 0, s66\n"
        "s_mov_b32 s69, 0\n"
        "v_rcp_iflag_f32 v0, v0\n"
        "s_nop 0\n"
        "v_mul_f32 v0, 0x4f7ffffe, v0\n"
        "v_cvt_u32_f32 v0, v0\n"
        "s_nop 0\n"
        "v_readfirstlane_b32 s76, v0\n"
        "s_mul_i32 s62, s62, s76\n"
        "s_mul_hi_u32 s62, s76, s62\n"
        "s_add_i32 s76, s76, s62\n"
        "s_mul_hi_u32 s62, s64, s76\n"
        "s_mul_i32 s67, s62, s66\n"
        "s_sub_i32 s67, s64, s67\n"
        "s_add_i32 s76, s62, 1\n"
        "s_sub_i32 s64, s67, s66\n"
        "s_cmp_ge_u32 s67, s66\n"
        "s_cselect_b32 s62, s76, s62\n"
        "s_cselect_b32 s67, s64, s67\n"
        "s_add_i32 s76, s62, 1\n"
        "s_cmp_ge_u32 s67, s66\n"
        "s_cselect_b32 s68, s76, s62\n"
        "L_dvr%=:\n"                       // Q = s[68:69]; R = |N| - Q |D|
        "s_mul_i32 s74, s68, s46\n"
        "s_mul_hi_u32 s75, s68, s46\n"
        "s_mul_i32 s62, s68, s47\n"
        "s_add_u32 s75, s75, s62\n"
        "s_mul_i32 s62, s69, s46\n"
        "s_add_u32 s75, s75, s62\n"
        "s_sub_u32 s74, s44, s74\n"
        "s_subb_u32 s75, s45, s75\n"
        "s_cmp_eq_u32 s52, 0\n"
        "s_cbranch_scc1 L_dvq%=\n"
        "s_sub_u32 s68, 0, s68\n"
        "s_subb_u32 s69, 0, s69\n"
        "L_dvq%=:\n"
        "s_cmp_eq_u32 s53, 0\n"
        "s_cbranch_scc1 L_dvsel%=\n"
        "s_sub_u32 s74, 0, s74\n"
        "s_subb_u32 s75, 0, s75\n"
        "L_dvsel%=:\n"
        "s_bitcmp1_b32 s36, 0\n"
        "s_cselect_b64 s[48:49], s[74:75], s[68:69]\n"
        "s_branch L_wb%=\n"
        // ---- branches on a, b (not av / bv)
        "L_bgeu%=:\n"                      // taken unless a <u b
        "s_cmp_lt_u32 s45, s43\n"
        "s_cbranch_scc1 L_nowb%=\n"
        "s_cmp_lg_u32 s45, s43\n"
        "s_cbranch_scc1 L_taken%=\n"
        "s_cmp_lt_u32 s44, s42\n"
        "s_cbranch_scc1 L_nowb%=\n"
        "s_branch L_taken%=\n"
        "L_beq%=:\n"
        "s_cmp_eq_u64 s[44:45], s[42:43]\n"
        "s_cbranch_scc1 L_taken%=\n"
        "s_branch L_nowb%=\n"
        "L_bne%=:\n"
        "s_cmp_lg_u64 s[44:45], s[42:43]\n"
        "s_cbranch_scc1 L_taken%=\n"
        "s_branch L_nowb%=\n"
        "L_blt%=:\n"
        "s_cmp_lt_i32 s45, s43\n"
        "s_cbranch_scc1 L_taken%=\n"
        "s_cmp_lg_u32 s45, s43\n"
        "s_cbranch_scc1 L_nowb%=\n"
        "s_cmp_lt_u32 s44, s42\n"
        "s_cbranch_scc1 L_taken%=\n"
        "s_branch L_nowb%=\n"
        "L_bge%=:\n"
        "s_cmp_lt_i32 s45, s43\n"
        "s_cbranch_scc1 L_nowb%=\n"
        "s_cmp_lg_u32 s45, s43\n"
        "s_cbranch_scc1 L_taken%=\n"
        "s_cmp_lt_u32 s44, s42\n"
        "s_cbranch_scc1 L_nowb%=\n"
        "s_branch L_taken%=\n"
        "L_bltu%=:\n"
        "s_cmp_lt_u32 s45, s43\n"
        "s_cbranch_scc1 L_taken%=\n"
        "s_cmp_lg_u32 s45, s43\n"
        "s_cbranch_scc1 L_nowb%=\n"
        "s_cmp_lt_u32 s44, s42\n"
        "s_cbranch_scc1 L_taken%=\n"
        "s_branch L_nowb%=\n"
        "L_taken%=:\n"                      // npc = pc + imm
        "s_add_u32 s50, s22, s5\n"
        "s_addc_u32 s51, s23, 0\n"
        "s_add_u32 s50, s50, s52\n"
        "s_addc_u32 s51, s51, s53\n"
        "s_branch L_jump%=\n"
        "L_jal%=:\n"                        // v = pc + len, npc = pc + imm
        "s_add_u32 s50, s22, s5\n"
        "s_addc_u32 s51, s23, 0\n"
        "s_add_u32 s48, s50, s60\n"
        "s_addc_u32 s49, s51, 0\n"
        "s_add_u32 s50, s50, s52\n"
        "s_addc_u32 s51, s51, s53\n"
        "s_branch L_jwb%=\n"
        "L_jalr%=:\n"                       // v = pc + len, npc = (a + imm) & ~1
        "s_add_u32 s50, s22, s5\n"
        "s_addc_u32 s51, s23, 0\n"
        "s_add_u32 s48, s50, s60\n"
        "s_addc_u32 s49, s51, 0\n"
        "s_add_u32 s50, s44, s52\n"
        "s_addc_u32 s51, s45, s53\n"
        "s_and_b32 s50, s50, -2\n"
        "L_jwb%=:\n"
        "s_cmp_eq_u32 s57, 0\n"
        "s_cselect_b32 m0, 32, s57\n"
        "v_writelane_b32 v28, s48, m0\n"
        "v_writelane_b32 v29, s49, m0\n"
        "L_jump%=:\n"
        "s_add_u32 s6, s6, 1\n"             // commit
        "s_bfe_u32 s62, s39, 0x10009\n"     // straddle tick (kPreStraddle)
        "s_add_u32 s8, s8, s62\n"
        "s_add_u32 s9, s9, s60\n"
        "s_sub_u32 s62, s50, s22\n"         // d = npc - tlo inside the text?
        "s_subb_u32 s64, s51, s23\n"
        "s_cmp_lg_u32 s64, 0\n"
        "s_cbranch_scc1 L_left%=\n"
        "s_cmp_ge_u32 s62, s11\n"
        "s_cbranch_scc1 L_left%=\n"
        "s_mov_b32 s5, s62\n"
        "s_branch L_top%=\n"
        // ---- loads and stores: the whole access in one mapped page
        "L_mem%=:\n"
        "s_bfe_u32 s54, s39, 0x2001c\n"     // log2 size
        "s_lshl_b32 s63, 1, s54\n"          // msz
        "s_add_u32 s64, s44, s52\n"         // ea = a + imm
        "s_addc_u32 s65, s45, s53\n"
        "s_lshr_b64 s[66:67], s[64:65], 12\n"
        "s_cmp_eq_u64 s[66:67], s[26:27]\n"
        "s_cbranch_scc1 L_pg%=\n"
        "s_cmp_eq_u64 s[66:67], s[70:71]\n"
        "s_cbranch_scc0 L_tlb%=\n"
        "s_mov_b64 s[74:75], s[26:27]\n"    // slot 1 hit: swap the slots
        "s_mov_b64 s[26:27], s[70:71]\n"
        "s_mov_b64 s[70:71], s[74:75]\n"
        "s_mov_b64 s[74:75], s[28:29]\n"
        "s_mov_b64 s[28:29], s[72:73]\n"
        "s_mov_b64 s[72:73], s[74:75]\n"
        "s_branch L_pg%=\n"
        "L_tlb%=:\n"                        // the lane's TLB (LaneMem tv0..tv3, tp0..tp3)
        "ds_read2_b64 v[0:3], v18 offset0:0 offset1:1\n"
        "ds_read2_b64 v[4:7], v18 offset0:2 offset1:3\n"
        "ds_read2_b64 v[8:11], v18 offset0:4 offset1:5\n"
        "ds_read2_b64 v[20:23], v18 offset0:6 offset1:7\n"
        "s_waitcnt lgkmcnt(0)\n"
        "v_readfirstlane_b32 s68, v0\n"
        "v_readfirstlane_b32 s69, v1\n"
        "s_cmp_eq_u64 s[68:69], s[66:67]\n"
        "s_cbranch_scc1 L_t0%=\n"
        "v_readfirstlane_b32 s68, v2\n"
        "v_readfirstlane_b32 s69, v3\n"
        "s_cmp_eq_u64 s[68:69], s[66:67]\n"
        "s_cbranch_scc1 L_t1%=\n"
        "v_readfirstlane_b32 s68, v4\n"
        "v_readfirstlane_b32 s69, v5\n"
        "s_cmp_eq_u64 s[68:69], s[66:67]\n"
        "s_cbranch_scc1 L_t2%=\n"
        "v_readfirstlane_b32 s68, v6\n"
        "v_readfirstlane_b32 s69, v7\n"
        "s_cmp_eq_u64 s[68:69], s[66:67]\n"
        "s_cbranch_scc0 L_slow%=\n"         // not in the TLB: the C++ loop's full lookup
        "v_readfirstlane_b32 s68, v22\n"
        "v_readfirstlane_b32 s69, v23\n"
        "s_branch L_tins%=\n"
        "L_t0%=:\n"
        "v_readfirstlane_b32 s68, v8\n"
        "v_readfirstlane_b32 s69, v9\n"
        "s_branch L_tins%=\n"
        "L_t1%=:\n"
        "v_readfirstlane_b32 s68, v10\n"
        "v_readfirstlane_b32 s69, v11\n"
        "s_branch L_tins%=\n"
        "L_t2%=:\n"
        "v_readfirstlane_b32 s68, v20\n"
        "v_readfirstlane_b32 s69, v21\n"
        "L_tins%=:\n"                       // slot 1 = slot 0, slot 0 = (vpn, page)
        "s_mov_b64 s[70:71], s[26:27]\n"
        "s_mov_b64 s[72:73], s[28:29]\n"
        "s_mov_b64 s[26:27], s[66:67]\n"
        "s_mov_b64 s[28:29], s[68:69]\n"
        "L_pg%=:\n"
        "s_and_b32 s78, s64, 0xfff\n"       // offset in the page
        "s_add_u32 s62, s78, s63\n"
        "s_cmp_gt_u32 s62, 0x1000\n"
        "s_cbranch_scc1 L_slow%=\n"         // crosses the page
        "s_and_b32 s76, s28, -2\n"          // address in the page
        "s_mov_b32 s77, s29\n"
        "s_add_u32 s76, s76, s78\n"
        "s_addc_u32 s77, s77, 0\n"
        "v_mov_b32 v0, s76\n"
        "v_mov_b32 v1, s77\n"
        "s_cmp_eq_u32 s56, 13\n"
        "s_cbranch_scc1 L_st%=\n"
        // load (nothing leaves from here on: its data bytes count); a
        // misaligned one inside the page byte by byte (L_mv)
        "s_add_u32 s10, s10, s63\n"
        "s_sub_u32 s62, s63, 1\n"
        "s_and_b32 s62, s78, s62\n"
        "s_mov_b32 s36, 0\n"
        "s_cbranch_scc1 L_mv%=\n"
        "s_cmp_eq_u32 s54, 3\n"
        "s_cbranch_scc1 L_ld8%=\n"
        "s_cmp_eq_u32 s54, 2\n"
        "s_cbranch_scc1 L_ld4%=\n"
        "s_cmp_eq_u32 s54, 1\n"
        "s_cbranch_scc1 L_ld2%=\n"
        "global_load_ubyte v2, v[0:1], off\n"
        "s_branch L_ldn%=\n"
        "L_ld2%=:\n"
        "global_load_ushort v2, v[0:1], off\n"
        "s_branch L_ldn%=\n"
        "L_ld4%=:\n"
        "global_load_dword v2, v[0:1], off\n"
        "s_branch L_ldn%=\n"
        "L_ld8%=:\n"
        "global_load_dwordx2 v[2:3], v[0:1], off\n"
        "L_ld8w%=:\n"
        "s_waitcnt vmcnt(0)\n"
        "v_readfirstlane_b32 s48, v2\n"
        "v_readfirstlane_b32 s49, v3\n"
        "s_branch L_wb%=\n"
        "L_ldn%=:\n"                        // 1, 2 or 4 bytes: zero- or sign-extended (U_SEXT)
        "s_waitcnt vmcnt(0)\n"
        "v_readfirstlane_b32 s48, v2\n"
        "s_mov_b32 s49, 0\n"
        "s_bitcmp1_b32 s39, 27\n"
        "s_cbranch_scc0 L_wb%=\n"
        "s_lshl_b32 s62, s63, 19\n"         // width 8 * msz, offset 0
        "s_bfe_i64 s[48:49], s[48:49], s62\n"
        "s_branch L_wb%=\n"
        // store: a page the lane owns, nothing of the code range
        "L_st%=:\n"
        "s_bitcmp1_b32 s28, 0\n"
        "s_cbranch_scc0 L_slow%=\n"
        "s_add_u32 s74, s64, s63\n"         // u = ea + msz - 1 - clo
        "s_addc_u32 s75, s65, 0\n"
        "s_sub_u32 s74, s74, 1\n"
        "s_subb_u32 s75, s75, 0\n"
        "s_sub_u32 s74, s74, s24\n"
        "s_subb_u32 s75, s75, s25\n"
        "s_cmp_lg_u32 s75, 0\n"
        "s_cbranch_scc1 L_stok%=\n"
        "s_add_u32 s62, s15, s63\n"         // overlaps [clo, clo + csz) iff u < csz + msz - 1
        "s_sub_u32 s62, s62, 1\n"
        "s_cmp_lt_u32 s74, s62\n"
        "s_cbranch_scc1 L_stc%=\n"
        "L_stok%=:\n"
        "s_add_u32 s10, s10, s63\n"         // data bytes
        "v_mov_b32 v2, s42\n"
        "v_mov_b32 v3, s43\n"
        "s_sub_u32 s62, s63, 1\n"           // misaligned inside the page: bytes
        "s_and_b32 s62, s78, s62\n"
        "s_cbranch_scc1 L_stmis%=\n"
        "s_cmp_eq_u32 s54, 3\n"
        "s_cbranch_scc1 L_st8%=\n"
        "s_cmp_eq_u32 s54, 2\n"
        "s_cbranch_scc1 L_st4%=\n"
        "s_cmp_eq_u32 s54, 1\n"
        "s_cbranch_scc1 L_st2%=\n"
        "global_store_byte v[0:1], v2, off\n"
        "s_branch L_std%=\n"
        "L_st2%=:\n"
        "global_store_short v[0:1], v2, off\n"
        "s_branch L_std%=\n"
        "L_st4%=:\n"
        "global_store_dword v[0:1], v2, off\n"
        "s_branch L_std%=\n"
        "L_st8%=:\n"
        "global_store_dwordx2 v[0:1], v[2:3], off\n"
        "L_std%=:\n"
        "s_nop 1\n"
        "s_branch L_nowb%=\n"
        // a misaligned store inside the page, byte by byte
        "L_stmis%=:\n"
        "v_lshrrev_b32 v4, 8, v2\n"
        "v_lshrrev_b32 v5, 16, v2\n"
        "v_lshrrev_b32 v6, 24, v2\n"
        "v_lshrrev_b32 v7, 8, v3\n"
        "v_lshrrev_b32 v8, 16, v3\n"
        "v_lshrrev_b32 v9, 24, v3\n"
        "global_store_byte v[0:1], v2, off\n"
        "global_store_byte v[0:1], v4, off offset:1\n"
        "s_cmp_eq_u32 s54, 1\n"
        "s_cbranch_scc1 L_std%=\n"
        "global_store_byte v[0:1], v5, off offset:2\n"
        "global_store_byte v[0:1], v6, off offset:3\n"
        "s_cmp_eq_u32 s54, 2\n"
        "s_cbranch_scc1 L_std%=\n"
        "global_store_byte v[0:1], v3, off offset:4\n"
        "global_store_byte v[0:1], v7, off offset:5\n"
        "global_store_byte v[0:1], v8, off offset:6\n"
        "global_store_byte v[0:1], v9, off offset:7\n"
        "s_branch L_std%=\n"
        // the value of a misaligned access inside the page (2, 4 or 8 bytes)
        // byte by byte into v2 (low word) / v3 (high word), zero-extended;
        // then back to the load (s36 = 0) or the code-store check (s36 = 1)
        "L_mv%=:\n"
        "global_load_ubyte v2, v[0:1], off\n"
        "global_load_ubyte v3, v[0:1], off offset:1\n"
        "s_cmp_eq_u32 s54, 1\n"
        "s_cbranch_scc1 L_mv2%=\n"
        "global_load_ubyte v4, v[0:1], off offset:2\n"
        "global_load_ubyte v5, v[0:1], off offset:3\n"
        "s_cmp_eq_u32 s54, 2\n"
        "s_cbranch_scc1 L_mv4%=\n"
        "global_load_ubyte v6, v[0:1], off offset:4\n"
        "global_load_ubyte v7, v[0:1], off offset:5\n"
        "global_load_ubyte v8, v[0:1], off offset:6\n"
        "global_load_ubyte v9, v[0:1], off offset:7\n"
        "s_waitcnt vmcnt(0)\n"
        "v_lshl_or_b32 v6, v7, 8, v6\n"
        "v_lshl_or_b32 v6, v8, 16, v6\n"
        "v_lshl_or_b32 v6, v9, 24, v6\n"
        "s_branch L_mv4c%=\n"
        "L_mv4%=:\n"
        "s_waitcnt vmcnt(0)\n"
        "v_mov_b32 v6, 0\n"
        "L_mv4c%=:\n"
        "v_lshl_or_b32 v2, v3, 8, v2\n"
        "v_lshl_or_b32 v2, v4, 16, v2\n"
        "v_lshl_or_b32 v2, v5, 24, v2\n"
        "v_mov_b32 v3, v6\n"
        "s_branch L_mvd%=\n"
        "L_mv2%=:\n"
        "s_waitcnt vmcnt(0)\n"
        "v_lshl_or_b32 v2, v3, 8, v2\n"
        "v_mov_b32 v3, 0\n"
        "L_mvd%=:\n"
        "s_cmp_eq_u32 s36, 0\n"
        "s_cbranch_scc0 L_stcmv%=\n"
        "s_cmp_eq_u32 s54, 3\n"
        "s_cbranch_scc1 L_ld8w%=\n"
        "s_branch L_ldn%=\n"
        "L_stcmv%=:\n"
        "s_cmp_eq_u32 s54, 3\n"
        "s_cbranch_scc1 L_stc8w%=\n"
        "s_and_b32 s62, s42, 0xffff\n"
        "s_cmp_eq_u32 s54, 2\n"
        "s_cselect_b32 s62, s42, s62\n"
        "s_branch L_stcw%=\n"
        // a store into the code range that writes the bytes already there
        // changes nothing (solo_pre_run: no rewrite to mark): it commits here
        // without writing; one that changes them marks the rewrite (L_stdirty)
        "L_stc%=:\n"
        "s_sub_u32 s62, s63, 1\n"
        "s_and_b32 s62, s78, s62\n"
        "s_mov_b32 s36, 1\n"
        "s_cbranch_scc1 L_mv%=\n"
        "s_cmp_eq_u32 s54, 3\n"
        "s_cbranch_scc1 L_stc8%=\n"
        "s_cmp_eq_u32 s54, 2\n"
        "s_cbranch_scc1 L_stc4%=\n"
        "s_cmp_eq_u32 s54, 1\n"
        "s_cbranch_scc1 L_stc2%=\n"
        "global_load_ubyte v2, v[0:1], off\n"
        "s_and_b32 s62, s42, 0xff\n"
        "s_branch L_stcw%=\n"
        "L_stc2%=:\n"
        "global_load_ushort v2, v[0:1], off\n"
        "s_and_b32 s62, s42, 0xffff\n"
        "s_branch L_stcw%=\n"
        "L_stc4%=:\n"
        "global_load_dword v2, v[0:1], off\n"
        "s_mov_b32 s62, s42\n"
        "L_stcw%=:\n"
        "s_waitcnt vmcnt(0)\n"
        "v_readfirstlane_b32 s74, v2\n"
        "s_cmp_eq_u32 s74, s62\n"
        "s_cbranch_scc0 L_stdirty%=\n"
        "s_add_u32 s10, s10, s63\n"         // data bytes
        "s_branch L_nowb%=\n"
        "L_stc8%=:\n"
        "global_load_dwordx2 v[2:3], v[0:1], off\n"
        "L_stc8w%=:\n"
        "s_waitcnt vmcnt(0)\n"
        "v_readfirstlane_b32 s74, v2\n"
        "v_readfirstlane_b32 s75, v3\n"
        "s_cmp_eq_u64 s[74:75], s[42:43]\n"
        "s_cbranch_scc0 L_stdirty%=\n"
        "s_add_u32 s10, s10, s63\n"
        "s_branch L_nowb%=\n"
        // a store that rewrites code bytes [ea, ea + msz): mark it as
        // solo_pre_run does (mark_dirty_solo + its window + cache drops), then
        // store.  A first rewrite (no window yet: the map starts then) is the
        // C++ loop's.
        "L_stdirty%=:\n"
        "s_cmp_eq_u32 s12, -1\n"
        "s_cbranch_scc1 L_slow%=\n"
        // LaneMem dlo = min(dlo, ea), dhi = max(dhi, ea + msz)
        "ds_read2_b64 v[2:5], v18 offset0:12 offset1:13\n"
        "s_add_u32 s66, s64, s63\n"         // s[66:67] = ea + msz
        "s_addc_u32 s67, s65, 0\n"
        "s_waitcnt lgkmcnt(0)\n"
        "v_readfirstlane_b32 s68, v2\n"
        "v_readfirstlane_b32 s69, v3\n"
        "v_readfirstlane_b32 s40, v4\n"
        "v_readfirstlane_b32 s41, v5\n"
        "s_sub_u32 s62, s64, s68\n"         // ea < dlo?
        "s_subb_u32 s62, s65, s69\n"
        "s_cselect_b64 s[68:69], s[64:65], s[68:69]\n"
        "s_sub_u32 s62, s40, s66\n"         // dhi < ea + msz?
        "s_subb_u32 s62, s41, s67\n"
        "s_cselect_b64 s[40:41], s[66:67], s[40:41]\n"
        "v_mov_b32 v2, s68\n"
        "v_mov_b32 v3, s69\n"
        "v_mov_b32 v4, s40\n"
        "v_mov_b32 v5, s41\n"
        "ds_write2_b64 v18, v[2:3], v[4:5] offset0:12 offset1:13\n"
        // the window as text offsets: o0 = max(ea, tlo) - tlo, o1 = ea + msz - tlo
        "s_sub_u32 s68, s64, s22\n"
        "s_subb_u32 s69, s65, s23\n"
        "s_cselect_b32 s68, 0, s68\n"       // (ea below the text: 0)
        "s_sub_u32 s69, s66, s22\n"         // o1
        "s_min_u32 s12, s12, s68\n"
        "s_add_u32 s62, s69, 3\n"
        "s_max_u32 s13, s13, s62\n"
        // drop the decode-cache and entry-cache entries whose tag t is in
        // [o0 - 3, o1) -- all 64 at once, every lane of the wave
        "s_sub_u32 s68, s68, 3\n"           // lo3 = o0 >= 3 ? o0 - 3 : 0
        "s_cselect_b32 s68, 0, s68\n"
        "s_sub_u32 s69, s69, s68\n"         // width o1 - lo3
        "v_readfirstlane_b32 s40, v16\n"    // DCT (LDS)
        "s_mov_b64 s[74:75], exec\n"
        "s_mov_b64 exec, -1\n"
        "v_subrev_u32 v2, s68, v24\n"
        "v_cmp_gt_u32 vcc, s69, v2\n"
        "v_cndmask_b32_e64 v24, v24, -1, vcc\n"
        "v_mbcnt_lo_u32_b32 v4, -1, 0\n"
        "v_mbcnt_hi_u32_b32 v4, -1, v4\n"
        "v_lshl_add_u32 v5, v4, 2, s40\n"
        "ds_read_b32 v6, v5\n"
        "s_waitcnt lgkmcnt(0)\n"
        "v_subrev_u32 v7, s68, v6\n"
        "v_cmp_gt_u32 vcc, s69, v7\n"
        "s_mov_b64 exec, vcc\n"
        "v_mov_b32 v6, -1\n"
        "ds_write_b32 v5, v6\n"
        "s_mov_b64 exec, s[74:75]\n"
        // the LDS map: granules (max(ea, clo) - clo) >> sh .. (min(ea + msz, chi) - 1 - clo) >> sh
        "ds_read2_b32 v[2:3], v31 offset0:32 offset1:33\n"
        "s_sub_u32 s68, s64, s24\n"         // e0 = ea - clo (0 below the code)
        "s_subb_u32 s69, s65, s25\n"
        "s_cselect_b32 s68, 0, s68\n"
        "s_sub_u32 s69, s66, s24\n"         // e1 = min(ea + msz - clo, csz)
        "s_min_u32 s69, s69, s15\n"
        "s_sub_u32 s69, s69, 1\n"
        "s_waitcnt lgkmcnt(0)\n"
        "v_readfirstlane_b32 s40, v2\n"     // dl (LDS; 0: no map)
        "v_readfirstlane_b32 s41, v3\n"     // shift
        "s_cmp_eq_u32 s40, 0\n"
        "s_cbranch_scc1 L_stok%=\n"
        "s_lshr_b32 s68, s68, s41\n"
        "s_lshr_b32 s69, s69, s41\n"
        "L_dmark%=:\n"
        "s_lshr_b32 s62, s68, 5\n"
        "s_lshl_b32 s62, s62, 2\n"
        "s_add_u32 s62, s62, s40\n"
        "s_lshl_b32 s41, 1, s68\n"          // (the shift count's low 5 bits: q & 31)
        "v_mov_b32 v2, s62\n"
        "v_mov_b32 v3, s41\n"
        "ds_or_b32 v2, v3\n"
        "s_add_u32 s68, s68, 1\n"
        "s_cmp_gt_u32 s68, s69\n"
        "s_cbranch_scc0 L_dmark%=\n"
        "s_waitcnt lgkmcnt(0)\n"
        "s_branch L_stok%=\n"
        // ================================================================ exits
        "L_left%=:\n"
        "s_mov_b32 s19, 3\n"
        "s_branch L_out%=\n"
        "L_budget%=:\n"
        "s_mov_b32 s19, 0\n"
        "s_branch L_out%=\n"
        "L_leader%=:\n"
        "s_mov_b32 s19, 2\n"
        "s_branch L_out%=\n"
        "L_slow%=:\n"
        "s_mov_b32 s19, 1\n"
        "L_out%=:\n"
        "v_mov_b32 v0, s5\n"
        "v_mov_b32 v1, s6\n"
        "v_mov_b32 v2, s8\n"
        "v_mov_b32 v3, s9\n"
        "v_mov_b32 v4, s10\n"
        "v_mov_b32 v5, s19\n"
        "v_mov_b32 v6, s26\n"
        "v_mov_b32 v7, s27\n"
        "v_mov_b32 v8, s28\n"
        "v_mov_b32 v9, s29\n"
        "v_mov_b32 v10, s50\n"
        "v_mov_b32 v11, s51\n"
        "ds_write2_b32 v31, v0, v1 offset0:0 offset1:1\n"
        "ds_write2_b32 v31, v2, v3 offset0:3 offset1:4\n"
        "ds_write_b32 v31, v4 offset:20\n"
        "ds_write_b32 v31, v5 offset:56\n"
        "v_mov_b32 v12, s12\n"              // ddlo, ddhi + 3 (a rewrite may have grown them)
        "v_mov_b32 v13, s13\n"
        "ds_write2_b32 v31, v12, v13 offset0:7 offset1:8\n"
        "ds_write2_b64 v31, v[6:7], v[8:9] offset0:13 offset1:14\n"
        "ds_write_b64 v31, v[10:11] offset:120\n"
        "v_readfirstlane_b32 s62, v15\n"    // the guest registers back to R (lanes 0..31)
        "s_mov_b64 s[74:75], exec\n"
        "s_mov_b32 exec_lo, -1\n"
        "s_mov_b32 exec_hi, 0\n"
        "v_mbcnt_lo_u32_b32 v14, -1, 0\n"
        "v_lshl_add_u32 v14, v14, 3, s62\n"
        "ds_write_b64 v14, v[28:29]\n"
        "s_mov_b64 exec, s[74:75]\n"
        "v_readfirstlane_b32 s62, v19\n"   // the entry cache back to LDS (all lanes)
        "s_mov_b64 s[74:75], exec\n"
        "s_mov_b64 exec, -1\n"
        "v_mbcnt_lo_u32_b32 v30, -1, 0\n"
        "v_mbcnt_hi_u32_b32 v30, -1, v30\n"
        "v_lshl_add_u32 v30, v30, 4, s62\n"
        "ds_write_b128 v30, v[24:27]\n"
        "s_mov_b64 exec, s[74:75]\n"
        "s_waitcnt vmcnt(0) lgkmcnt(0)\n"
        "s_mov_b32 m0, s4\n"
        :
        : [io] "v"(a)
        : "s4", "s5", "s6", "s7", "s8", "s9", "s10", "s11", "s12", "s13", "s14", "s15", "s16", "s17", "s18", "s19",
          "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29",
          "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50",
          "s51", "s52", "s53", "s54", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66",
          "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82",
          "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15",
          "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30",
          "v31", "vcc", "memory");
}

// 64-bit unsigned / signed compares of uniform values on the scalar unit
// (SALU compares are 32-bit; a 64-bit one otherwise goes through VALU + VCC)
__device__ __forceinline__ bool slt64(uint64_t a, uint64_t b) {
    const int32_t ah = (int32_t)(a >> 32), bh = (int32_t)(b >> 32);
    return ah < bh || (ah == bh && (uint32_t)a < (uint32_t)b);
}
__device__ __forceinline__ uint64_t r64(const lds_u64 *R, uint32_t r) { return uni64(R[r]); }

template <bool kOdd>
__device__ __noinline__ void solo_pre_run(KCtx *CX, lds_u64 *R, lds_mem *mp, lds_u32 *DCT, lds_pre4 *DCE,
                                          lds_u32 *LC, lds_pio *io) {
    CX = (KCtx *)(uintptr_t)uni64((uint64_t)(uintptr_t)CX);
    R = (lds_u64 *)(uintptr_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)R);
    mp = (lds_mem *)(uintptr_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)mp);
    DCT = (lds_u32 *)(uintptr_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)DCT);
    DCE = (lds_pre4 *)(uintptr_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)DCE);
    LC = (lds_u32 *)(uintptr_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)LC);
    io = (lds_pio *)(uintptr_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)io);
    LaneMem &m = *(LaneMem *)mp;   // lookup_full / fetch_lane / mark_dirty_solo take it by reference
    const uint64_t slot = uni64(io->slot);
    WaveMem w;
    w.tab = (const PageEnt *)uni64((uint64_t)io->tab);
    w.tab_n = uni32(io->tab_n);
    const uint32_t budget = uni32(io->budget);
#ifdef FI_TX
    const uint32_t tx_gate = uni32(io->tx_gate), tx_gate1 = tx_gate > 1 ? tx_gate : 1u;
#endif
    int32_t watch = (int32_t)uni32((uint32_t)io->watch);
    // pcs as 32-bit offsets from the text base while the run stays in the text
    // (the host keeps the text inside one 4 GiB window)
    const uint64_t tlo = CX->text_lo, clo = CX->code_lo, chi = CX->code_hi;
    const uint32_t tby = CX->text_bytes;
    const uint32_t clo_o = (uint32_t)(clo - tlo), chi_o = (uint32_t)(chi - tlo);   // the code range as text offsets
    const const_u32 *const pre = (const const_u32 *)(uintptr_t)CX->pre;
    // the last page translated, in registers (the TLB itself stays in LDS:
    // mappings do not change inside a run, lookup_full only inserts)
    uint64_t cvpn = ~0ULL, cpg = 0;
    // rewritten code: the bounding range as text offsets [ddlo, ddhi) (empty
    // when clean), the LDS map for the exact test
    const bool have_dl = m.dl != nullptr;
    const __attribute__((address_space(3))) uint32_t *const dl = (const __attribute__((address_space(3))) uint32_t *)m.dl;
    const uint32_t dsh = CX->dmap_shift;
    uint32_t ddlo = 0xFFFFFFFFu, ddhi = 0u;
    if (m.code_dirty) {
        const uint64_t a = uni64(m.dlo), b = uni64(m.dhi);
        ddlo = (uint32_t)((a > tlo ? a : tlo) - tlo);
        ddhi = (uint32_t)((b > tlo ? b : tlo) - tlo);
    }
    uint64_t spc = uni64(io->spc);
    uint32_t steps = 0, xticks = 0, fbytes = 0, dbytes = 0;
    uint32_t n_fast = 0, n_fast_steps = 0, n_fast_back = 0;   // diagnostics: stats[53..55]
#ifdef FI_PROF   // phases: fetch (+ decode of rewritten code), operands, execute, commit
    uint64_t pacc[4] = {0, 0, 0, 0}, plast = __builtin_amdgcn_s_memtime();
#define PST(k)                                                  \
    do {                                                        \
        const uint64_t _t = __builtin_amdgcn_s_memtime();       \
        pacc[k] += _t - plast;                                  \
        plast = _t;                                             \
    } while (0)
#else
#define PST(k) do { } while (0)
#endif
    if ((uint32_t)((spc - tlo) >> 32) == 0 && (uint32_t)(spc - tlo) < tby) {
        uint32_t po = (uint32_t)(spc - tlo);
        // the entry of the instruction at po (odd pcs fetch like pc | 2 of their
        // word: halfword (po >> 1) | 1; text_lo is page-aligned).  Offsets up to
        // tby + 5 land on the zero (K_SLOW) entries past the text
        // (fi_engine.cpp kPreTail), so no clamp.
#define PRE_AT(o_, x_, y_, z_)                                                      \
    do {                                                                            \
        const const_u32 *q_ = pre + 4 * (((o_) >> 1) | ((o_) & 1u));                \
        x_ = q_[1]; y_ = q_[2]; z_ = q_[3];                                         \
    } while (0)
        uint32_t q1, q2, q3;
        PRE_AT(po, q1, q2, q3);
#ifndef FI_PROF
        // the assembly inner loop (solo_fast_run) takes over once a run has
        // gone 8 instructions (short runs stay here: its entry costs ~200
        // instructions), and again after each instruction it hands back
        uint32_t fast_at = 8;
        __shared__ SoloFastIO fio[1];
#endif
        while (steps < budget) {
            PST(3);
#ifndef FI_PROF
            if (steps >= fast_at && watch <= 0) {
                lds_fio *F = (lds_fio *)fio;
                F->po = po; F->steps = steps; F->budget = budget; F->xticks = xticks;
                F->fbytes = fbytes; F->dbytes = dbytes; F->tby = tby; F->ddlo = ddlo;
                F->ddhi3 = ddhi + 3u; F->clo_o = clo_o; F->csz = chi_o - clo_o;
#ifdef FI_TX
                F->gate = tx_gate1; F->lbe = kPreLeader; F->lbo = kOdd ? kPreOddLeader : 0u;
#else
                F->gate = 0xFFFFFFFFu; F->lbe = 0; F->lbo = 0;
#endif
                F->r_lds = (uint32_t)(uintptr_t)R; F->dct_lds = (uint32_t)(uintptr_t)DCT;
                F->dce_lds = (uint32_t)(uintptr_t)DCE; F->tlb_lds = (uint32_t)(uintptr_t)&mp->tv0;
                F->lc_lds = (uint32_t)(uintptr_t)LC;
                F->dl_lds = have_dl ? (uint32_t)(uintptr_t)dl : 0u; F->dsh = dsh;
                F->pre = (uint64_t)(uintptr_t)CX->pre; F->tlo = tlo; F->clo = clo; F->cvpn = cvpn; F->cpg = cpg;
                solo_fast_run(F);
                n_fast++;
                n_fast_steps += uni32(F->steps) - steps;
                po = uni32(F->po); steps = uni32(F->steps); xticks = uni32(F->xticks);
                fbytes = uni32(F->fbytes); dbytes = uni32(F->dbytes);
                cvpn = uni64(F->cvpn); cpg = uni64(F->cpg);
                ddlo = uni32(F->ddlo); ddhi = uni32(F->ddhi3) - 3u;   // (rewrites it marked)
                const uint32_t why = uni32(F->reason);
                if (why == 3) { spc = uni64(F->npc); goto leave; }   // a jump left the text
                if (why == 4) { spc = tlo + po; goto leave; }         // so did the fall-through
                if (why == 0) break;                                  // budget spent
                n_fast_back++;
                PRE_AT(po, q1, q2, q3);                               // the instruction it hands back
                fast_at = steps + 1;
            }
#endif
            // ---- rewritten bytes under this instruction: the decode cache
            // (an entry is the decode of the lane's current bytes: stores drop
            // the entries they overlap), else the lane's own bytes, decoded
            if (po + 6 > ddlo && po < ddhi + 3u) {   // (a superset of [pc & ~3, pc + 6) meeting the range)
                const uint32_t ci = (po >> 1) & (kSoloDC - 1);
                const uint32_t tag = uni32(DCT[ci]);
                const uint32_t e1 = uni32(DCE[ci].y), e2 = uni32(DCE[ci].z), e3 = uni32(DCE[ci].w);
                const bool in_code = po >= clo_o && po < chi_o;
                if (in_code && tag == po) {
                    q1 = e1; q2 = e2; q3 = e3;
                } else if (!have_dl || dmap_any(dl, clo, chi, dsh, (tlo + po) & ~3ULL, tlo + po + 6)) {
                    uint32_t raw = 0, t = 1;
                    uint64_t fva = 0;
                    if (fetch_lane(CX, w, m, slot, tlo + po, raw, t, fva) != 0) break;
                    Dec dd = rv_decode(uni32(raw));
                    const uint32_t u = uop_of(dd);
                    q1 = (uint32_t)dd.op | ((uint32_t)dd.rd << 8) | ((uint32_t)dd.rs1 << 16) | ((uint32_t)dd.rs2 << 24);
                    q2 = (uint32_t)dd.imm;
                    q3 = (uint32_t)dd.len | ((uint32_t)(kPreValid | (uni32(t) == 2 ? kPreStraddle : 0) | dd.flags) << 8) |
                         (u << 16);
                    q1 = uni32(q1); q2 = uni32(q2); q3 = uni32(q3);
                    if (in_code) {
                        DCT[ci] = po;
                        DCE[ci].x = dd.raw; DCE[ci].y = q1; DCE[ci].z = q2; DCE[ci].w = q3;
                    }
                } else if (in_code) {   // clean bytes in the window: the pre-decoded entry, cached for solo_fast_run
                    DCT[ci] = po;
                    DCE[ci].x = pre[4 * ((po >> 1) | (po & 1u))]; DCE[ci].y = q1; DCE[ci].z = q2; DCE[ci].w = q3;
                }
            }
            PST(0);
            const uint32_t fl = (q3 >> 8) & 0xFF, kind = (q3 >> 16) & 63;
            // (an invalid entry has kind K_SLOW too: fi_predecode_kernel leaves aux 0,
            // the entries past the text are zero, decoded entries are valid)
            if (kind == K_SLOW && !solo_fp_ok(q1 & 0xFF)) break;   // (F/D/Zfh ops: solo_fp_op below)
#ifdef FI_TX
            // a block leader (odd pcs: the solo-odd kernel's odd-pc leaders) past the first instruction
            static_assert(kPreOddLeader == kPreLeader << 1, "leader flags");
            const uint32_t lb = kOdd ? ((uint32_t)kPreLeader << (po & 1)) : ((po & 1) ? 0u : (uint32_t)kPreLeader);
            if ((fl & lb) && steps >= tx_gate1) break;
#endif
            const uint32_t rd = (q1 >> 8) & 0xFF, rs1 = (q1 >> 16) & 0xFF, rs2 = q1 >> 24;
            if (watch > 0 && (((fl & kPreRs1) && rs1 == (uint32_t)watch) || ((fl & kPreRs2) && rs2 == (uint32_t)watch)))
                break;
            const uint32_t len = q3 & 0xFF, aux = q3 >> 16;
            const int64_t imm = (int32_t)q2;
            const uint64_t pc = tlo + po;
            const uint64_t a0 = r64(R, rs1), b0 = r64(R, rs2);
            // the fall-through's entry loads while this instruction executes
            uint32_t f1, f2, f3;
            PRE_AT(po + len, f1, f2, f3);
            const uint64_t av = (aux & U_APC) ? pc : a0;
            const uint64_t bv = (aux & U_BIMM) ? (uint64_t)imm : b0;
#ifdef FI_PROF
            asm volatile("" :: "s"(av), "s"(bv));
#endif
            PST(1);
            const bool w32 = aux & U_W32;
            const uint32_t shm = w32 ? 31 : 63;
            uint64_t v = 0, npc = pc + len;
            uint32_t msz = 0;
            bool wr = true, jump = false;   // jump: npc is not the fall-through
            // (add/addi/mv/li and the compressed forms are the most common op:
            // tested before the compare tree of the switch)
            if (__builtin_expect(kind == K_ADD, 1)) {
                v = av + bv;
            } else switch (kind) {
            case K_LOAD: case K_STORE: {   // the whole access inside one mapped page
                const bool st = kind == K_STORE;
                msz = 1u << ((aux >> 12) & 3);
                const uint64_t ea = a0 + imm, vpn = ea >> 12;
                const uint32_t off = (uint32_t)ea & 4095u;
                uint64_t p = cpg;
                if (vpn != cvpn) {
                    p = uni64(tlb_find(m, vpn));
                    if (!p) p = uni64(lookup_full(CX, w, m, slot, vpn));
                    if (p) { cvpn = vpn; cpg = p; }
                }
                if (!(p && (!st || (p & 1)) && off + msz <= 4096)) { msz = 0xFFFFFFFFu; break; }   // the general path's
                __attribute__((address_space(1))) uint8_t *pg =
                    (__attribute__((address_space(1))) uint8_t *)(uintptr_t)(p & ~1ULL);
                const bool al = (off & (msz - 1)) == 0;
                if (st) {
                    wr = false;
                    // a store into the code range that changes its bytes rewrites
                    // the lane's code (one that writes the bytes already there
                    // leaves them as they were: nothing to mark)
                    bool chg = false;
                    if (!(!ult64(ea, chi) || !ult64(clo, ea + msz))) {
                        uint64_t old = 0;
                        for (uint32_t i = 0; i < msz; i++) old |= (uint64_t)pg[off + i] << (8 * i);
                        const uint64_t mk = msz == 8 ? ~0ULL : ((1ULL << (8 * msz)) - 1);
                        chg = ((uni64(old) ^ b0) & mk) != 0;
                    }
                    if (chg) {   // rewrites the lane's code
                        // (the LDS map only: the kernel writes it to the slot's map when the lane suspends)
                        mark_dirty_solo(CX, m, ea, ea + msz);
                        const uint32_t o0 = (uint32_t)((ea > tlo ? ea : tlo) - tlo), o1 = (uint32_t)(ea + msz - tlo);
                        ddlo = o0 < ddlo ? o0 : ddlo;
                        ddhi = o1 > ddhi ? o1 : ddhi;
                        for (uint32_t q = (o0 > 3 ? o0 - 3 : 0); q < o1; q++) {   // decode-cache entries over them
                            const uint32_t i = (q >> 1) & (kSoloDC - 1);
                            if (DCT[i] == q) DCT[i] = 0xFFFFFFFFu;
                            if (LC[4 * i] == q) LC[4 * i] = 0xFFFFFFFFu;   // (solo_fast_run's entry cache)
                        }
                    }
                    if (al) {
                        switch (msz) {
                        case 1: pg[off] = (uint8_t)b0; break;
                        case 2: *(__attribute__((address_space(1))) uint16_t *)(pg + off) = (uint16_t)b0; break;
                        case 4: *(__attribute__((address_space(1))) uint32_t *)(pg + off) = (uint32_t)b0; break;
                        default: *(__attribute__((address_space(1))) uint64_t *)(pg + off) = b0; break;
                        }
                    } else {
                        for (uint32_t i = 0; i < msz; i++) pg[off + i] = (uint8_t)(b0 >> (8 * i));
                    }
                } else {
                    uint64_t t = 0;
                    if (al) {
                        switch (msz) {
                        case 1: t = pg[off]; break;
                        case 2: t = *(const __attribute__((address_space(1))) uint16_t *)(pg + off); break;
                        case 4: t = *(const __attribute__((address_space(1))) uint32_t *)(pg + off); break;
                        default: t = *(const __attribute__((address_space(1))) uint64_t *)(pg + off); break;
                        }
                    } else {
                        for (uint32_t i = 0; i < msz; i++) t |= (uint64_t)pg[off + i] << (8 * i);
                    }
                    t = uni64(t);
                    v = (aux & U_SEXT) ? (uint64_t)sext64(t, 8 * msz) : t;
                }
                break;
            }
            case K_BEQ: case K_BNE: case K_BLT: case K_BGE: case K_BLTU: case K_BGEU: {
                wr = false;
                bool c;
                switch (kind) {
                case K_BEQ: c = a0 == b0; break;
                case K_BNE: c = a0 != b0; break;
                case K_BLT: c = slt64(a0, b0); break;
                case K_BGE: c = !slt64(a0, b0); break;
                case K_BLTU: c = ult64(a0, b0); break;
                default: c = !ult64(a0, b0); break;
                }
                if (c) { npc = pc + imm; jump = true; }
                break;
            }
            case K_SUB: v = av - bv; break;
            case K_AND: v = av & bv; break;
            case K_OR: v = av | bv; break;
            case K_XOR: v = av ^ bv; break;
            case K_SLT: v = slt64(av, bv) ? 1 : 0; break;
            case K_SLTU: v = ult64(av, bv) ? 1 : 0; break;
            case K_SLL: v = av << (bv & shm); break;
            case K_SRL: v = (w32 ? (av & 0xFFFFFFFFULL) : av) >> (bv & shm); break;
            case K_SRA: v = (uint64_t)((w32 ? (int64_t)(int32_t)av : (int64_t)av) >> (bv & shm)); break;
            case K_JAL: v = pc + len; npc = pc + imm; jump = true; break;
            case K_JALR: v = pc + len; npc = (a0 + imm) & ~1ULL; jump = true; break;
            case K_NOP: wr = false; break;
            case K_MUL: v = av * bv; break;
            case K_MULH: v = (uint64_t)__mul64hi((int64_t)av, (int64_t)bv); break;
            case K_MULHU: v = __umul64hi(av, bv); break;
            case K_MULHSU: v = __umul64hi(av, bv) - (((int64_t)av < 0) ? bv : 0); break;
            case K_DIV: v = w32 ? divw(av, bv) : div64(av, bv); break;
            case K_DIVU:
                v = w32 ? ((uint32_t)bv == 0 ? ~0ULL : sx32((uint32_t)av / (uint32_t)bv)) : (bv == 0 ? ~0ULL : av / bv);
                break;
            case K_REM: v = w32 ? remw(av, bv) : rem64(av, bv); break;
            case K_REMU:
                v = w32 ? ((uint32_t)bv == 0 ? sx32(av) : sx32((uint32_t)av % (uint32_t)bv)) : (bv == 0 ? av : av % bv);
                break;
            case K_SLOW: {   // an F/D/Zfh op (solo_fp_ok), out of line
                uint32_t fm = 0;
                const uint32_t r = solo_fp_op(CX, w, m, slot, R, io, q1, q2, v, fm);
                if (!r) { msz = 0xFFFFFFFFu; break; }
                wr = r == 2;
                msz = fm;
                break;
            }
            default: msz = 0xFFFFFFFFu; break;
            }
            if (msz == 0xFFFFFFFFu) break;   // nothing committed for this instruction
            v = uni64(v);
#ifdef FI_PROF
            asm volatile("" :: "s"(v));
#endif
            PST(2);
            if (w32) v = sx32(v);
            if (wr && rd) R[rd] = v;
            if (watch > 0 && wr && rd == (uint32_t)watch) watch = -1;   // overwritten before read
            steps++; xticks += (fl & kPreStraddle) ? 1u : 0u; fbytes += len; dbytes += msz;
            if (!jump) {
                po += len;
                q1 = f1; q2 = f2; q3 = f3;
            } else {
                npc = uni64(npc);
                const uint64_t d = npc - tlo;
                if ((uint32_t)(d >> 32) != 0 || (uint32_t)d >= tby) { spc = npc; goto leave; }   // left the text
                po = (uint32_t)d;
                PRE_AT(po, q1, q2, q3);
            }
            if (po >= tby) { spc = tlo + po; goto leave; }
        }
        spc = tlo + po;
#undef PRE_AT
    }
leave:
    if (n_fast) {
        atomicAdd(&CX->stats[53], (unsigned long long)n_fast);
        atomicAdd(&CX->stats[54], (unsigned long long)n_fast_steps);
        atomicAdd(&CX->stats[55], (unsigned long long)n_fast_back);
    }
    io->spc = spc; io->watch = watch;
    io->steps = steps; io->xticks = xticks; io->fbytes = fbytes; io->dbytes = dbytes;
#ifdef FI_PROF
    for (int k = 0; k < 4; k++) io->prof[k] = pacc[k];
#endif
#undef PST
}

// Waves per SIMD the register allocation must allow (the translated build
// sets it per engine; see fi_jit.cpp).
// solo kernel register budget: 4 waves per SIMD (<= 128 VGPRs).  A/B on
// crc32 (tools/gpu/solo_ab.sh, profiles/r02j_solo_ab.txt): 1 (no bound, 136-140
// VGPRs, 3 waves) 6.44M, 4: 7.06M trials/s; VGPR-pinned guest registers
// 3.2-3.7M.
#ifndef FI_SOLO_DIRTY_PRIO   // solo waves of trials that rewrote code run at this priority (0: no change)
#define FI_SOLO_DIRTY_PRIO 0
#endif
#ifndef FI_SOLO_AGE   // solo waves raise their priority at 2^k, 2^(k+1), 2^(k+2) instructions (0: off)
#define FI_SOLO_AGE 0
#endif
#ifndef FI_SOLO_WAVES_PER_EU
#define FI_SOLO_WAVES_PER_EU 4
#endif
#ifndef FI_WAVES_PER_EU
#define FI_WAVES_PER_EU 1
#endif
// A trial that leaves the translated blocks after fewer than FI_TX_SHORT
// instructions four times running stays in the interpreter: if it rewrote
// code, for the next FI_TX_SKIP (a round trip costs more than the blocks save:
// qsort 631236 re-entered every 11 instructions, ~5 us per round trip against
// ~0.2 us per instruction in the assembly interpreter).  64, not 32: intmix
// 53499 (a loop that rewrites its head every iteration) leaves after 32-63
// instructions; the intmix step 319 -> 252 ms, qsort +1.5 %, crc32 even
// (profiles/ab_bench_r05tm_*.jsonl)
#ifndef FI_TX_SHORT
#define FI_TX_SHORT 64
#endif
#ifndef FI_TX_SKIP
#define FI_TX_SKIP 4096
#endif
// ... and a trial that rewrote nothing the next FI_TX_SKIP_CLEAN, doubling
// while the short runs recur (qsort's returns into their own epilogue:
// ~3 us per instruction before, tools/gpu/launch_size.py census r05c)
#ifndef FI_TX_SKIP_CLEAN
#define FI_TX_SKIP_CLEAN 256
#endif
// (a clean trial's runs count as short below FI_TX_SHORT_CLEAN instructions,
// sixteen of them running)
#ifndef FI_TX_SHORT_CLEAN
#define FI_TX_SHORT_CLEAN 4
#endif
// Solo kernel: the launch context through a plain pointer, so that the
// compiler can keep loop-invariant fields in registers (a one-lane wave has
// VGPR lanes to spill them to) instead of a scalar load + wait at each use
// (through the opaque pointer: crc32 10.05M against 11.20M trials/s,
// profiles/r02l_ab.txt).
// kOdd: the solo-odd instantiation, whose translated blocks (the solo body
// again plus the odd-pc streams) are entered at odd pcs too.
template <uint32_t kNL, bool kOdd = false>
__device__ __forceinline__ void trial_body() {
    KCtx *const kc = (KCtx *)__builtin_amdgcn_kernarg_segment_ptr();
#define CX (kNL == 1 ? kc : opq(kc))
// Out-of-line helpers take the lane's memory state and the wave's page table
// by reference.  (Running them on copies, so that the reference does not pin
// LaneMem in scratch, made the interpreter-bound solo tail trials 10-20 %
// faster but cost the crc32 bench 12 %, 10.0M -> 8.8M trials/s,
// profiles/r02l_ab.txt.)
#define OOL(stmt)                                 \
    do {                                          \
        LaneMem &mc_ = m;                         \
        const WaveMem &wc_ = w;                   \
        stmt;                                     \
    } while (0)
    __shared__ uint64_t R[kRows * kNL];
    const uint64_t t_start = __builtin_amdgcn_s_memtime(), rt_start = __builtin_amdgcn_s_memrealtime();
    const uint32_t lane = lane_id<kNL>();
    // ---- the lane's slot: a fresh launch takes slot = global lane index, a
    // resume launch (epochs) the slots of suspended lanes, sorted by pc
    const bool resume = CX->resume != nullptr;
    uint32_t nlw = kNL == 1 ? 1u : CX->lanes;
    if (kNL > 1 && resume && CX->resume_waves) {   // few survivors: fewer per wave (the grid allows one per wave)
        const uint32_t ns = *CX->resume_n, per = (ns + CX->resume_waves - 1) / CX->resume_waves;
        uint32_t l = 1;
        while (l < per && l < nlw) l <<= 1;
        nlw = l;
    }
    // surplus waves of a resume grid (sized for the fewest lanes per wave) leave
    // at once; a solo-odd launch takes the list from *resume_lo on
    const uint32_t rlo = (resume && CX->resume_lo) ? *CX->resume_lo : 0u;
    if (resume && (CX->wrange ? blockIdx.x >= *CX->n_waves : (uint64_t)blockIdx.x * nlw + rlo >= *CX->resume_n)) return;
    uint64_t gidx = (uint64_t)blockIdx.x * nlw + lane + rlo;
    bool live = lane < nlw && (resume ? gidx < *CX->resume_n : gidx < CX->n);
    if (resume && CX->wrange) {   // packed resume: this wave's same-pc run of survivors
        const uint32_t b = blockIdx.x;
        const bool have = b < *CX->n_waves;
        const uint32_t ws = have ? CX->wrange[2 * b] : 0u, we = have ? CX->wrange[2 * b + 1] : 0u;
        gidx = (uint64_t)ws + lane;
        live = gidx < we;
    }
    const uint64_t slot = live ? (resume ? CX->resume[gidx] : gidx) : (uint64_t)CX->n_slots + lane;
    fi_site s;
    s.inst = kNone; s.mask = 0; s.addr = 0; s.target = 0; s.trial = 0;
    uint32_t sidx = 0;
    bool fw_dead = false;
    if (live && !CX->record) {
        sidx = CX->perm[slot]; s = CX->sites[sidx];
        if (CX->eff) {   // first-access forwarding (fi_forward_kernel)
            const uint64_t f = CX->eff[sidx];
            fw_dead = f == kFwDead;
            s.inst = fw_dead ? s.inst : f;
        }
    }

    // ---- start snapshot: the last one at or before the wave's earliest
    // inject time (lane 0 holds it: slots are sorted by inject time)
    uint32_t j = 0;
    if (!resume && !CX->record && CX->snap_start && CX->n_snap > 1) {
        const uint32_t i0 = CX->perm[(uint64_t)blockIdx.x * nlw];
        const uint64_t e0 = CX->eff ? CX->eff[i0] : CX->sites[i0].inst;
        const uint64_t t0 = uni64(e0 == kFwDead ? 0 : e0);
        const uint64_t k = t0 / CX->snap_interval;
        j = (uint32_t)(k < CX->n_snap ? k : CX->n_snap - 1);
    }
    const LaneSave *SV = CX->save + slot;
    if (resume) j = live ? SV->snap_j : 0;
    const SnapState *S0 = CX->snaps + j;
    WaveMem w;   // per lane: resumed lanes come from different start snapshots
    w.tab = CX->snap_tab + S0->tab_off;
    w.tab_n = S0->tab_n;
    if (resume) {
#pragma unroll
        for (int r = 0; r < 32; r++) RREG(r) = live ? SV->regs[r] : 0;
    } else {
#pragma unroll
        for (int r = 0; r < 32; r++) RREG(r) = S0->regs[r];
    }
    RREG(kSinkRow) = 0;

    Lane L;
    L.pc = S0->pc; L.ninst = S0->ninst; L.ncyc = S0->ncyc; L.out_pos = S0->out_pos; L.err_pos = S0->err_pos;
    L.fetch_b = L.data_b = 0;
    L.next_chk = kNone;
    L.nfail = 0;
    L.watch = -1; L.out_bad = false; L.fp = false; L.done = !live; L.injected = (CX->record || !live) ? 1 : 0;
    L.fflags = L.frm = 0;
    L.res.cls = 0; L.res.sub = 0; L.res.exit_code = 0; L.res.flags = 0; L.res.detail = 0; L.res.ninst = 0;
    // the solo kernel's LaneMem lives in LDS: the out-of-line helpers take it
    // by reference, which would otherwise pin it in scratch, and every TLB
    // probe and dirty-range check of the hot loops would be a scratch load
    __shared__ LaneMem m_lds[1];
    LaneMem m_priv;
    LaneMem &m = kNL == 1 ? m_lds[0] : m_priv;
    m.stack_min = S0->stack_min;
    tlb_flush(m);
    m.tp0 = m.tp1 = m.tp2 = m.tp3 = 0;
    m.tnext = 0; m.n_priv = 0; m.req_vpn = kNone; m.req_src = nullptr; m.code_dirty = false;
    m.dlo = m.dhi = 0;
    m.resv = m.lock = kNone;
    m.vm = false;
    m.vcfg = 0;
    m.nmiss = 0;
    if (CX->ov_blocks && live && !resume) CX->ov_of[slot] = 0xFFFFFFFFu;   // no overflow block yet
    // the solo kernel's LDS copy of the slot's rewritten-code map
    __shared__ uint32_t DMAP[kNL == 1 ? kDmapWords : 1];
    m.dl = (kNL == 1 && CX->dmap) ? DMAP : nullptr;
    if (m.dl)
        for (uint32_t i = 0; i < CX->dmap_words; i++) m.dl[i] = 0;
    if (CX->fp0 && live && !resume) {   // a checkpoint with FP state: every lane starts with it
        for (int r = 0; r < 32; r++) CX->fregs[(uint64_t)r * CX->n_slots + slot] = CX->fp0[r];
        L.fp = true;
        L.fflags = (uint8_t)(CX->fcsr0 & 0x1F); L.frm = (uint8_t)((CX->fcsr0 >> 5) & 7);
        if (CX->record) CX->stats[22] = 1;   // FP state outside the snapshots (host disables snapshot starts)
    }
    if (resume && live) {
        L.pc = SV->pc; L.ninst = SV->ninst; L.ncyc = SV->ncyc; L.out_pos = SV->out_pos; L.err_pos = SV->err_pos;
        L.next_chk = SV->next_chk; L.nfail = SV->nfail; L.watch = SV->watch;
        L.out_bad = SV->flags & 1; L.injected = (uint8_t)((SV->flags >> 1) & 3); L.fp = (SV->flags >> 4) & 1;
        L.fflags = (uint8_t)(SV->pad & 0x1F); L.frm = (uint8_t)((SV->pad >> 5) & 7);
        m.vcfg = SV->pad >> 8;
        m.stack_min = SV->stack_min; m.n_priv = SV->n_priv; m.code_dirty = (SV->flags >> 3) & 1;
        m.dlo = CX->code_lo + SV->dlo; m.dhi = CX->code_lo + SV->dhi;
        m.resv = SV->resv; m.lock = SV->lock;
        m.vm = (SV->flags >> 5) & 1;
        if (m.dl && m.code_dirty)
            for (uint32_t i = 0; i < CX->dmap_words; i++) m.dl[i] = CX->dmap[slot * CX->dmap_words + i];
    }
    if (CX->stdin_data && live && !resume) CX->in_pos[slot] = S0->in_pos;
    if (fw_dead && !resume) {   // dead at injection: the trial is the golden run
        L.injected = 1;
        finish(L, FI_MASKED, (int)CX->gsub, (int)CX->gexit, CX->gdetail);
        L.res.ninst = CX->gninst;
        if (kSoloOnce) atomicAdd(&CX->stats[27], 1ull);
    }
    bool suspended = false;
    const uint64_t start_inst = (live && !resume) ? L.ninst : 0;
    const uint64_t launch_inst = live ? L.ninst : 0;   // executed instructions = L.ninst - this at the end
    uint64_t proved_skip = 0;                           // ... less those a proved hang or crash skipped
    bool no_proof = false;                              // a loop proof came out undecided: no more
    uint64_t pages_made = 0;
    uint64_t next_snap = (CX->record && CX->rec_interval) ? 0 : kNone;   // record mode: capture points
    uint32_t snaps_taken = 0;
    uint32_t tpos = 0;   // record mode: golden trace events so far (uniform)
#ifdef FI_PROF
    uint64_t pacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t plast = __builtin_amdgcn_s_memtime();
#endif
    uint32_t n_iter = 0;   // per-wave loop iterations (uniform)
    // solo: a lane whose translated runs keep ending after a few instructions
    // (its loop holds rewritten code, so every block exit writes back and
    // reloads the register file) stays in the pre-decoded path for a while
    uint32_t tx_short = 0, tx_skip_until = 0, tx_skip_n = FI_TX_SKIP_CLEAN;
    // per-wave diagnostic counters live in LDS, not SGPRs (the loop's scalar
    // registers are scarce): slow fetches, min-PC reductions, lane-instructions,
    // snapshot checks, early exits, translated instructions and entries.  Every
    // lane writes the same (uniform) value.
    __shared__ uint32_t WS[8];
#pragma unroll
    for (int k = 0; k < 8; k++) WS[k] = 0;
    // solo only: decode cache of the lane's rewritten code (code range, keyed by
    // exact pc).  Every store into the code range goes through mem_access (the
    // pre-decoded and translated paths refuse them), which drops the entries
    // it overlaps, so a hit equals a fresh fetch + decode.
    constexpr uint32_t kDC = kNL == 1 ? 64u : 1u;
    __shared__ uint32_t DCT[kDC];   // tag: pc - text_lo (0xFFFFFFFF empty)
    __shared__ alignas(16) Pre4 DCE[kDC];
    // ... and the entry cache of solo_fast_run between its calls: per lane of
    // its VGPR cache a 16-byte record {tag = text offset, y, z, w}
    __shared__ alignas(16) uint32_t LC[kNL == 1 ? 4 * kSoloDC : 4];
    if constexpr (kNL == 1) {
#pragma unroll 8
        for (uint32_t k = 0; k < kDC; k++) DCT[k] = 0xFFFFFFFFu;
#pragma unroll 8
        for (uint32_t k = 0; k < kSoloDC; k++) LC[4 * k] = 0xFFFFFFFFu;
    }
    // solo only: the dynamic loop proof's state (LoopProbe)
    __shared__ alignas(8) uint32_t LPB[kNL == 1 ? (sizeof(LoopProbe) + 3) / 4 : 2];
    LoopProbe &LP = *(LoopProbe *)LPB;
    if constexpr (kNL == 1) {
        LP.on = 0; LP.cnt = 0; LP.at = FI_LP_START;
    }
    // (a constant false in the 64-lane kernel)
#define LP_ON (kNL == 1 && LP.on != 0)
// (eligibility for a loop probe: injected, no watched register, live)
#define LP_ELIGIBLE (!L.done && (L.injected == 1 || L.injected == 2) && L.watch <= 0)
#define DC_INVAL(lo_, sz_)                                                                          \
    do {                                                                                            \
        if constexpr (kNL == 1) {                                                                   \
            const uint64_t a_ = (lo_), e_ = a_ + (sz_);                                             \
            if (a_ < CX->code_hi && e_ > CX->code_lo)                                               \
                for (uint64_t q_ = (a_ > 3 ? a_ - 3 : 0); q_ < e_; q_++) {                          \
                    const uint32_t i_ = (uint32_t)(q_ >> 1) & (kDC - 1);                            \
                    if (DCT[i_] == (uint32_t)(q_ - CX->text_lo)) DCT[i_] = 0xFFFFFFFFu;             \
                    if (LC[4 * i_] == (uint32_t)(q_ - CX->text_lo)) LC[4 * i_] = 0xFFFFFFFFu;       \
                }                                                                                   \
        }                                                                                           \
    } while (0)
#define n_slow WS[0]
#define n_min WS[1]
#define n_exec WS[2]
#define n_chk WS[3]
#define n_early WS[4]
#define n_tx WS[5]
#define n_txin WS[6]
#define n_simt WS[7]

    bool prio_up = false;
    for (;;) {
        // ---- solo: a trial that has run long in this dispatch takes issue
        // priority over the short ones sharing its SIMD (the dispatch ends
        // with the longest trials; the short ones are not on the critical path)
        if constexpr (kNL == 1) {
            if (!prio_up && L.ninst - launch_inst >= kSoloPrioInsts) {
                __builtin_amdgcn_s_setprio(3);
                prio_up = true;
            }
        }
        // ---- epochs: after wave_budget iterations the wave suspends its live
        // lanes (a pending copy-on-write is dropped: its tick simply retries)
        if (CX->wave_budget && n_iter >= CX->wave_budget) {
            if (!L.done) {
                LaneSave *sv = CX->save + slot;
#pragma unroll
                for (int r = 0; r < 32; r++) sv->regs[r] = RREG(r);
                sv->pc = L.pc; sv->ninst = L.ninst; sv->ncyc = L.ncyc; sv->out_pos = L.out_pos; sv->err_pos = L.err_pos;
                sv->stack_min = m.stack_min; sv->next_chk = L.next_chk; sv->watch = L.watch; sv->nfail = L.nfail;
                sv->n_priv = m.n_priv; sv->snap_j = j;
                sv->dlo = m.code_dirty ? (uint32_t)(m.dlo > CX->code_lo ? m.dlo - CX->code_lo : 0) : 0;
                sv->dhi = m.code_dirty ? (uint32_t)((m.dhi < CX->code_hi ? m.dhi : CX->code_hi) - CX->code_lo) : 0;
                sv->flags = (L.out_bad ? 1u : 0u) | ((uint32_t)L.injected << 1) | (m.code_dirty ? 8u : 0u) |
                            (L.fp ? 16u : 0u) | (m.vm ? 32u : 0u);
                sv->resv = m.resv; sv->lock = m.lock;
                sv->pad = (uint32_t)L.fflags | ((uint32_t)L.frm << 5) | (m.vcfg << 8);
                if (m.dl && m.code_dirty)   // the solo kernel's map lives in LDS
                    for (uint32_t i = 0; i < CX->dmap_words; i++) CX->dmap[slot * CX->dmap_words + i] = m.dl[i];
                if (kSoloOnce) CX->surv[atomicAdd(CX->surv_n, 1u)] = (uint32_t)slot;
                suspended = true;
                L.done = true;
            }
            break;
        }
        // ---- A. materialise requested pages, whole wave cooperating
        if (wballot<kNL>(!L.done && m.req_vpn != kNone)) {
            // (a lane past its P pages takes its overflow block first: priv_room)
            const bool room = !L.done && m.req_vpn != kNone && priv_room(CX, slot, m.n_priv);
            uint64_t wl = wballot<kNL>(room);
            // (priv_room may have handed a lane its overflow block, ov_of[slot] in
            // global memory, which the other lanes read back in priv_frame below)
            if (wl) __threadfence_block();
            while (wl) {
                const int l = __ffsll((unsigned long long)wl) - 1;
                wl &= wl - 1;
                const uint32_t np = (uint32_t)rdl32<kNL>((uint32_t)m.n_priv, l);
                const uint64_t lslot = rdl64<kNL>(slot, l);
                const uint4 *src = (const uint4 *)rdl64<kNL>((uint64_t)m.req_src, l);
                page_copy<kNL>((uint4 *)priv_frame(CX, lslot, np), src, lane);
            }
            __syncthreads();
            if (!L.done && m.req_vpn != kNone) {
                if (!room) {
                    finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, (uint32_t)L.pc);
                } else {
                    priv_ent(CX, slot, m.n_priv) = m.req_vpn;
                    m.n_priv++;
                    pages_made++;
                }
                m.req_vpn = kNone;
                tlb_flush(m);
            }
        }
        // ---- B. tick-top events: fault injection and the max-insts (hang)
        // exit both fire in serviceInstCountEvents at the first tick with
        // numInst >= n (src/cpu/simple/base.cc:321-325, src/cpu/base.cc:764-770)
        if (!L.done && !L.injected && L.ninst >= s.inst) {
            if (s.target >= 1 && s.target <= 31) {
                RREG(s.target) ^= s.mask;
                if ((CX->protect_mask >> s.target) & 1) L.watch = (int)s.target;
                L.injected = 1;
            } else if (s.target == FI_T_PC) {
                L.pc ^= s.mask;
                L.injected = 1;
                if ((CX->protect_mask >> 32) & 1) finish(L, FI_DETECTED, 0, 0, (uint32_t)L.pc);
            } else if (s.target == FI_T_RESULT) {
                L.injected = 3;   // armed: the next instruction that commits (general path) is the target
            } else if (s.target == FI_T_MEM) {
                uint64_t p;
                OOL(p = lookup(CX, wc_, mc_, slot, s.addr >> 12));
                if (!p) {
                    L.injected = 2;    // page not mapped at t: nothing to flip
                    if (CX->mem_live) {   // ... so the trial is the golden run
                        finish(L, FI_MASKED, (int)CX->gsub, (int)CX->gexit, CX->gdetail);
                        L.res.ninst = CX->gninst;
                        if (kSoloOnce) atomicAdd(&CX->stats[26], 1ull);
                    }
                } else if (CX->mem_live && mem_dead(CX, s.addr, s.mask, L.ninst)) {
                    L.injected = 1;
                    finish(L, FI_MASKED, (int)CX->gsub, (int)CX->gexit, CX->gdetail);
                    L.res.ninst = CX->gninst;
                    if (kSoloOnce) atomicAdd(&CX->stats[26], 1ull);
                } else if (!(p & 1)) {
                    m.req_vpn = s.addr >> 12; m.req_src = page_of(p);   // copy-on-write first, flip next iteration
                } else {
                    uint64_t *wp = (uint64_t *)(const_cast<uint8_t *>(page_of(p)) + (s.addr & 4095));
                    *wp ^= s.mask;
                    if (s.addr < CX->code_hi && s.addr + 8 > CX->code_lo) mark_dirty(CX, m, slot, s.addr, s.addr + 8);
                    DC_INVAL(s.addr, 8);
                    L.injected = 1;
                }
            } else {
                L.injected = 1;
            }
            if (L.injected && CX->early_exit) {
                const uint64_t k = L.ninst / CX->snap_interval + 1;
                L.next_chk = k < CX->n_snap ? k * CX->snap_interval : kNone;
            }
        }
        // (a hang's record names no pc: a proved hang, below, ends before the cap)
        if (!L.done && L.ninst >= CX->hang_cap) finish(L, FI_HANG, 1, 0, 0u);

        // ---- B'. golden comparator at snapshot boundaries (exact early exit)
        if (CX->early_exit) {
            uint64_t pend = wballot<kNL>(!L.done && m.req_vpn == kNone && L.ninst == L.next_chk);
            if (pend) __syncthreads();   // the lanes' own stores are complete before others read them
            while (pend) {
                const int ld = __ffsll((unsigned long long)pend) - 1;
                const uint64_t kn = uni64(rdl64<kNL>(L.ninst, ld));
                const bool grp = !L.done && m.req_vpn == kNone && L.ninst == L.next_chk && L.ninst == kn;
                pend &= ~wballot<kNL>(grp);
                const SnapState *S = CX->snaps + (uint32_t)(kn / CX->snap_interval);
                // (with wrong output so far, bit 1: the trial can only go on as the
                // golden run does from here, so it ends as SDC with the golden exit)
                bool eq = grp && L.pc == S->pc && L.out_pos == S->out_pos && L.err_pos == S->err_pos &&
                          (!L.out_bad || (CX->early_exit & 2)) &&
                          m.stack_min == S->stack_min && !L.fp && L.injected != 3 && m.resv == kNone &&
                          m.lock == kNone && !m.vm && !m.vcfg &&
                          // the golden suffix reads curTick: the same future needs the same tick count
                          // too (a path with other non-counting ticks -- ecalls, straddled fetches --
                          // reconverges with the same numInst but would print another time)
                          (kn >= CX->clk_until || L.ncyc == S->ncyc) &&
                          (!CX->stdin_data || CX->in_pos[slot] == S->in_pos);
                if (wballot<kNL>(eq)) {
                    // a register the golden future writes before reading it cannot
                    // influence the outcome (liveness from the golden trace)
                    const uint32_t lv = S->live;
#pragma unroll
                    for (int r = 1; r < 32; r++) eq = eq && (RREG(r) == S->regs[r] || !((lv >> r) & 1));
                }
                n_chk += (uint32_t)__popcll(wballot<kNL>(grp));
                uint64_t mm = wballot<kNL>(eq);
                while (mm) {
                    const int l = __ffsll((unsigned long long)mm) - 1;
                    mm &= mm - 1;
                    WaveMem wl;
                    wl.tab = (const PageEnt *)rdl64<kNL>((uint64_t)w.tab, l);
                    wl.tab_n = (uint32_t)rdl32<kNL>((uint32_t)w.tab_n, l);
                    const bool same = lane_mem_equal<kNL>(CX, wl, rdl64<kNL>(slot, l),
                                                     (uint32_t)rdl32<kNL>((uint32_t)m.n_priv, l), S, lane);
                    if ((int)lane == l) eq = same;
                }
                if (grp) {
                    if (eq) {
                        finish(L, L.out_bad ? FI_SDC : FI_MASKED, (int)CX->gsub, (int)CX->gexit, CX->gdetail);
                        L.res.ninst = CX->gninst;
                    } else {
                        // back off after repeated mismatches (any schedule is exact)
                        const uint32_t sh = L.nfail < 4 ? 0 : (L.nfail < 7 ? L.nfail - 3 : 4);
                        L.nfail++;
                        const uint64_t nx = L.next_chk + (CX->snap_interval << sh);
                        L.next_chk = nx / CX->snap_interval < CX->n_snap ? nx : kNone;
                    }
                }
                n_early += (uint32_t)__popcll(wballot<kNL>(grp && eq));
            }
        }

        // ---- B''. record mode: capture a golden snapshot (one live lane)
        if (CX->record && uni64(rdl64<kNL>(L.ninst, 0)) == next_snap && !rdl32<kNL>((uint32_t)L.done, 0)) {
            if (snaps_taken < CX->rec_max_snaps) {
                SnapState *S = CX->rec_snaps + snaps_taken;
                const uint32_t np = (uint32_t)rdl32<kNL>((uint32_t)m.n_priv, 0);
                if (lane == 0) {
#pragma unroll
                    for (int r = 0; r < 32; r++) S->regs[r] = RREG(r);
                    S->pc = L.pc; S->ninst = L.ninst; S->ncyc = L.ncyc; S->out_pos = L.out_pos; S->err_pos = L.err_pos;
                    S->stack_min = m.stack_min; S->tab_off = 0; S->tab_n = np;
                    S->live = 0; S->trace_pos = tpos;
                    S->in_pos = CX->stdin_data ? CX->in_pos[0] : 0;
                }
                for (uint32_t i = 0; i < np; i++) {
                    if (lane == 0) CX->rec_vpns[(uint64_t)snaps_taken * CX->priv_pages + i] = CX->priv_vpn[i * CX->n_slots];
                    const uint4 *src = (const uint4 *)priv_frame(CX, 0, i);
                    page_copy<kNL>((uint4 *)(CX->rec_pages + (((uint64_t)snaps_taken * CX->priv_pages + i) << 12)), src, lane);
                }
            }
            snaps_taken++;
            next_snap += CX->rec_interval;
        }

#if FI_SOLO_DIRTY_PRIO
        // a solo trial that rewrote its code runs interpreted, ~10x slower per
        // instruction than translated code: the issue arbiter prefers it
        if constexpr (kNL == 1) {
            if (m.code_dirty) __builtin_amdgcn_s_setprio(FI_SOLO_DIRTY_PRIO);
        }
#endif
        const bool ready = !L.done && m.req_vpn == kNone;
        const uint64_t act = wballot<kNL>(ready);
        if (act == 0) {
            if (wballot<kNL>(!L.done) == 0) break;
            continue;
        }
        // ---- C. leader PC: first ready lane, or min-PC if the lanes diverged
        const int leader = __ffsll((unsigned long long)act) - 1;
        uint64_t lpc = rdl64<kNL>(L.pc, leader);
        n_iter++;
        if constexpr (kNL == 1) n_min++;   // solo (no groups to reduce): counts the trips through this loop
        if (wballot<kNL>(ready && L.pc == lpc) != act) { lpc = wmin64<kNL>(ready ? L.pc : kNone); n_min++; }
        lpc = uni64(lpc);   // wave-uniform: keeps fetch/decode/dispatch on the scalar unit
        bool mine = ready && L.pc == lpc;
        // lanes of other groups wait; the group keeps the wave only while its PC
        // stays below theirs (min-PC order, so groups merge when they meet)
        const uint64_t wait_min = (wballot<kNL>(mine) != act) ? uni64(wmin64<kNL>((ready && !mine) ? L.pc : kNone)) : kNone;
        // next instruction-count event of this lane: injection, snapshot
        // comparison, hang cap, or (record mode) snapshot capture
        uint64_t next_ev = CX->hang_cap;
        if (!L.injected) next_ev = s.inst < next_ev ? s.inst : next_ev;
        if (L.next_chk < next_ev) next_ev = L.next_chk;
        if (next_snap < next_ev) next_ev = next_snap;

        // ---- DIVERGED LANES (64-lane kernel): when the ready
        // lanes sit at different pcs, every one of them on unmodified golden
        // text executes its own pre-decoded micro-op -- per-lane entry,
        // registers, TLB and pages, a divergent switch over the ~30 kinds --
        // instead of one pc group at a time.  A lane stops at anything else
        // (K_SLOW ops, faults, misses lookup_full cannot resolve, copy-on-write,
        // stores into the code range, page-crossing accesses, odd pcs, its next
        // instruction-count event, a watched register or an armed result fault,
        // an LR/SC lock record) and the group machinery below serves it.  The
        // step loop runs while at least half of the lanes it started with
        // commit.  Same counters as the fast path, per lane.
        if constexpr (kNL > 1) {
            if (CX->simt_min && !CX->record && CX->pre_ok && wait_min != kNone) {
                const uint64_t lim = (ready && L.watch <= 0 && L.injected != 3 && m.lock == kNone && next_ev > L.ninst)
                                         ? next_ev - L.ninst : 0;
                bool run = lim != 0;
                const uint32_t n0 = (uint32_t)__popcll(wballot<kNL>(run));
                if (n0 >= CX->simt_min) {
                    uint64_t pc = L.pc;
                    uint32_t lst = 0, lxt = 0, lfb = 0, ldb = 0;   // per lane: insts, straddles, fetch/data bytes
                    uint32_t wst = 0, nex = 0;                     // wave steps, lane-instructions
                    const uint32_t wbud = uni32(CX->wave_budget ? CX->wave_budget - n_iter : (1u << 30));
                    const uint64_t tlo = CX->text_lo, clo = CX->code_lo, chi = CX->code_hi;
                    const uint32_t tby = CX->text_bytes;
                    const uint4 *const pre4 = (const uint4 *)CX->pre;
                    for (;;) {
                        const uint64_t toff = pc - tlo;
                        bool go = run && toff < tby && !(pc & 1) && !dirty_at(CX, m, pc);
                        uint4 e = make_uint4(0u, 0u, 0u, 0u);
                        if (go) e = pre4[toff >> 1];
                        const uint32_t aux = e.w >> 16, kind = aux & 63, pf = (e.w >> 8) & 0xFF;
                        go = go && (pf & kPreValid) && kind != K_SLOW;
                        const uint32_t rd = (e.y >> 8) & 0xFF, rs1 = (e.y >> 16) & 0xFF, rs2 = e.y >> 24;
                        const int64_t imm = (int32_t)e.z;
                        const uint32_t len = e.w & 0xFF;
                        const uint64_t ft = pc + len;
                        uint64_t v = 0, npc = ft;
                        uint32_t msz = 0;
                        bool wr = true;
                        if (go) {
                            const uint64_t a0 = RREG(rs1), b0 = RREG(rs2);
                            const uint64_t av = (aux & U_APC) ? pc : a0;
                            const uint64_t bv = (aux & U_BIMM) ? (uint64_t)imm : b0;
                            const bool w32 = aux & U_W32;
                            const uint32_t shm = w32 ? 31 : 63;
                            switch (kind) {
                            case K_ADD: v = av + bv; break;
                            case K_SUB: v = av - bv; break;
                            case K_AND: v = av & bv; break;
                            case K_OR: v = av | bv; break;
                            case K_XOR: v = av ^ bv; break;
                            case K_SLT: v = (int64_t)av < (int64_t)bv ? 1 : 0; break;
                            case K_SLTU: v = av < bv ? 1 : 0; break;
                            case K_SLL: v = av << (bv & shm); break;
                            case K_SRL: v = (w32 ? (av & 0xFFFFFFFFULL) : av) >> (bv & shm); break;
                            case K_SRA: v = (uint64_t)((w32 ? (int64_t)(int32_t)av : (int64_t)av) >> (bv & shm)); break;
                            case K_MUL: v = av * bv; break;
                            case K_MULH: v = (uint64_t)__mul64hi((int64_t)av, (int64_t)bv); break;
                            case K_MULHU: v = __umul64hi(av, bv); break;
                            case K_MULHSU: v = __umul64hi(av, bv) - (((int64_t)av < 0) ? bv : 0); break;
                            case K_DIV: v = w32 ? divw(av, bv) : div64(av, bv); break;
                            case K_DIVU:
                                v = w32 ? ((uint32_t)bv == 0 ? ~0ULL : sx32((uint32_t)av / (uint32_t)bv))
                                        : (bv == 0 ? ~0ULL : av / bv);
                                break;
                            case K_REM: v = w32 ? remw(av, bv) : rem64(av, bv); break;
                            case K_REMU:
                                v = w32 ? ((uint32_t)bv == 0 ? sx32(av) : sx32((uint32_t)av % (uint32_t)bv))
                                        : (bv == 0 ? av : av % bv);
                                break;
                            case K_NOP: wr = false; break;
                            case K_JAL: v = ft; npc = pc + imm; break;
                            case K_JALR: v = ft; npc = (a0 + imm) & ~1ULL; break;
                            case K_BEQ: wr = false; npc = a0 == b0 ? pc + imm : ft; break;
                            case K_BNE: wr = false; npc = a0 != b0 ? pc + imm : ft; break;
                            case K_BLT: wr = false; npc = (int64_t)a0 < (int64_t)b0 ? pc + imm : ft; break;
                            case K_BGE: wr = false; npc = (int64_t)a0 >= (int64_t)b0 ? pc + imm : ft; break;
                            case K_BLTU: wr = false; npc = a0 < b0 ? pc + imm : ft; break;
                            case K_BGEU: wr = false; npc = a0 >= b0 ? pc + imm : ft; break;
                            default: {   // K_LOAD / K_STORE inside one mapped page
                                const bool st = kind == K_STORE;
                                msz = 1u << ((aux >> 12) & 3);
                                const uint64_t ea = a0 + imm;
                                const uint32_t off = (uint32_t)(ea & 4095);
                                uint64_t p = tlb_find(m, ea >> 12);
                                if (!p) OOL(p = lookup_full(CX, wc_, mc_, slot, ea >> 12));
                                const bool code_st = st && !(ea >= chi || ea + msz <= clo);
                                if (!(p && (!st || ((p & 1) && !code_st)) && off + msz <= 4096)) { go = false; break; }
                                uint8_t *pg = const_cast<uint8_t *>(page_of(p));
                                const bool al = (off & (msz - 1)) == 0;
                                if (st) {
                                    wr = false;
                                    if (al) {
                                        switch (msz) {
                                        case 1: pg[off] = (uint8_t)b0; break;
                                        case 2: *(uint16_t *)(pg + off) = (uint16_t)b0; break;
                                        case 4: *(uint32_t *)(pg + off) = (uint32_t)b0; break;
                                        default: *(uint64_t *)(pg + off) = b0; break;
                                        }
                                    } else {
                                        for (uint32_t i = 0; i < msz; i++) pg[off + i] = (uint8_t)(b0 >> (8 * i));
                                    }
                                } else {
                                    uint64_t t = 0;
                                    if (al) {
                                        switch (msz) {
                                        case 1: t = pg[off]; break;
                                        case 2: t = *(const uint16_t *)(pg + off); break;
                                        case 4: t = *(const uint32_t *)(pg + off); break;
                                        default: t = *(const uint64_t *)(pg + off); break;
                                        }
                                    } else {
                                        for (uint32_t i = 0; i < msz; i++) t |= (uint64_t)pg[off + i] << (8 * i);
                                    }
                                    v = (aux & U_SEXT) ? (uint64_t)sext64(t, 8 * msz) : t;
                                }
                                break;
                            }
                            }
                            if (go) {
                                if (w32) v = sx32(v);
                                RREG((wr && rd) ? rd : kSinkRow) = v;
                                pc = npc;
                                lst++; lxt += (pf & kPreStraddle) ? 1 : 0; lfb += len; ldb += msz;
                            }
                        }
                        run = go && lst < lim;   // a lane that stopped stays stopped in this loop
                        const uint32_t na = (uint32_t)__popcll(wballot<kNL>(go));
                        wst++;
                        nex += na;
                        if (2 * na < n0 || wballot<kNL>(run) == 0 || wst >= wbud) break;
                    }
                    if (lst) { L.pc = pc; L.ninst += lst; L.ncyc += lst + lxt; L.fetch_b += lfb; L.data_b += ldb; }
                    n_iter += wst;
                    n_exec += nex;
                    n_simt += nex;
                    if (nex) continue;
                }
            }
        }

#ifdef FI_TX
        // ---- TRANSLATED PATH (load-time build only): the golden run's basic
        // blocks compiled to straight-line code with the guest registers in
        // VGPRs.  Entered at a block leader by a converged group
        // with nothing watched or modified.  Divergence is handled inside, by
        // the same min-PC rule as the interpreter: at a divergent branch the
        // lanes bound for the higher pc park (lp) and the others run on; a
        // block entered at or past the lowest parked pc merges or switches
        // groups (tx_sched).  Everything runs in uniform control flow with
        // every lane active: register writes are selects on `mine`, lanes
        // outside the running group read the zero page and store to a sink.
        // It leaves (tx_out) at anything the blocks do not cover (events,
        // faults, copy-on-write, syscalls, TLB misses, divergent jalr,
        // untranslated pcs, lanes outside the entry group), every counter
        // exact and per lane.
        if (!CX->record) {
            TextRef tx;
            tx.pre = CX->pre; tx.lo = (uint32_t)CX->text_lo; tx.hi = (uint32_t)(CX->text_lo >> 32);
            tx.bytes = CX->text_bytes; tx.clo = CX->code_lo; tx.chi = CX->code_hi;
            const PreRef E0 = pre_entry(tx, lpc);
            // (odd pcs: the solo-odd body's odd-pc blocks, flagged on their key's entry)
            const bool tx_entry = E0.in && ((lpc & 1) ? (kOdd && ((uni32(E0.e.w) >> 8) & kPreOddLeader))
                                                      : ((uni32(E0.e.w) >> 8) & kPreLeader));
            if constexpr (kNL == 1) {
                // ---- solo: one trial, every value uniform -- no groups, no
                // parking, plain register writes; the same exits and counters
                if (tx_entry && mine && n_iter >= tx_skip_until && L.injected != 3 && m.lock == kNone && !LP_ON) {
                    const uint64_t rem64 = next_ev - L.ninst;
                    const uint32_t rem = rem64 > (1u << 30) ? (1u << 30) : (uint32_t)rem64;
                    const uint32_t wbud = CX->wave_budget ? CX->wave_budget - n_iter : (1u << 30);
                    uint32_t bud = rem < wbud ? rem : wbud;
                    // odd-pc streams: a trial past the golden run's length can only
                    // end by a crash or at the hang cap, and the static proofs do
                    // not cover these streams -- its translated instructions count
                    // toward a loop probe, and a call returns at the golden length and
                    // when the probe is due (qsort's odd-pc hangs ran 228k translated
                    // instructions to the cap)
                    if (kOdd && CX->hang_proof && LP_ELIGIBLE) {
                        const uint32_t due = L.ninst < CX->gninst
                                                 ? (uint32_t)(CX->gninst - L.ninst + 1 < bud ? CX->gninst - L.ninst + 1 : bud)
                                                 : (LP.at > LP.cnt ? LP.at - LP.cnt : 1u);
                        bud = due < bud ? due : bud;
                    }
                    // rewritten code bytes as offsets from the text base (empty range if none)
                    const uint64_t tlo = CX->text_lo;
                    __shared__ SoloTxIO sio[1];
                    sio->spc = lpc; sio->bud = bud; sio->lwm = L.watch > 0 ? (1u << L.watch) : 0u;
                    {
                        const uint64_t hl = CX->hang_cap - L.ninst;
                        sio->hleft = hl > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)hl;
                        sio->hok = CX->hang_proof && !no_proof && (L.injected == 1 || L.injected == 2) ? 1u : 0u;
                    }
                    sio->sdlo = m.code_dirty ? (uint32_t)((m.dlo > tlo ? m.dlo : tlo) - tlo) : 0xFFFFFFFFu;
                    sio->sdhi = m.code_dirty ? (uint32_t)((m.dhi > tlo ? m.dhi : tlo) - tlo) : 0u;
                    if (!kOdd && !m.code_dirty && L.watch <= 0)
                        solo_tx_clean_run(CX, (lds_u64 *)R, (lds_mem *)&m, (lds_io *)sio);
                    else
                        solo_tx_run<kOdd>(CX, (lds_u64 *)R, (lds_mem *)&m, (lds_io *)sio);
                    const uint32_t st = uni32(sio->st), xt = uni32(sio->xt), fb = uni32(sio->fb), db = uni32(sio->db);
                    const uint64_t spc = uni64(sio->spc);
                    if (sio->schg) {
                        const uint32_t cslo = uni32(sio->cslo), cshi = uni32(sio->cshi);
#pragma unroll 8
                        for (uint32_t k = 0; k < kDC; k++) {   // decode-cache entries whose bytes were rewritten
                            const uint32_t tg = DCT[k];
                            if (tg != 0xFFFFFFFFu && tg + 4 > cslo && tg < cshi) DCT[k] = 0xFFFFFFFFu;
                            const uint32_t tl = LC[4 * k];
                            if (tl != 0xFFFFFFFFu && tl + 4 > cslo && tl < cshi) LC[4 * k] = 0xFFFFFFFFu;
                        }
                    }
                    L.ninst += st; L.ncyc += st + xt; L.fetch_b += fb; L.data_b += db; L.pc = spc;
                    n_iter += st;
                    n_tx += st;
                    n_txin++;
#if FI_SOLO_AGE
                    // ageing: a solo trial that has run long is likely to run long
                    // still (the campaign's tail); it gets the issue arbiter's
                    // preference over the younger waves of its CU
                    if (n_iter >= (4u << FI_SOLO_AGE)) __builtin_amdgcn_s_setprio(3);
                    else if (n_iter >= (2u << FI_SOLO_AGE)) __builtin_amdgcn_s_setprio(2);
                    else if (n_iter >= (1u << FI_SOLO_AGE)) __builtin_amdgcn_s_setprio(1);
#endif
                    if (kOdd && L.ninst > CX->gninst && !uni32(sio->hang)) {
                        LP.cnt += st;
                        if (LP.cnt >= LP.at) lp_count((lds_lp *)&LP, CX, (const lds_u64 *)R, slot, L.pc, L.fp, LP_ELIGIBLE, 0u);
                    }
                    if (uni32(sio->hang)) {   // a loop that cannot leave before the cap
                        uint64_t kf = 0, fva = 0;
                        const uint64_t left = L.ninst < CX->hang_cap ? CX->hang_cap - L.ninst : 0;
                        // (always: the body proved it against hleft, capped at 2^32 - 1;
                        // loop_outcome re-checks every loop against the 64-bit `left`)
                        const int r = loop_outcome(CX, w, m, slot, (const lds_u64 *)R, (const lds_io *)sio, left, kf,
                                                   fva);
                        if (r == 1) {   // a proved hang: the record of one that ran to the cap
                            proved_skip = left;
                            L.ninst += left;
                            finish(L, FI_HANG, 1, 0, 0u);
                            atomicAdd(&CX->stats[56], 1ull);
                        } else if (r == 2) {   // a proved page fault kf instructions on
                            proved_skip = kf;
                            L.ninst += kf;
                            finish(L, FI_CRASH, FI_CRASH_PAGE_FAULT, 134, (uint32_t)fva);
                            atomicAdd(&CX->stats[57], 1ull);
                        } else {   // undecided: the trial runs on, without asking again
                            no_proof = true;
                            atomicAdd(&CX->stats[58], 1ull);
                        }
                        continue;
                    }
                    // thrash guard: runs that keep ending after a few instructions
                    // (a loop entered mid-block, e.g. a return into its own
                    // epilogue, leaves at every dispatch) cost a round trip each;
                    // the interpreter takes the next FI_TX_SKIP (rewritten code)
                    // or tx_skip_n instructions, doubling while it recurs
                    if (m.code_dirty ? st < FI_TX_SHORT : st < FI_TX_SHORT_CLEAN) {
                        if (++tx_short >= (m.code_dirty ? 4u : 16u)) {
                            tx_short = 0;
                            tx_skip_until = n_iter + (m.code_dirty ? FI_TX_SKIP : tx_skip_n);
                            tx_skip_n = tx_skip_n < (1u << 20) ? 2 * tx_skip_n : tx_skip_n;
                        }
                    } else {
                        tx_short = 0;
                        if (st >= 8 * FI_TX_SHORT) tx_skip_n = FI_TX_SKIP_CLEAN;
                    }
                    // the clean body tests its budget once per run of blocks: one that
                    // stops at a test with nothing run leaves the rest up to the event
                    // (fewer instructions than the run) to the interpreter
                    if (!st && uni32(sio->bst)) tx_skip_until = n_iter + bud;
                    if (st) continue;
                }
            } else if (tx_entry &&
                       wballot<kNL>(mine && (dirty_near(m, lpc) || L.injected == 3 || m.lock != kNone)) == 0) {
                // lanes that rewrote code: every block checks its bytes against their range
                const bool wdirty = uni32(wballot<kNL>(m.code_dirty) != 0);
                const uint64_t ldlo = m.code_dirty ? m.dlo : kNone, ldhi = m.code_dirty ? m.dhi : 0;
                // lanes watching a protected flipped register: blocks that touch it exit first
                const bool wwatch = uni32(wballot<kNL>(L.watch > 0) != 0);
                const uint32_t lwm = L.watch > 0 ? (1u << L.watch) : 0u;
                const uint64_t gm = wballot<kNL>(mine);      // the entry group
                uint64_t gmr = gm;                        // the running group
                uint64_t pend = 0, pmin = kNone;          // parked lanes, their lowest pc
                const uint64_t owm = wait_min;            // lanes outside the entry group
                uint64_t wmin = owm;                      // min(pmin, owm)
                const uint64_t rem64 = mine ? next_ev - L.ninst : 0;
                const uint32_t rem = rem64 > (1u << 30) ? (1u << 30) : (uint32_t)rem64;
                // n_iter is uniform in value but not provably so (divergent updates
                // elsewhere in the loop); a divergent bound here would make every
                // branch of the translated code divergent
                const uint32_t wbud = uni32(CX->wave_budget ? CX->wave_budget - n_iter : (1u << 30));
                // scalar lower bound of the budget checks (translated blocks)
                const uint32_t urem = (uint32_t)uni64(wmin64<kNL>(mine ? (uint64_t)rem : kNone));
                const uint32_t ubud = urem < wbud ? urem : wbud;
                const uint8_t *const zp = CX->zero_page;
                uint8_t *const sink = CX->tx_sink + 8 * lane;
                uint32_t lst = 0, lxt = 0, lfb = 0, ldb = 0;   // per lane: insts, straddles, fetch/data bytes
                uint32_t wst = 0;                              // wave iterations
                uint64_t spc = lpc, lp = 0, dpc = 0;
                uint32_t etgt = 0xFFFFFFFFu;   // block an entry is routed to through its cycle headers
                bool jdiv = false;
#define TXR(r) uint64_t X##r = RREG(r);
                TXR(1) TXR(2) TXR(3) TXR(4) TXR(5) TXR(6) TXR(7) TXR(8) TXR(9) TXR(10) TXR(11) TXR(12) TXR(13)
                TXR(14) TXR(15) TXR(16) TXR(17) TXR(18) TXR(19) TXR(20) TXR(21) TXR(22) TXR(23) TXR(24) TXR(25)
                TXR(26) TXR(27) TXR(28) TXR(29) TXR(30) TXR(31)
#undef TXR
// a group parked at pc joins the running group (pc == pmin, lanes outside the
// entry group all wait at higher pcs)
#define TXMERGE(pc)                                                                          \
    do {                                                                                     \
        const bool jn_ = ((pend >> lane) & 1) && lp == (pc);                                 \
        const uint64_t b_ = TXB(jn_);                                                        \
        mine = mine || jn_;                                                                  \
        gmr = uni64(gmr | b_);                                                               \
        pend = uni64(pend & ~b_);                                                            \
        pmin = uni64(pend ? wmin64<kNL>(((pend >> lane) & 1) ? lp : kNone) : kNone);         \
        wmin = uni64(ult64(pmin, owm) ? pmin : owm);                                         \
    } while (0)
                TX_TEMPS();
                goto tx_dispatch;
                /*@TX_BODY@*/
#undef TXMERGE
            tx_sched:   // spc >= wmin: merge with the parked group, switch to it, or leave
                if (!ult64(pmin, owm)) goto tx_out;   // lanes outside run first (or no parked lanes)
                if (spc == pmin) {
                    const bool jn = ((pend >> lane) & 1) && lp == spc;
                    const uint64_t b = TXB(jn);
                    mine = mine || jn;
                    gmr = uni64(gmr | b);
                    pend = uni64(pend & ~b);
                } else {
                    lp = mine ? spc : lp;
                    pend = uni64(pend | gmr);
                    const bool jn = ((pend >> lane) & 1) && lp == pmin;
                    mine = jn;
                    gmr = uni64(TXB(jn));
                    pend = uni64(pend & ~gmr);
                    spc = pmin;
                }
                pmin = uni64(pend ? wmin64<kNL>(((pend >> lane) & 1) ? lp : kNone) : kNone);
                wmin = uni64(ult64(pmin, owm) ? pmin : owm);
                goto tx_dispatch;
            tx_out:
                if ((gm >> lane) & 1) {
#define TXW(r) RREG(r) = X##r;
                    TXW(1) TXW(2) TXW(3) TXW(4) TXW(5) TXW(6) TXW(7) TXW(8) TXW(9) TXW(10) TXW(11) TXW(12) TXW(13)
                    TXW(14) TXW(15) TXW(16) TXW(17) TXW(18) TXW(19) TXW(20) TXW(21) TXW(22) TXW(23) TXW(24) TXW(25)
                    TXW(26) TXW(27) TXW(28) TXW(29) TXW(30) TXW(31)
#undef TXW
                    L.ninst += lst; L.ncyc += lst + lxt; L.fetch_b += lfb; L.data_b += ldb;
                    L.pc = ((pend >> lane) & 1) ? lp : (jdiv ? dpc : spc);
                }
                n_iter += wst;
                n_tx += wst;
                n_txin++;
                if (wst) continue;
            }
        }
#endif

        // ---- FAST PATH: the group is converged on golden text with nothing
        // watched or modified -- run pre-decoded micro-ops with PC, instruction,
        // cycle and byte counts in SGPRs until an event is due, the group
        // diverges, meets another group, or hits something the general path owns
        // (K_SLOW op, fault, page request, syscall).  Nothing commits unless the
        // whole instruction commits for every group lane.
        // (an armed result fault commits in the general path, and a lane holding
        // an LR/SC lock record stays there: only its stores erase the record)
        if (!LP_ON && CX->pre_ok && lpc >= CX->text_lo && lpc < CX->text_hi &&
            wballot<kNL>(mine && (L.injected == 3 || m.lock != kNone)) == 0) {
            // lanes that rewrote code run here too, until they reach a rewritten
            // instruction; lanes watching a protected flipped register, until an
            // instruction reads it (the general path classifies the detection)
            bool any_dirty = wballot<kNL>(mine && m.code_dirty) != 0;
            const bool any_watch = wballot<kNL>(mine && L.watch > 0) != 0;
            const uint64_t gm = wballot<kNL>(mine);
            const int glane = __ffsll((unsigned long long)gm) - 1;
            uint64_t budget64 = uni64(wmin64<kNL>(mine ? next_ev - L.ninst : kNone));
            if (CX->wave_budget && budget64 > CX->wave_budget - n_iter) budget64 = CX->wave_budget - n_iter;
            const uint32_t budget = budget64 > (1u << 30) ? (1u << 30) : (uint32_t)budget64;
            if constexpr (kNL == 1) {
                if (!CX->record) {   // solo: the out-of-line run (solo_pre_run), then the general path
                    __shared__ SoloPreIO pio[1];
                    pio->spc = lpc; pio->slot = slot; pio->tab = w.tab; pio->tab_n = w.tab_n;
                    pio->budget = budget; pio->watch = L.watch;
                    pio->fps = (L.fp ? 1u : 0u) | ((uint32_t)L.fflags << 8) | ((uint32_t)L.frm << 16);
                    pio->tx_gate = tx_skip_until > n_iter ? tx_skip_until - n_iter : 0u;
                    solo_pre_run<kOdd>(CX, (lds_u64 *)R, (lds_mem *)&m, (lds_u32 *)DCT, (lds_pre4 *)DCE, (lds_u32 *)LC,
                                       (lds_pio *)pio);
                    const uint32_t steps = uni32(pio->steps);
#ifdef FI_PROF
                    for (int k = 0; k < 4; k++) pacc[k] += pio->prof[k];
#endif
                    if (steps) {
                        L.ninst += steps; L.ncyc += steps + uni32(pio->xticks);
                        L.fetch_b += uni32(pio->fbytes); L.data_b += uni32(pio->dbytes);
                        L.pc = uni64(pio->spc); L.watch = (int)uni32((uint32_t)pio->watch);
                        const uint32_t fps = uni32(pio->fps);
                        L.fp = fps & 1; L.fflags = (uint8_t)((fps >> 8) & 0x1F);
                        // (interpreted: counts toward a loop probe)
                        LP.cnt += steps;
                        if (LP.cnt >= LP.at) lp_count((lds_lp *)&LP, CX, (const lds_u64 *)R, slot, L.pc, L.fp, LP_ELIGIBLE, 0u);
                        n_iter += steps;
                        n_exec += steps;
                        continue;
                    }
                }
            }
            uint64_t spc = lpc;
            uint32_t steps = 0, xticks = 0, fbytes = 0, dbytes = 0;
            bool div = false;
            TextRef tx;
            tx.pre = CX->pre; tx.lo = (uint32_t)CX->text_lo; tx.hi = (uint32_t)(CX->text_lo >> 32);
            tx.bytes = CX->text_bytes; tx.clo = CX->code_lo; tx.chi = CX->code_hi;
            PreRef E = pre_entry(tx, spc);
            while (budget) {
                PSTAMP(3);
                spc = uni64(spc);
                if (any_dirty && wballot<kNL>(mine && dirty_at(CX, m, spc)) != 0) {
                    // the group rewrote this instruction: decode the bytes the
                    // lanes hold now (Decoder::moreBytes on their own pages) when
                    // they all hold the same; otherwise the general path
                    bool hit = false;
                    const bool in_code = spc >= CX->code_lo && spc < CX->code_hi;
                    if constexpr (kNL == 1) {
                        const uint32_t ci = (uint32_t)(spc >> 1) & (kDC - 1);
                        if (in_code && DCT[ci] == (uint32_t)(spc - CX->text_lo)) { E.e = DCE[ci]; E.in = true; hit = true; }
                    }
                    if (!hit) {
                    uint32_t raw = 0, t = 1;
                    uint64_t fva = 0;
                    int fr = 0;
                    if (mine) OOL(fr = fetch_lane(CX, wc_, mc_, slot, spc, raw, t, fva));
                    const uint32_t raw0 = (uint32_t)rdl32<kNL>((uint32_t)raw, glane);
                    const uint32_t t0 = (uint32_t)rdl32<kNL>((uint32_t)t, glane);
                    if (wballot<kNL>(mine && (fr != 0 || raw != raw0)) != 0) break;
                    Dec dd = rv_decode(uni32(raw0));
                    const uint32_t u = uop_of(dd);
                    E.in = true;
                    E.e.x = dd.raw;
                    E.e.y = (uint32_t)dd.op | ((uint32_t)dd.rd << 8) | ((uint32_t)dd.rs1 << 16) | ((uint32_t)dd.rs2 << 24);
                    E.e.z = (uint32_t)dd.imm;
                    E.e.w = (uint32_t)dd.len |
                            ((uint32_t)(kPreValid | (uni32(t0) == 2 ? kPreStraddle : 0) | dd.flags) << 8) | (u << 16);
                    if constexpr (kNL == 1) {
                        if (in_code) {
                            const uint32_t ci = (uint32_t)(spc >> 1) & (kDC - 1);
                            DCT[ci] = (uint32_t)(spc - CX->text_lo);
                            DCE[ci] = E.e;
                        }
                    }
                    }
                    PSTAMP(5);
                }
                const uint32_t q1 = uni32(E.e.y), q2 = uni32(E.e.z), q3 = uni32(E.e.w);
                const uint32_t aux = q3 >> 16, kind = aux & 63;
                if (!E.in || !((q3 >> 8) & kPreValid) || kind == K_SLOW) break;
#ifdef FI_TX
                // translated blocks take over here (odd pcs: only the solo-odd
                // kernel's odd-pc blocks, flagged on the entry of the halfword they fetch)
                const bool lead = ((uint32_t)spc & 1) ? (kOdd && ((q3 >> 8) & kPreOddLeader)) : ((q3 >> 8) & kPreLeader);
                if (steps && lead && (kNL == 1 || !(any_dirty && wballot<kNL>(mine && dirty_near(m, spc)) != 0)) &&
                    n_iter + steps >= tx_skip_until)
                    break;
#endif
                const uint32_t rd = q1 >> 8 & 0xFF, rs1 = q1 >> 16 & 0xFF, rs2 = q1 >> 24;
                if (any_watch) {
                    const uint32_t fl = q3 >> 8;
                    const bool rw = L.watch > 0 && (((fl & kPreRs1) && rs1 == (uint32_t)L.watch) ||
                                                    ((fl & kPreRs2) && rs2 == (uint32_t)L.watch));
                    if (wballot<kNL>(mine && rw) != 0) break;
                }
                const int64_t imm = (int32_t)q2;
                const uint32_t len = q3 & 0xFF, straddle = ((q3 >> 8) & kPreStraddle) ? 1 : 0;
                const uint64_t a0 = RREG(rs1), b0 = RREG(rs2);
                // prefetch the successors' entries while this instruction executes
                const uint64_t ft = spc + len;
                const PreRef Eft = pre_entry(tx, ft);
                const PreRef Etg = pre_entry(tx, spc + imm);   // unconditional: no phi, no early wait
                const uint64_t av = (aux & U_APC) ? spc : a0;
                const uint64_t bv = (aux & U_BIMM) ? (uint64_t)imm : b0;
#ifdef FI_PROF
                asm volatile("" :: "v"(av), "v"(bv));
                PSTAMP(0);
#endif
                const bool w32 = aux & U_W32;
                const uint32_t shm = w32 ? 31 : 63;
                uint64_t v = 0, npc = ft;
                uint32_t msz = 0;
                bool wr = true, took = false, ind = false;
                switch (kind) {
                case K_ADD: v = av + bv; break;
                case K_SUB: v = av - bv; break;
                case K_AND: v = av & bv; break;
                case K_OR: v = av | bv; break;
                case K_XOR: v = av ^ bv; break;
                case K_SLT: v = (int64_t)av < (int64_t)bv ? 1 : 0; break;
                case K_SLTU: v = av < bv ? 1 : 0; break;
                case K_SLL: v = av << (bv & shm); break;
                case K_SRL: v = (w32 ? (av & 0xFFFFFFFFULL) : av) >> (bv & shm); break;
                case K_SRA: v = (uint64_t)((w32 ? (int64_t)(int32_t)av : (int64_t)av) >> (bv & shm)); break;
                case K_MUL: v = av * bv; break;
                // M-extension high products and division (utility.hh:171-231)
                case K_MULH: v = (uint64_t)__mul64hi((int64_t)av, (int64_t)bv); break;
                case K_MULHU: v = __umul64hi(av, bv); break;
                case K_MULHSU: v = __umul64hi(av, bv) - (((int64_t)av < 0) ? bv : 0); break;
                case K_DIV: v = w32 ? divw(av, bv) : div64(av, bv); break;
                case K_DIVU:
                    v = w32 ? ((uint32_t)bv == 0 ? ~0ULL : sx32((uint32_t)av / (uint32_t)bv)) : (bv == 0 ? ~0ULL : av / bv);
                    break;
                case K_REM: v = w32 ? remw(av, bv) : rem64(av, bv); break;
                case K_REMU:
                    v = w32 ? ((uint32_t)bv == 0 ? sx32(av) : sx32((uint32_t)av % (uint32_t)bv)) : (bv == 0 ? av : av % bv);
                    break;
                case K_NOP: wr = false; break;
                case K_JAL: v = ft; npc = spc + imm; took = true; break;
                case K_JALR: {
                    v = ft;
                    const uint64_t t = (a0 + imm) & ~1ULL;
                    const uint64_t t0 = rdl64<kNL>(t, glane);
                    if (wballot<kNL>(mine && t != t0) == 0) { npc = uni64(t0); ind = true; }
                    else { div = true; if (mine) L.pc = t; }
                    break;
                }
                case K_BEQ: case K_BNE: case K_BLT: case K_BGE: case K_BLTU: case K_BGEU: {
                    wr = false;
                    bool cnd;
                    switch (kind) {
                    case K_BEQ: cnd = a0 == b0; break;
                    case K_BNE: cnd = a0 != b0; break;
                    case K_BLT: cnd = (int64_t)a0 < (int64_t)b0; break;
                    case K_BGE: cnd = (int64_t)a0 >= (int64_t)b0; break;
                    case K_BLTU: cnd = a0 < b0; break;
                    default: cnd = a0 >= b0; break;
                    }
                    const uint64_t tk = wballot<kNL>(mine && cnd);
                    if (tk == gm) { npc = spc + imm; took = true; }
                    else if (tk != 0) { div = true; if (mine) L.pc = cnd ? spc + imm : ft; }
                    break;
                }
                default: {   // K_LOAD / K_STORE: the whole access inside one mapped page
                    const bool st = kind == K_STORE;
                    msz = 1u << ((aux >> 12) & 3);
                    const uint64_t ea = a0 + imm;
                    const uint32_t off = (uint32_t)(ea & 4095);
                    uint64_t p = 0;
                    if (mine) {
                        p = tlb_find(m, ea >> 12);
                        if (!p) OOL(p = lookup_full(CX, wc_, mc_, slot, ea >> 12));
                    }
                    // a store into the code range rewrites the lane's code: the
                    // general path's business, except in the solo kernel, which
                    // marks it here (dirty range, decode cache, any_dirty)
                    const bool code_st = st && !(ea >= tx.chi || ea + msz <= tx.clo);
                    const bool ok = p && (!st || ((p & 1) && (kNL == 1 || !code_st))) && off + msz <= 4096;
                    if (wballot<kNL>(mine && !ok) != 0) { msz = 0xFFFFFFFFu; break; }   // bail: general path
                    if (CX->record && mine) rec_mem(CX, ea, msz, L.ninst + steps, st ? 2u : 1u);
                    if constexpr (kNL == 1) {
                        if (code_st) {
                            mark_dirty(CX, m, slot, ea, ea + msz);
                            DC_INVAL(ea, msz);
                            any_dirty = true;
                        }
                    }
                    if (mine) {
                        uint8_t *pg = const_cast<uint8_t *>(page_of(p));
                        const bool al = (off & (msz - 1)) == 0;
                        if (st) {
                            if (al) {
                                switch (msz) {
                                case 1: pg[off] = (uint8_t)b0; break;
                                case 2: *(uint16_t *)(pg + off) = (uint16_t)b0; break;
                                case 4: *(uint32_t *)(pg + off) = (uint32_t)b0; break;
                                default: *(uint64_t *)(pg + off) = b0; break;
                                }
                            } else {
                                for (uint32_t i = 0; i < msz; i++) pg[off + i] = (uint8_t)(b0 >> (8 * i));
                            }
                        } else {
                            uint64_t t = 0;
                            if (al) {
                                switch (msz) {
                                case 1: t = pg[off]; break;
                                case 2: t = *(const uint16_t *)(pg + off); break;
                                case 4: t = *(const uint32_t *)(pg + off); break;
                                default: t = *(const uint64_t *)(pg + off); break;
                                }
                            } else {
                                for (uint32_t i = 0; i < msz; i++) t |= (uint64_t)pg[off + i] << (8 * i);
                            }
                            v = (aux & U_SEXT) ? (uint64_t)sext64(t, 8 * msz) : t;
                        }
                    }
                    if (st) wr = false;
                    break;
                }
                }
                if (msz == 0xFFFFFFFFu) break;            // nothing committed for this instruction
#ifdef FI_PROF
                asm volatile("" :: "v"(v));
                PSTAMP(1);
#endif
                if (w32) v = sx32(v);
                const uint32_t row = (wr && rd) ? rd : kSinkRow;
                if (mine) RREG(row) = v;
                if (any_watch && mine && row == (uint32_t)L.watch) L.watch = -1;   // overwritten before read
                if (CX->record) {   // golden trace for the liveness pass (one lane, uniform)
                    if (tpos < CX->rec_trace_cap && lane == 0)
                        CX->rec_trace[tpos] = ((((uint32_t)spc & ~1u) | (((uint32_t)spc & 1u) << 1)) - tx.lo) >> 1;
                    tpos++;
                }
                steps++; xticks += straddle; fbytes += len; dbytes += msz;
                if (div) break;
                spc = npc;
                E = ind ? pre_entry(tx, npc) : (took ? Etg : Eft);
                PSTAMP(2);
                if (steps >= budget || !ult64(spc, wait_min)) break;
            }
            if (steps) {
                if (mine) {
                    L.ninst += steps; L.ncyc += steps + xticks; L.fetch_b += fbytes; L.data_b += dbytes;
                    if (!div) L.pc = spc;
                }
                n_iter += steps;
                n_exec += steps * (uint32_t)__popcll(gm);
                continue;
            }
        }

        // ---- inner loop: one guest instruction per iteration while the group
        // stays converged, with no event due and no page request pending
        for (;;) {
        // ---- D. fetch + decode (wave-uniform)
        Dec d;
        uint32_t ticks = 1;
        bool fast = false;
        const uint64_t key = (lpc & 3) ? ((lpc & ~3ULL) | 2) : lpc;
        if (CX->pre_ok && key >= CX->text_lo && key < CX->text_hi && wballot<kNL>(mine && dirty_at(CX, m, lpc)) == 0) {
            const Pre4 q = pre_load(CX->pre + ((key - CX->text_lo) >> 1));
            const uint32_t pflags = (q.w >> 8) & 0xFF;
            if (pflags & kPreValid) {
                fast = true;
                d.raw = q.x; d.op = (uint8_t)q.y; d.rd = (uint8_t)(q.y >> 8); d.rs1 = (uint8_t)(q.y >> 16);
                d.rs2 = (uint8_t)(q.y >> 24); d.imm = (int32_t)q.z; d.len = (uint8_t)q.w;
                d.flags = (uint8_t)pflags; d.aux = (uint16_t)(q.w >> 16);
                ticks = (pflags & kPreStraddle) ? 2 : 1;
            }
        }
        if constexpr (kNL == 1) {   // solo: rewritten code decoded before (DCT/DCE)
            if (!fast && L.pc >= CX->code_lo && L.pc < CX->code_hi) {
                const uint32_t ci = (uint32_t)(L.pc >> 1) & (kDC - 1);
                if (DCT[ci] == (uint32_t)(L.pc - CX->text_lo)) {
                    const Pre4 q = DCE[ci];
                    const uint32_t pflags = (q.w >> 8) & 0xFF;
                    fast = true;
                    d.raw = q.x; d.op = (uint8_t)q.y; d.rd = (uint8_t)(q.y >> 8); d.rs1 = (uint8_t)(q.y >> 16);
                    d.rs2 = (uint8_t)(q.y >> 24); d.imm = (int32_t)q.z; d.len = (uint8_t)q.w;
                    d.flags = (uint8_t)pflags; d.aux = (uint16_t)(q.w >> 16);
                    ticks = (pflags & kPreStraddle) ? 2 : 1;
                }
            }
        }
        if (!fast) {
            PSTAMP(4);
            n_slow++;
            uint32_t raw = 0, t = 1;
            uint64_t fva = 0;
            if (mine) {
                int fr;
                OOL(fr = fetch_lane(CX, wc_, mc_, slot, L.pc, raw, t, fva));
                if (fr) {
                    // the faulting tick(s) count, nothing commits; decoder reset;
                    // GenericPageTableFault::invoke -> fixupFault (sim/faults.cc:95-105)
                    L.ncyc += t;
                    mine = false;
                    int h;
                    OOL(h = fixup_fault(CX, mc_, slot, fva));
                    if (h == 0) finish(L, FI_CRASH, FI_CRASH_PAGE_FAULT, 134, (uint32_t)fva);
                    else if (h == -1) finish(L, FI_CRASH, FI_CRASH_STACK_LIMIT, 1, (uint32_t)L.pc);
                    else if (h == -2) finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, (uint32_t)L.pc);
                }
            }
            const uint64_t okm = wballot<kNL>(mine);
            if (okm == 0) break;
            const int ld = __ffsll((unsigned long long)okm) - 1;
            const uint32_t lraw = (uint32_t)rdl32<kNL>((uint32_t)raw, ld);
            const uint32_t lt = (uint32_t)rdl32<kNL>((uint32_t)t, ld);
            mine = mine && raw == lraw;
            PSTAMP(5);
            d = rv_decode(lraw);
            ticks = lt;
            if constexpr (kNL == 1) {
                if (L.pc >= CX->code_lo && L.pc < CX->code_hi) {
                    Dec dd = d;
                    const uint32_t u = uop_of(dd);   // uop_of may normalise dd.imm (the fast path's form)
                    const uint32_t ci = (uint32_t)(L.pc >> 1) & (kDC - 1);
                    DCT[ci] = (uint32_t)(L.pc - CX->text_lo);
                    DCE[ci].x = dd.raw;
                    DCE[ci].y = (uint32_t)dd.op | ((uint32_t)dd.rd << 8) | ((uint32_t)dd.rs1 << 16) |
                                ((uint32_t)dd.rs2 << 24);
                    DCE[ci].z = (uint32_t)dd.imm;
                    DCE[ci].w = (uint32_t)dd.len | ((uint32_t)(kPreValid | (lt == 2 ? kPreStraddle : 0) | dd.flags) << 8) |
                                (u << 16);
                }
            }
#ifdef FI_PROF
            asm volatile("" :: "s"((uint32_t)d.op), "s"((uint32_t)d.imm));
#endif
            PSTAMP(6);
        }
        // force every decoded field into SGPRs: the op switch below must be a
        // scalar branch tree, never a per-lane waterfall
        d.op = (uint8_t)uni32(d.op); d.rd = (uint8_t)uni32(d.rd); d.rs1 = (uint8_t)uni32(d.rs1);
        d.rs2 = (uint8_t)uni32(d.rs2); d.len = (uint8_t)uni32(d.len); d.flags = (uint8_t)uni32(d.flags);
        d.imm = (int32_t)uni32((uint32_t)d.imm); d.aux = (uint16_t)uni32(d.aux); d.raw = uni32(d.raw);
        ticks = uni32(ticks);
        const uint64_t gmask = wballot<kNL>(mine);
        n_exec += (uint32_t)__popcll(gmask);
        int f = F_NONE;
        {   // every lane evaluates the (uniform) op: the switch stays a scalar
            // branch tree in uniform control flow; only group lanes commit
        // ---- E. execute: the generated StaticInst::execute bodies of
        // src/arch/riscv/isa/decoder.isa for the modelled subset
        const uint64_t pc = L.pc;
        const uint64_t a = RREG(d.rs1), b = RREG(d.rs2);
        const int64_t imm = d.imm;
        uint64_t npc = pc + d.len;
        uint64_t v = 0, fva = 0, t = 0;
        bool wrd = true;
        uint32_t msz = 0, mext = 0;   // memory access size / sign-extension width (uniform)
        bool mst = false;
        uint64_t sval = b;            // store data (an FP register for FP stores)
        uint64_t fval = 0;            // FP destination value
        uint32_t fbox = 0;            // FP destination: 0 none, 1 fval, 16/32/64 loaded (NaN-boxed) width
        uint32_t fpst = 0;            // FP status update: 0x100 | flags raised, 0x200 | fflags | frm << 5 written
        uint32_t xticks = 0;          // extra micro-op ticks (AMO fences)
        int amo = -1;                 // AMO read-modify-write op (amo_apply), -1 none
        int llsc = 0;                 // 1 LR, 2 SC
        uint32_t cbo = 0;             // cache-block op: 1 translate only, 2 zero the line
        bool m5 = false;              // M5Op: a1 = 0 at commit
        uint32_t m5x = 0, m5code = 0; // an M5 op that ends the run once it commits: 1 exit, 2 fail, 3 quiesce
        uint32_t nvcfg = ~0u;         // vset*: the vector configuration from the next instruction on
        bool xdet = false;            // a replica watch read through an M5Op's ABI arguments
#define FREG_RD(r) (L.fp ? CX->fregs[(uint64_t)(r) * CX->n_slots + slot] : 0ULL)
        // detected-by-replica: the flipped protected register is read before
        // being overwritten (build-defined SHREWD semantics)
        const bool detect = L.watch > 0 &&
            (((d.flags & kPreRs1) && d.rs1 == L.watch) || ((d.flags & kPreRs2) && d.rs2 == L.watch) ||
             (d.op == OP_ecall && (L.watch == 17 || (L.watch >= 10 && L.watch <= 15))));
        {
            switch (d.op) {
            case OP_UNKNOWN: f = F_UNKNOWN; break;
            case OP_ESC_FP: case OP_ESC_VEC: case OP_ESC_AMO: case OP_ESC_SYS: case OP_ESC_CRYPTO: case OP_ESC_CBO:
            case OP_ESC_CMP: case OP_ESC_M5: case OP_ESC_HYP: f = F_ESCAPE; break;
            case OP_c_addi4spn: if (imm == 0) f = F_ILLEGAL; else v = a + imm; break;
            // loads/stores only describe the access here; the single access site
            // after the switch keeps the hot loop small (one inlined copy)
            case OP_c_lwsp: if (d.rd == 0) { f = F_ILLEGAL; break; } msz = 4; mext = 32; break;
            case OP_c_lw: case OP_lw: msz = 4; mext = 32; break;
            case OP_c_ldsp: if (d.rd == 0) { f = F_ILLEGAL; break; } msz = 8; break;
            case OP_c_ld: case OP_ld: msz = 8; break;
            case OP_c_lbu: case OP_lbu: msz = 1; break;
            case OP_c_lhu: case OP_lhu: msz = 2; break;
            case OP_c_lh: case OP_lh: msz = 2; mext = 16; break;
            case OP_lb: msz = 1; mext = 8; break;
            case OP_lwu: msz = 4; break;
            case OP_c_sb: case OP_sb: msz = 1; mst = true; wrd = false; break;
            case OP_c_sh: case OP_sh: msz = 2; mst = true; wrd = false; break;
            case OP_c_sw: case OP_sw: case OP_c_swsp: msz = 4; mst = true; wrd = false; break;
            case OP_c_sd: case OP_sd: case OP_c_sdsp: msz = 8; mst = true; wrd = false; break;
            case OP_c_addi: case OP_addi: v = a + imm; break;
            case OP_c_addiw: if (d.rd == 0) f = F_ILLEGAL; else v = sx32(a + imm); break;
            case OP_addiw: v = sx32(a + imm); break;
            case OP_c_li: case OP_lui: v = (uint64_t)imm; break;
            case OP_c_addi16sp: if (imm == 0) f = F_ILLEGAL; else v = a + imm; break;
            case OP_c_lui: if (imm == 0) f = F_ILLEGAL; else v = (uint64_t)imm; break;
            case OP_c_srli: case OP_srli: v = a >> imm; break;
            case OP_c_srai: case OP_srai: v = (uint64_t)((int64_t)a >> imm); break;
            case OP_c_andi: case OP_andi: v = a & (uint64_t)imm; break;
            case OP_c_sub: case OP_sub: v = a - b; break;
            case OP_c_xor: case OP_xor_: v = a ^ b; break;
            case OP_c_or: case OP_or_: v = a | b; break;
            case OP_c_and: case OP_and_: v = a & b; break;
            case OP_c_subw: case OP_subw: v = sx32((uint32_t)a - (uint32_t)b); break;
            case OP_c_addw: case OP_addw: v = sx32((uint32_t)a + (uint32_t)b); break;
            case OP_c_mul: case OP_mul: v = a * b; break;
            case OP_c_zext_b: v = a & 0xFF; break;
            case OP_c_sext_b: case OP_sext_b: v = (uint64_t)sext64(a & 0xFF, 8); break;
            case OP_c_zext_h: v = a & 0xFFFF; break;
            case OP_c_sext_h: case OP_sext_h: v = (uint64_t)sext64(a & 0xFFFF, 16); break;
            case OP_c_zext_w: v = a & 0xFFFFFFFFULL; break;
            case OP_c_not: v = ~a; break;
            case OP_c_j: npc = pc + imm; wrd = false; break;
            case OP_c_beqz: if (a == 0) npc = pc + imm; wrd = false; break;
            case OP_c_bnez: if (a != 0) npc = pc + imm; wrd = false; break;
            case OP_c_slli: case OP_slli: v = a << imm; break;
            case OP_c_jr: if (d.rs1 == 0) f = F_ILLEGAL; else npc = a & ~1ULL; wrd = false; break;
            case OP_c_mv: v = b; break;
            case OP_c_ebreak: case OP_ebreak: f = F_BREAK; break;
            case OP_c_jalr: v = npc; npc = a & ~1ULL; break;
            case OP_c_add: case OP_add: v = a + b; break;
            case OP_fence: case OP_fence_i: wrd = false; break;
            case OP_bseti: v = a | (1ULL << (imm & 63)); break;
            case OP_bclri: v = a & ~(1ULL << (imm & 63)); break;
            case OP_binvi: v = a ^ (1ULL << (imm & 63)); break;
            case OP_clz: v = a ? __builtin_clzll(a) : 64; break;
            case OP_ctz: v = a ? __builtin_ctzll(a) : 64; break;
            case OP_cpop: v = __builtin_popcountll(a); break;
            case OP_slti: v = (int64_t)a < imm ? 1 : 0; break;
            case OP_sltiu: v = a < (uint64_t)imm ? 1 : 0; break;
            case OP_xori: v = a ^ (uint64_t)imm; break;
            case OP_orc_b: v = orc_b(a); break;
            case OP_bexti: v = (a >> (imm & 63)) & 1; break;
            case OP_rori: v = (a >> imm) | (a << ((64 - imm) & 63)); break;
            case OP_rev8: v = __builtin_bswap64(a); break;
            case OP_prefetch_i: case OP_prefetch_r: case OP_prefetch_w: wrd = false; break;
            case OP_ori_hint: case OP_ori: v = a | (uint64_t)imm; break;
            case OP_auipc: v = pc + imm; break;
            case OP_slliw: v = sx32((uint32_t)a << imm); break;
            case OP_slli_uw: v = (a & 0xFFFFFFFFULL) << imm; break;
            case OP_clzw: v = (uint32_t)a ? __builtin_clz((uint32_t)a) : 32; break;
            case OP_ctzw: v = (uint32_t)a ? __builtin_ctz((uint32_t)a) : 32; break;
            case OP_cpopw: v = __builtin_popcount((uint32_t)a); break;
            case OP_srliw: v = sx32((uint32_t)a >> imm); break;
            case OP_sraiw: v = (uint64_t)(int64_t)((int32_t)(uint32_t)a >> imm); break;
            case OP_roriw: { const uint32_t x = (uint32_t)a; v = sx32((x >> imm) | (x << ((32 - imm) & 31))); break; }
            case OP_sll: v = a << (b & 63); break;
            case OP_mulh: v = (uint64_t)__mul64hi((int64_t)a, (int64_t)b); break;
            case OP_clmul: v = clmul(a, b); break;
            case OP_bset: v = a | (1ULL << (b & 63)); break;
            case OP_bclr: v = a & ~(1ULL << (b & 63)); break;
            case OP_rol: { const int sh = (int)(b & 63); v = (a << sh) | (a >> ((64 - sh) & 63)); break; }
            case OP_binv: v = a ^ (1ULL << (b & 63)); break;
            case OP_slt: v = (int64_t)a < (int64_t)b ? 1 : 0; break;
            case OP_mulhsu: v = __umul64hi(a, b) - (((int64_t)a < 0) ? b : 0); break;
            case OP_clmulr: v = clmulr(a, b); break;
            case OP_sh1add: v = (a << 1) + b; break;
            case OP_sltu: v = a < b ? 1 : 0; break;
            case OP_mulhu: v = __umul64hi(a, b); break;
            case OP_clmulh: v = clmulh(a, b); break;
            case OP_div_: v = div64(a, b); break;
            case OP_pack: v = (b << 32) | (a & 0xFFFFFFFFULL); break;
            case OP_min_: v = (int64_t)a < (int64_t)b ? a : b; break;
            case OP_sh2add: v = (a << 2) + b; break;
            case OP_xnor: v = ~(a ^ b); break;
            case OP_srl: v = a >> (b & 63); break;
            case OP_divu: v = b == 0 ? ~0ULL : a / b; break;
            case OP_czero_eqz: v = b == 0 ? 0 : a; break;
            case OP_sra: v = (uint64_t)((int64_t)a >> (b & 63)); break;
            case OP_minu: v = a < b ? a : b; break;
            case OP_bext: v = (a >> (b & 63)) & 1; break;
            case OP_ror: { const int sh = (int)(b & 63); v = (a >> sh) | (a << ((64 - sh) & 63)); break; }
            case OP_rem: v = rem64(a, b); break;
            case OP_max_: v = (int64_t)a > (int64_t)b ? a : b; break;
            case OP_sh3add: v = (a << 3) + b; break;
            case OP_orn: v = a | ~b; break;
            case OP_remu: v = b == 0 ? a : a % b; break;
            case OP_packh: v = ((b & 0xFF) << 8) | (a & 0xFF); break;
            case OP_maxu: v = a > b ? a : b; break;
            case OP_czero_nez: v = b != 0 ? 0 : a; break;
            case OP_andn: v = a & ~b; break;
            case OP_mulw: v = sx32((uint32_t)a * (uint32_t)b); break;
            case OP_add_uw: v = (a & 0xFFFFFFFFULL) + b; break;
            case OP_sllw: v = sx32((uint32_t)a << (b & 31)); break;
            case OP_rolw: v = rolw(a, b); break;
            case OP_sh1add_uw: v = ((a & 0xFFFFFFFFULL) << 1) + b; break;
            case OP_divw: v = divw(a, b); break;
            case OP_packw: v = sx32(((b & 0xFFFF) << 16) | (a & 0xFFFF)); break;
            case OP_sh2add_uw: v = ((a & 0xFFFFFFFFULL) << 2) + b; break;
            case OP_srlw: v = sx32((uint32_t)a >> (b & 31)); break;
            case OP_divuw: v = (uint32_t)b == 0 ? ~0ULL : sx32((uint32_t)a / (uint32_t)b); break;
            case OP_sraw: v = (uint64_t)(int64_t)((int32_t)(uint32_t)a >> (b & 31)); break;
            case OP_rorw: v = rorw(a, b); break;
            case OP_remw: v = remw(a, b); break;
            case OP_sh3add_uw: v = ((a & 0xFFFFFFFFULL) << 3) + b; break;
            case OP_remuw: v = (uint32_t)b == 0 ? sx32(a) : sx32((uint32_t)a % (uint32_t)b); break;
            case OP_beq: if (a == b) npc = pc + imm; wrd = false; break;
            case OP_bne: if (a != b) npc = pc + imm; wrd = false; break;
            case OP_blt: if ((int64_t)a < (int64_t)b) npc = pc + imm; wrd = false; break;
            case OP_bge: if ((int64_t)a >= (int64_t)b) npc = pc + imm; wrd = false; break;
            case OP_bltu: if (a < b) npc = pc + imm; wrd = false; break;
            case OP_bgeu: if (a >= b) npc = pc + imm; wrd = false; break;
            case OP_jalr: v = npc; npc = (a + imm) & ~1ULL; break;
            case OP_jal: v = npc; npc = pc + imm; break;
            case OP_ecall: f = F_SYSCALL; break;
            case OP_csr: {
                const uint32_t csr = d.raw >> 20;
                if (csr >= 1 && csr <= 3) {
                    // fflags / frm / fcsr (oracle/rv64se.c OP_csr; CSRExecute, formats/standard.isa:
                    // 325-447; ISA::readCSR / writeCSR, isa.cc:1141-1300)
                    const uint32_t f3 = (d.raw >> 12) & 7, idx = (uint32_t)d.imm;   // rs1 field / uimm
                    const uint64_t src = f3 >= 5 ? (uint64_t)idx : a;
                    const bool rdc = (f3 == 1 || f3 == 5) ? d.rd != 0 : true;
                    const bool wrc = (f3 == 1 || f3 == 5) ? true : idx != 0;
                    const uint64_t data = !rdc ? 0 : csr == 1 ? L.fflags : csr == 2 ? L.frm
                                                                 : (uint64_t)(L.fflags | (L.frm << 5));
                    v = data;
                    const uint64_t nd = (f3 & 3) == 1 ? src : (f3 & 3) == 2 ? (data | src) : (data & ~src);
                    if (wrc) {
                        uint32_t nf = L.fflags, nr = L.frm;
                        if (csr == 1) nf = (uint32_t)(nd & 0x1F);
                        else if (csr == 2) nr = (uint32_t)(nd & 7);
                        else { nf = (uint32_t)(nd & 0x1F); nr = (uint32_t)((nd >> 5) & 7); }
                        fpst = 0x200u | nf | (nr << 5);
                    }
                    break;
                }
                f = csr_u_accessible(csr) ? F_ESCCSR : F_ILLEGAL;
                break;
            }
            // ---- F/D/Zfh data movement: loads/stores through the single access
            // site below (access first, then the FPU-status update, which never
            // faults in SE: fs = INITIAL, isa.cc:390)
            case OP_flh: msz = 2; fbox = 16; wrd = false; break;
            case OP_flw: msz = 4; fbox = 32; wrd = false; break;
            case OP_fld: case OP_c_fld: case OP_c_fldsp: msz = 8; fbox = 64; wrd = false; break;
            case OP_fsh: msz = 2; mst = true; wrd = false; sval = FREG_RD(d.rs2); break;
            case OP_fsw: msz = 4; mst = true; wrd = false; sval = FREG_RD(d.rs2); break;
            case OP_fsd: case OP_c_fsd: case OP_c_fsdsp: msz = 8; mst = true; wrd = false; sval = FREG_RD(d.rs2); break;
            case OP_fmv_x_w: v = sx32(FREG_RD(d.rs1)); break;
            case OP_fmv_x_d: v = FREG_RD(d.rs1); break;
            case OP_fmv_x_h: v = (uint64_t)sext64(FREG_RD(d.rs1) & 0xFFFF, 16); break;
            case OP_fmv_w_x: fval = 0xFFFFFFFF00000000ULL | (a & 0xFFFFFFFFULL); fbox = 1; wrd = false; break;
            case OP_fmv_d_x: fval = a; fbox = 1; wrd = false; break;
            case OP_fmv_h_x: fval = 0xFFFFFFFFFFFF0000ULL | (a & 0xFFFF); fbox = 1; wrd = false; break;
            case OP_fsgnj_s: case OP_fsgnjn_s: case OP_fsgnjx_s: {
                const uint64_t x = fp_unbox32(FREG_RD(d.rs1)), y = fp_unbox32(FREG_RD(d.rs2));
                const uint64_t sg = d.op == OP_fsgnj_s ? y : d.op == OP_fsgnjn_s ? ~y : (x ^ y);
                fval = 0xFFFFFFFF00000000ULL | (x & 0x7FFFFFFFULL) | (sg & 0x80000000ULL); fbox = 1; wrd = false;
                break;
            }
            case OP_fsgnj_d: case OP_fsgnjn_d: case OP_fsgnjx_d: {
                const uint64_t x = FREG_RD(d.rs1), y = FREG_RD(d.rs2);
                const uint64_t sg = d.op == OP_fsgnj_d ? y : d.op == OP_fsgnjn_d ? ~y : (x ^ y);
                fval = (x & 0x7FFFFFFFFFFFFFFFULL) | (sg & 0x8000000000000000ULL); fbox = 1; wrd = false;
                break;
            }
            case OP_fsgnj_h: case OP_fsgnjn_h: case OP_fsgnjx_h: {
                const uint64_t x = fp_unbox16(FREG_RD(d.rs1)), y = fp_unbox16(FREG_RD(d.rs2));
                const uint64_t sg = d.op == OP_fsgnj_h ? y : d.op == OP_fsgnjn_h ? ~y : (x ^ y);
                fval = 0xFFFFFFFFFFFF0000ULL | (x & 0x7FFF) | (sg & 0x8000); fbox = 1; wrd = false;
                break;
            }
            case OP_fclass_s: v = fp_classify(fp_unbox32(FREG_RD(d.rs1)), 8, 23); break;
            case OP_fclass_d: v = fp_classify(FREG_RD(d.rs1), 11, 52); break;
            case OP_fclass_h: v = fp_classify(fp_unbox16(FREG_RD(d.rs1)), 5, 10); break;
            case OP_fadd: case OP_fsub: case OP_fmul: case OP_fdiv: case OP_fsqrt: case OP_fmadd: case OP_fmsub:
            case OP_fnmsub: case OP_fnmadd: case OP_fmin: case OP_fmax: case OP_feq: case OP_flt: case OP_fle:
            case OP_fcvt_f2i: case OP_fcvt_i2f: case OP_fcvt_f2f: case OP_fli: case OP_fround: case OP_fcvtmod: {
                const uint32_t ui = (uint32_t)d.imm;
                const FpRes fr = fp_exec(d.op, ui, d.rs2, FREG_RD(d.rs1), FREG_RD(d.rs2), FREG_RD((ui >> 8) & 31), a,
                                         L.frm);
                if (fr.kind == 2) { f = F_ILLEGAL; break; }
                fpst = 0x100u | fr.fl;
                if (fr.kind == 1) v = fr.v;
                else { fval = fr.v; fbox = 1; wrd = false; }
                break;
            }
            // ---- A-extension RMW: AtomicSimpleCPU::amoMem (atomic.cc:546-608)
            // panics on a 64-byte-line crossing before translating; one
            // translation, then read-modify-write; rl/aq fences are extra
            // micro-op ticks (amo.isa macro-op constructors)
            case OP_amoadd_w: case OP_amoswap_w: case OP_amoxor_w: case OP_amoor_w: case OP_amoand_w:
            case OP_amomin_w: case OP_amomax_w: case OP_amominu_w: case OP_amomaxu_w:
            case OP_amoadd_d: case OP_amoswap_d: case OP_amoxor_d: case OP_amoor_d: case OP_amoand_d:
            case OP_amomin_d: case OP_amomax_d: case OP_amominu_d: case OP_amomaxu_d: {
                const bool w32 = d.op <= OP_amomaxu_w;
                msz = w32 ? 4 : 8;
                if (((a + msz - 1) & ~63ULL) > a) { f = F_AMOLINE; msz = 0; break; }
                amo = (int)d.op - (w32 ? OP_amoadd_w : OP_amoadd_d);
                xticks = ((d.raw >> 25) & 1) + ((d.raw >> 26) & 1);   // rl, aq (pre-decoded aux holds the micro-op)
                break;
            }
            // ---- LR / SC (formats/amo.isa LoadReserved / StoreCond; the rl / aq
            // fence micro-ops are one tick each, like the AMOs')
            case OP_lr_w: case OP_lr_d:
                msz = d.op == OP_lr_w ? 4 : 8; mext = msz == 4 ? 32 : 0; llsc = 1;
                xticks = ((d.raw >> 25) & 1) + ((d.raw >> 26) & 1);
                if (CX->record) CX->stats[22] = 1;   // golden LR/SC state is not in the snapshots
                break;
            case OP_sc_w: case OP_sc_d:
                msz = d.op == OP_sc_w ? 4 : 8; llsc = 2;
                xticks = ((d.raw >> 25) & 1) + ((d.raw >> 26) & 1);
                if (CX->record) CX->stats[22] = 1;
                break;
            // ---- privileged SYSTEM / hypervisor load-store from PRV_U, cache-block
            // ops, M5 pseudo-ops, scalar crypto (oracle/rv64se.c refine_misc, execute)
            case OP_priv: if (!d.imm) f = F_ILLEGAL; wrd = false; break;
            case OP_cbo: wrd = false; cbo = d.imm == 4 ? 2u : 1u; msz = d.imm == 4 ? 64u : 1u; mst = d.imm == 4; break;
            case OP_m5op: {   // a0 = result, a1 = 0 (M5Op::execute); pseudoInstWork under SE defaults
                m5 = true;
                switch ((uint32_t)d.imm) {
                // rpns: curTick() in ns during this instruction's execute -- its
                // fetch tick(s) already elapsed (the commit adds them to ncyc)
                case 0x07:
                    if (CX->clk_esc) { f = F_TKCLOCK; break; }
                    v = (CX->tick0 + (L.ncyc + ticks - 1) * CX->clk_period) / 1000;
                    if (CX->record) CX->stats[52] = L.ninst + 1;
                    break;
                case 0x23:   // m5sum(a0..a5)
                    xdet = L.watch >= 10 && L.watch <= 15;
                    v = RREG(10) + RREG(11) + RREG(12) + RREG(13) + RREG(14) + RREG(15);
                    break;
                case 0x30: {   // initParam: key = the C string in a0, a1 ("", dist-rank, dist-size)
                    xdet = L.watch == 10 || L.watch == 11;
                    const uint64_t k0 = RREG(10), k1 = RREG(11);
                    if ((k0 & 0xFF) == 0) v = 0;
                    else if (k0 == 0x6E61722D74736964ULL && (k1 & 0xFFFF) == 0x6B) v = 0;
                    else if (k0 == 0x7A69732D74736964ULL && (k1 & 0xFFFF) == 0x65) v = 1;
                    else f = F_M5PANIC;
                    break;
                }
                case 0x51: f = F_BREAK; break;       // debugbreak -> SIGTRAP
                case 0x54: f = F_M5PANIC; break;     // m5_panic
                // quiesce: the only context suspends after this commit and nothing
                // wakes it -- a hang (oracle/rv64se.c OP_m5op, thread_context.cc:167)
                case 0x01: m5x = 3; break;
                // m5_exit(delay) / m5_fail(delay, code) with delay 0: the stdlib
                // run script ends the simulation after this tick (pseudo_inst.cc:
                // 178-204, simulate/exit_handler.py:551-557); a delayed one escapes
                case 0x21: case 0x22:
                    xdet = L.watch == 10 || (d.imm == 0x22 && L.watch == 11);
                    if (RREG(10) != 0) { f = F_ESCAPE; break; }
                    m5x = d.imm == 0x21 ? 1u : 2u;
                    m5code = d.imm == 0x22 ? (uint32_t)(RREG(11) & 0xff) : 0u;
                    break;
                // checkpoint (the stdlib saves one and continues), switchcpu (not a
                // switchable processor): no architectural effect, result 0
                case 0x43: case 0x52: v = 0; break;
                case 0x02: case 0x03: case 0x04: case 0x4f:
                case 0x53: case 0x5a: case 0x5b: case 0x62: case 0x70: case 0x71:
                    f = F_ESCAPE; break;             // simulator control / host files
                default: v = 0; break;               // no architectural effect: result 0
                }
                break;
            }
            case OP_crypto: v = rvk::exec(d.imm, a, b); break;
            // RVV in the process-start vector configuration (oracle/rv64se.c
            // VEC_*): no-op (one or two micro-op ticks), IllegalInst (vill),
            // undefined in gem5, needs vector state; under any other
            // configuration it needs the vector unit's state (escape)
            case OP_vec:
                wrd = false;
                if (m.vcfg) f = F_ESCAPE;
                else if (d.imm == 3) xticks = 1;
                else if (d.imm == 4) f = F_ILLEGAL;
                else if (d.imm == 5) f = F_UNDEF;
                else if (d.imm == 6) f = F_ESCAPE;
                break;
            // vset* (oracle/rv64se.c OP_vset; formats/vector_conf.isa:115-186):
            // getNewVtype (a request other than the current vtype: vsew > 3
            // trips getSew's assert, an illegal one gives vill), VLMAX =
            // VLEN 256 / SEW x LMUL, getNewVL on the rd / rs1 indices with a
            // uint32_t requested vl; rd = vl, the configuration from the next
            // instruction on (committed with the instruction)
            case OP_vset: {
                const uint32_t form = ((uint32_t)d.imm >> 16) & 3u;
                const uint64_t req = form == 1 ? b : (uint64_t)((uint32_t)d.imm & 0xFFFFu);
                const uint32_t vc = m.vcfg ^ 0x100u;
                const uint64_t old = (uint64_t)(vc & 0xFF) | ((uint64_t)((vc >> 8) & 1) << 63);
                uint64_t nt = old;
                if (req != old) {
                    const uint32_t vsew = (uint32_t)(req >> 3) & 7, vlmul = (uint32_t)req & 7;
                    const uint32_t lim = vlmul <= 3 ? 64 : vlmul == 5 ? 8 : vlmul == 6 ? 16 : vlmul == 7 ? 32 : 0;
                    if (vsew > 3) { f = F_VSEW; break; }
                    nt = (vlmul == 4 || (8u << vsew) > lim || ((req >> 8) & ((1ULL << 55) - 1)) != 0) ? (1ULL << 63) : req;
                }
                uint32_t vlmax = 0;
                if (!(nt >> 63)) {
                    const uint32_t vsew = (uint32_t)(nt >> 3) & 7, vlmul = (uint32_t)nt & 7, per = 32u >> vsew;
                    vlmax = vlmul <= 3 ? per << vlmul : per >> (8 - vlmul);
                }
                const uint32_t rs1b = form == 2 ? 1u : d.rs1, rqvl = form == 2 ? ((uint32_t)d.imm >> 20) : (uint32_t)a;
                const uint32_t cur = vc >> 9;
                const uint32_t nvl = vlmax == 0 ? 0u
                                   : (d.rd == 0 && rs1b == 0) ? (cur < vlmax ? cur : vlmax)
                                   : rs1b == 0 ? vlmax : (rqvl < vlmax ? rqvl : vlmax);
                nvcfg = ((uint32_t)(nt & 0xFF) | ((uint32_t)(nt >> 63) << 8) | (nvl << 9)) ^ 0x100u;
                v = nvl;
                break;
            }
            default: f = F_UNKNOWN; break;
            }
        }
        if (detect || xdet) f = F_DETECT;   // the op does not execute
        bool lp_silent = false;   // a loop probe's plain store wrote the bytes already there
        if (mine) {
        if (msz && f == F_NONE) {
            // one call site (an AMO reads, then writes, in a second pass): a
            // second inlined copy of mem_access puts the lane state in scratch
            const uint64_t ea = cbo ? (a & ~63ULL) : (amo >= 0 || llsc) ? a : a + imm;
            uint64_t old = 0;
            if constexpr (kNL == 1) {
                if (LP.on && mst && amo < 0 && !llsc && !cbo) {   // the bytes before the store (no side effect)
                    uint64_t ov = 0, fv = 0;
                    int fo;
                    OOL(fo = mem_access(CX, wc_, mc_, slot, ea, msz, false, ov, fv, 0));
                    const uint64_t mk = msz >= 8 ? ~0ULL : ((1ULL << (8 * msz)) - 1);
                    lp_silent = fo == F_NONE && ((ov ^ sval) & mk) == 0;
                }
            }
#pragma unroll 1
            for (int pass = 0; pass < (amo >= 0 ? 2 : 1); pass++) {
                t = pass ? amo_apply(amo, old, b, msz == 4) : (amo >= 0 ? 0 : (llsc == 2 ? b : sval));
                OOL(f = mem_access(CX, wc_, mc_, slot, ea, msz, pass ? true : mst, t, fva, amo >= 0 ? 3 : llsc));
                if (f != F_NONE) break;
                if (!pass) old = t;
            }
            if (f == F_NONE) {
                if (CX->record)   // an AMO reads, then writes; a failed SC touches nothing
                    rec_mem(CX, ea, msz, L.ninst, amo >= 0 ? 3u : llsc == 2 ? (t ? 2u : 0u) : (mst ? 2u : 1u));
                if (mst || amo >= 0 || (llsc == 2 && t)) DC_INVAL(ea, msz);   // rewritten code: drop its cached decodes
                if ((llsc != 2 || t) && cbo != 1) L.data_b += amo >= 0 ? 2 * msz : msz;
                if (amo >= 0) v = msz == 4 ? sx32(old) : old;
                else if (llsc == 2) v = t ? 0 : 1;   // rd = !success (amo.isa StoreCondExecute)
                else if (!mst) {
                    if (fbox) fval = fbox == 16 ? (0xFFFFFFFFFFFF0000ULL | t) : fbox == 32 ? (0xFFFFFFFF00000000ULL | t) : t;
                    else v = mext ? (uint64_t)sext64(t, mext) : t;
                }
            }
        }
        // F_NEEDPAGE: copy-on-write first; the tick is retried (no commit)
        // ---- F. commit: countInst only on NoFault (atomic.cc:687-689), then
        // advancePC (src/cpu/simple/base.cc:493-512)
        if (f != F_NEEDPAGE) {
        L.ncyc += ticks;
        L.fetch_b += d.len;
        if (CX->record && (f == F_NONE || f == F_SYSCALL)) {
            const uint64_t ho = ((pc & ~1ULL) | ((pc & 1) << 1)) - CX->text_lo;
            const uint32_t ev = ho < CX->text_bytes ? (uint32_t)(ho >> 1) : 0x7FFFFFFFu;
            if (tpos < CX->rec_trace_cap) CX->rec_trace[tpos] = ev | (f == F_SYSCALL ? 0x80000000u : 0u);
            tpos++;
        }
        if (f == F_NONE) {
            if (fbox || fpst) {   // FP state written: materialise the lane's FP file on its first write
                if (!L.fp) {
                    for (int r = 0; r < 32; r++) CX->fregs[(uint64_t)r * CX->n_slots + slot] = 0;
                    L.fp = true;
                    if (CX->record) CX->stats[22] = 1;   // the golden run uses FP state (host disables snapshots)
                }
                if (fbox) CX->fregs[(uint64_t)d.rd * CX->n_slots + slot] = fval;
                if (fpst & 0x100u) L.fflags |= (uint8_t)(fpst & 0x1F);       // FFLAGS_EXE: accumulate
                if (fpst & 0x200u) { L.fflags = (uint8_t)(fpst & 0x1F); L.frm = (uint8_t)((fpst >> 5) & 7); }
            }
            L.ncyc += xticks;
            if (nvcfg != ~0u) {
                m.vcfg = nvcfg;
                if (CX->record && nvcfg) CX->stats[22] = 1;   // golden vector state is not in the snapshots
            }
            bool rdet = false;
            if (L.injected == 3) {   // result fault (oracle/rv64se.c:result_fault)
                if (!(wrd && d.rd)) L.injected = 2;
                else if (replicated(CX, op_class(d.op), L.ninst)) rdet = true;
                else { v ^= s.mask; L.injected = 1; }
            }
            if (wrd && d.rd) RREG(d.rd) = v;
            if (wrd && L.watch > 0 && (d.flags & kPreRd) && d.rd == L.watch) L.watch = -1;
            if (m5) { RREG(11) = 0; if (L.watch == 11) L.watch = -1; }
            L.ninst++;
            if (rdet) finish(L, FI_DETECTED, 0, 0, (uint32_t)pc);   // the shadow disagrees at commit
            else L.pc = npc;
            if (m5x && !L.done) {   // the M5 op that ends the run has committed
                if (m5x == 3) {
                    finish(L, FI_HANG, FI_HANG_QUIESCE, 0, (uint32_t)L.pc);
                } else if (CX->record) {
                    finish(L, FI_MASKED, m5x == 1 ? FI_END_M5_EXIT : FI_END_M5_FAIL, (int)m5code, (uint32_t)L.pc);
                } else {
                    const bool same = !L.out_bad && L.out_pos == CX->gout_len && L.err_pos == CX->gerr_len &&
                                      m5code == CX->gexit && CX->gsub == (m5x == 1 ? FI_END_M5_EXIT : FI_END_M5_FAIL);
                    finish(L, same ? FI_MASKED : FI_SDC, m5x == 1 ? FI_END_M5_EXIT : FI_END_M5_FAIL, (int)m5code,
                           (uint32_t)L.pc);
                }
            }
            if constexpr (kNL == 1) {
                if (!LP.on) {
                    if (++LP.cnt >= LP.at) lp_count((lds_lp *)&LP, CX, (const lds_u64 *)R, slot, L.pc, L.fp, LP_ELIGIBLE, 0u);
                } else if (!L.done &&
                           lp_commit((lds_lp *)&LP, CX, (const lds_u64 *)R, slot, L.pc, L.fp, d.op, d.rd, d.rs1, d.rs2,
                                     d.flags, d.imm, lp_silent)) {
                    // the record of a hang at the cap
                    const uint64_t left = L.ninst < CX->hang_cap ? CX->hang_cap - L.ninst : 0;
                    proved_skip += left;
                    L.ninst += left;
                    finish(L, FI_HANG, 1, 0, 0u);
                }
            }
        } else {
        switch (f) {
        case F_SYSCALL: {   // SyscallFault::invokeSE advances the PC first (arch/riscv/faults.cc:325-333)
            if constexpr (kNL == 1) {
                if (LP.on) lp_fail((lds_lp *)&LP, CX);
            }
            L.pc = pc + d.len;
            // (out of line on copies: the interpreter's state stays in registers)
            Lane Ls = L;
            LaneMem ms = m;
            const bool chg = do_syscall<kNL>(CX, w, Ls, ms, slot, R, lane);
            L = Ls;
            m = ms;
            (void)chg;
            if constexpr (kNL == 1) {
                // the code mapping changed, or a proxy write (read, clock_gettime,
                // uname, ...) may have stored into cached code: forget the decodes
                for (uint32_t k = 0; k < kDC; k++) DCT[k] = 0xFFFFFFFFu;
                for (uint32_t k = 0; k < kSoloDC; k++) LC[4 * k] = 0xFFFFFFFFu;
            }
            break;
        }
        case F_BREAK: finish(L, FI_CRASH, FI_CRASH_SIGTRAP, 133, (uint32_t)pc); break;
        case F_ILLEGAL: finish(L, FI_CRASH, FI_CRASH_ILLEGAL_INST, 134, (uint32_t)pc); break;
        case F_UNKNOWN: finish(L, FI_CRASH, FI_CRASH_UNKNOWN_INST, 134, (uint32_t)pc); break;
        case F_ESCAPE: finish(L, FI_ESCAPE, FI_ESC_INST, 0, d.raw); break;
        case F_ESCCSR: finish(L, FI_ESCAPE, FI_ESC_CSR, 0, d.raw); break;
        case F_DETECT: finish(L, FI_DETECTED, 0, 0, (uint32_t)pc); break;
        case F_AMOLINE: finish(L, FI_CRASH, FI_CRASH_AMO_LINE, 134, (uint32_t)pc); break;
        case F_SCLINE: finish(L, FI_CRASH, FI_CRASH_SC_LINE, 134, (uint32_t)pc); break;
        case F_M5PANIC: finish(L, FI_CRASH, FI_CRASH_M5_PANIC, 134, (uint32_t)pc); break;
        case F_VSEW: finish(L, FI_CRASH, FI_CRASH_VSET_SEW, 134, (uint32_t)pc); break;
        case F_UNDEF: finish(L, FI_ESCAPE, FI_ESC_UNDEF, 0, d.raw); break;
        case F_TKCLOCK: finish(L, FI_ESCAPE, FI_ESC_TIMING, FI_TK_CLOCK, (uint32_t)pc); break;
        case F_PGFAULT: {   // GenericPageTableFault::invoke -> fixupFault (sim/faults.cc:95-105)
            int h;
            OOL(h = fixup_fault(CX, mc_, slot, fva));
            if (h == 0) finish(L, FI_CRASH, FI_CRASH_PAGE_FAULT, 134, (uint32_t)fva);
            else if (h == -1) finish(L, FI_CRASH, FI_CRASH_STACK_LIMIT, 1, (uint32_t)pc);
            else if (h == -2) finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, (uint32_t)pc);
            break;
        }
        default: break;
        }
        }   // fault disposition
        }   // f != F_NEEDPAGE
        }   // mine (commit)
        }   // execute
#ifdef FI_PROF
        if (!fast) PSTAMP(7);
#endif
        // ---- stay in the inner loop? every group lane committed, none reached
        // its next event, all at one PC that is still the wave's minimum
        const bool cont = mine && f == F_NONE && !L.done && L.ninst < next_ev;
        const uint64_t cm = wballot<kNL>(cont);
        if (cm != gmask) break;
        const uint64_t npc0 = uni64(rdl64<kNL>(L.pc, __ffsll((unsigned long long)cm) - 1));
        if (wballot<kNL>(cont && L.pc == npc0) != cm || npc0 >= wait_min) break;
        if (CX->wave_budget && n_iter + 1 >= CX->wave_budget) break;
        if (CX->pre_ok && !LP_ON) {   // back to the fast path (or translated blocks) when they can take the next one
            TextRef tn;
            tn.pre = CX->pre; tn.lo = (uint32_t)CX->text_lo; tn.hi = (uint32_t)(CX->text_lo >> 32);
            tn.bytes = CX->text_bytes; tn.clo = CX->code_lo; tn.chi = CX->code_hi;
            const PreRef En = pre_entry(tn, npc0);
            const uint32_t wn = uni32(En.e.w);
            // (solo: a lane in rewritten code goes back too; the pre-decoded
            // path decodes its own bytes through the decode cache)
            const bool dty = wballot<kNL>(cont && dirty_at(CX, m, npc0)) != 0;
            const bool lck = wballot<kNL>(cont && m.lock != kNone) != 0;
            if (!lck && En.in && ((wn >> 8) & kPreValid) &&
                ((kNL == 1 && dty) || (((wn >> 16) & 63) != K_SLOW && !dty)))
                break;
        }
        lpc = npc0;
        mine = cont;
        n_iter++;
        }   // inner loop
    }

    if (live && !suspended) CX->out[CX->record ? 0 : sidx] = L.res;
    if (CX->record && live) {
        CX->stats[3] = L.ncyc;
        CX->stats[4] = L.out_pos;
        CX->stats[5] = L.err_pos;
        CX->stats[13] = snaps_taken;
        CX->stats[15] = tpos;
    }
#ifdef FI_PROF
    if (lane == 0 && kSoloOnce)
        for (int k = 0; k < 8; k++) atomicAdd(&CX->stats[32 + k], (unsigned long long)pacc[k]);
#endif
    if (lane == 0 && CX->wave_dbg) {
        uint64_t *wd = CX->wave_dbg + 10 * ((uint64_t)blockIdx.x + rlo);   // (solo-odd: after the solo entries)
        wd[0] = __builtin_amdgcn_s_memtime() - t_start;
        wd[1] = n_iter;
        wd[2] = n_tx;
        wd[3] = n_slow | ((uint64_t)n_min << 32);         // slow fetches | min-PC reductions (solo: loop trips)
        wd[4] = rt_start;                                // s_memrealtime (100 MHz) at the wave's start / end
        wd[5] = __builtin_amdgcn_s_memrealtime();
        wd[6] = live ? (uint64_t)sidx : ~0ULL;           // lane 0's trial (index into the sites)
        wd[7] = live ? L.ninst - launch_inst - proved_skip : 0;   // lane 0's instructions in this dispatch
        wd[8] = n_txin;                                  // translated-code entries
        wd[9] = m.nmiss;                                 // lane 0's full page-table lookups
    }
    // the dispatch's busy span: waves that ran a trial (a surplus wave of a
    // resume grid returned above; one lane's vector atomics)
    if (CX->span && wballot<kNL>(live) != 0 && lane == 0) {
        atomicMin(&CX->span[0], (unsigned long long)rt_start);
        atomicMax(&CX->span[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
    if (blockIdx.x == 0 && lane == 0) {
        CX->stats[20] = __builtin_amdgcn_s_memtime() - t_start;
        CX->stats[21] = __builtin_amdgcn_s_memrealtime() - rt_start;
    }
    if (CX->record) pages_made = m.n_priv;   // golden: every private entry (pages, tombstones)
    const uint64_t fb = wsum64<kNL>(L.fetch_b), db = wsum64<kNL>(L.data_b), pm = wsum64<kNL>(pages_made);
    const uint64_t si = wsum64<kNL>(start_inst);
    const uint64_t xi = wsum64<kNL>(live ? L.ninst - launch_inst - proved_skip : 0);
    if (lane == 0 && kSoloOnce) {
        atomicAdd(&CX->stats[23], (unsigned long long)xi);
        atomicAdd(&CX->stats[0], (unsigned long long)fb);
        atomicAdd(&CX->stats[1], (unsigned long long)db);
        atomicAdd(&CX->stats[2], (unsigned long long)pm);
        {   // the same per kernel: 0 64-lane, 1 solo, 2 solo-odd (the bench's per-kernel roofline)
            constexpr uint32_t kk = kNL > 1 ? 0u : (kOdd ? 2u : 1u);
            atomicAdd(&CX->stats[40 + 4 * kk], (unsigned long long)fb);
            atomicAdd(&CX->stats[41 + 4 * kk], (unsigned long long)db);
            atomicAdd(&CX->stats[42 + 4 * kk], (unsigned long long)pm);
            atomicAdd(&CX->stats[43 + 4 * kk], (unsigned long long)xi);
        }
        atomicAdd(&CX->stats[6], (unsigned long long)n_iter);
        atomicAdd(&CX->stats[7], (unsigned long long)n_exec);
        atomicAdd(&CX->stats[8], (unsigned long long)n_slow);
        atomicAdd(&CX->stats[9], (unsigned long long)n_min);
        atomicMax(&CX->stats[10], (unsigned long long)n_iter);
        atomicAdd(&CX->stats[11], (unsigned long long)n_chk);
        atomicAdd(&CX->stats[12], (unsigned long long)n_early);
        atomicAdd(&CX->stats[14], (unsigned long long)si);
        atomicAdd(&CX->stats[16], (unsigned long long)n_tx);
        atomicAdd(&CX->stats[17], (unsigned long long)n_txin);
        atomicAdd(&CX->stats[24], (unsigned long long)n_simt);
        // the slowest wave: iterations, translated permille, entries (packed)
        atomicMax(&CX->stats[18], ((unsigned long long)n_iter << 32) |
                                      ((unsigned long long)(n_iter ? (uint64_t)n_tx * 1000 / n_iter : 0) << 20) |
                                      (n_txin < (1u << 20) ? n_txin : (1u << 20) - 1));
        atomicMax(&CX->stats[19], ((unsigned long long)n_iter << 32) | (n_slow < 0xFFFFFFFFu ? n_slow : 0xFFFFFFFFu));
#undef n_slow
#undef n_min
#undef n_exec
#undef n_chk
#undef n_early
#undef n_tx
#undef n_txin
#undef n_simt
    }
}

// The instantiations (load-time build: with the translated blocks).
// FI_TX_PART (fi_jit.cpp): 0 = every kernel in one module; k = only kernel k
// (1 the 64-lane, 2 the solo, 3 the solo-odd), one module each, built in
// parallel at load time.
#ifdef __HIPCC_RTC__
#ifndef FI_TX_PART
#define FI_TX_PART 0
#endif
#if FI_TX_PART == 0 || FI_TX_PART == 1
extern "C" __global__ void __launch_bounds__(64, FI_WAVES_PER_EU) fi_trial_kernel_tx(DevCtx) { trial_body<64>(); }
#endif
#if FI_TX_PART == 0 || FI_TX_PART == 2
extern "C" __global__ void __launch_bounds__(kSoloLanes, FI_SOLO_WAVES_PER_EU) fi_trial_kernel_tx_solo(DevCtx) { trial_body<1>(); }
#endif
#if defined(FI_TX_SOLO_ODD) && (FI_TX_PART == 0 || FI_TX_PART == 3)
extern "C" __global__ void __launch_bounds__(kSoloLanes, FI_SOLO_WAVES_PER_EU) fi_trial_kernel_tx_solo_odd(DevCtx) {
    trial_body<1, true>();
}
#endif
#else
__global__ void __launch_bounds__(64, FI_WAVES_PER_EU) fi_trial_kernel(DevCtx) { trial_body<64>(); }
__global__ void __launch_bounds__(kSoloLanes, FI_SOLO_WAVES_PER_EU) fi_trial_kernel_solo(DevCtx) { trial_body<1>(); }

hipError_t launch_trials(const DevCtx &c, hipStream_t st) {
    const uint32_t gl = (c.resume && c.resume_waves) ? 1u : c.lanes;   // grid for the fewest lanes per wave
    hipLaunchKernelGGL(fi_trial_kernel, dim3((unsigned)((c.n + gl - 1) / gl)), dim3(64), 0, st, c);
    return hipGetLastError();
}
// one trial per single-lane workgroup (surplus workgroups of a resume grid exit at once)
hipError_t launch_trials_solo(const DevCtx &c, hipStream_t st) {
    hipLaunchKernelGGL(fi_trial_kernel_solo, dim3((unsigned)c.n), dim3(kSoloLanes), 0, st, c);
    return hipGetLastError();
}

// Test hook (include/fi_debug.h fi_debug_loop_outcome): loop_outcome and the
// body's capped proof on synthetic loop records, one per lane, against the
// process-start page set (snapshot 0, no private pages, the start VMAs).
__global__ void __launch_bounds__(64) fi_debug_loop_kernel(DevCtx, const fi_debug_loop *in, uint64_t n,
                                                           fi_debug_loop_out *out) {
    KCtx *const kx = (KCtx *)__builtin_amdgcn_kernarg_segment_ptr();
    const uint64_t i = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    const fi_debug_loop *d = in + i;
    const SnapState *S0 = kx->snaps;
    WaveMem w;
    w.tab = kx->snap_tab + S0->tab_off;
    w.tab_n = S0->tab_n;
    LaneMem m;
    m.stack_min = S0->stack_min;
    tlb_flush(m);
    m.tp0 = m.tp1 = m.tp2 = m.tp3 = 0;
    m.tnext = 0; m.n_priv = 0; m.req_vpn = kNone; m.req_src = nullptr; m.code_dirty = false;
    m.dlo = m.dhi = 0; m.resv = m.lock = kNone; m.vm = false; m.vcfg = 0; m.nmiss = 0; m.dl = nullptr;
    uint64_t k = 0, fva = 0;
    const int r = loop_outcome(kx, w, m, 0, d->regs, d, d->left, k, fva);
    // the body's proof (TXHANG in solo_tx_clean_run) against hleft capped as the kernel caps it
    const uint32_t cnt = d->lp_cnt, cr = cnt & 0xFF, tr = (cnt >> 8) & 0xFF;
    const uint32_t hl = d->left > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d->left;
    const bool body = cr && d->lp_m && tx_hang_proof(d->regs[cr] - (tr ? d->regs[tr] : 0ULL),
                                                     (int)(int8_t)(uint8_t)(cnt >> 16), d->lp_m, hl);
    fi_debug_loop_out o;
    o.verdict = r; o.body_proof = body ? 1u : 0u; o.k = k; o.fva = fva;
    out[i] = o;
}
hipError_t launch_debug_loop(const DevCtx &c, const fi_debug_loop *in, uint64_t n, fi_debug_loop_out *out,
                             hipStream_t st) {
    hipLaunchKernelGGL(fi_debug_loop_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, c, in, n, out);
    return hipGetLastError();
}
#endif

}  // namespace fi
