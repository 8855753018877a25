// fi_kernels.hip -- CDNA4 (gfx950) kernels around the interpreter:
//
//   fi_sample_kernel    fault-site sampler: SplitMix64 keyed by (seed, trial)
//   fi_predecode_kernel decodes every halfword of the golden text once
//   fi_hist_kernel      outcome histogram (structure x first-bit x class)
//   hipcub radix sort   trials by inject time, so a wave's 64 lanes share the
//                       golden prefix and start at the same snapshot
//
// The interpreter itself (fi_trial_kernel) is in fi_trial.hip.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "fi_types.h"
#include "fi_device.h"
#include "rv64_isa.h"
#include "fi_softfp.h"
#include "fi_crypto.h"

namespace fi {

// SplitMix64 (Steele, Lea & Flood 2014)
__host__ __device__ inline uint64_t splitmix(uint64_t &s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// ------------------------------------------------------------------ sampler
__global__ void fi_sample_kernel(SampleCtx c, uint64_t n, fi_site *sites, uint64_t *keys, uint32_t *perm) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t id = c.first + i;
    uint64_t st = c.seed ^ (id * 0xD6E8FEB86659FD93ULL);
    const uint64_t r0 = splitmix(st), r1 = splitmix(st), r2 = splitmix(st), r3 = splitmix(st);
    fi_site s;
    s.inst = __umul64hi(r0, c.golden_ninst);
    uint64_t k = __umul64hi(r1, (uint64_t)c.n_struct);
    uint64_t m = c.structures;
    for (uint64_t j = 0; j < k; j++) m &= m - 1;
    s.target = (uint32_t)__builtin_ctzll(m);
    uint64_t b;
    if (c.bits == (c.burst == 1 ? ~0ULL : ((2ULL << (64 - c.burst)) - 1))) {
        b = __umul64hi(r2, (uint64_t)(65 - c.burst));   // every position
    } else {                                             // the k-th eligible position
        uint64_t mm = c.bits;
        const uint64_t kk = __umul64hi(r2, (uint64_t)__popcll(mm));
        for (uint64_t j = 0; j < kk; j++) mm &= mm - 1;
        b = (uint64_t)__builtin_ctzll(mm);
    }
    s.mask = (c.burst == 64 ? ~0ULL : ((1ULL << c.burst) - 1)) << b;
    s.addr = 0;
    if (s.target == FI_T_MEM) {
        const uint64_t w = __umul64hi(r3, c.n_mem_pages * 512);
        s.addr = c.mem_pages[w / 512] + (w % 512) * 8;
    }
    s.trial = (uint32_t)id;
    sites[i] = s;
    keys[i] = s.inst;
    perm[i] = (uint32_t)i;
}

__global__ void fi_keys_kernel(const fi_site *sites, uint64_t n, uint64_t *keys, uint32_t *perm) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keys[i] = sites[i].inst;
    perm[i] = (uint32_t)i;
}

// First-access forwarding.  A register site (x1..x31) at
// time t is injected at the golden run's next access of that register
// instead: the golden run neither reads nor writes it in between, so the
// trial's machine is the same.  Next access a write (or none): dead, the
// trial is the golden run.  A memory site likewise moves to the next golden
// access of any of its flipped bytes, if its page is mapped at t (present
// in the page table of the snapshot at or before t; the golden run maps and
// unmaps nothing) and it lies outside the text (fetches are not accesses);
// its dead case stays with the kernel (mem_dead).  Sort key = the effective
// time (dead: 0, they end at once).
__device__ __forceinline__ bool fw_mapped(const FwdCtx &c, uint64_t vpn, uint64_t t) {
    const uint64_t k = t / c.snap_interval;
    const SnapState &S = c.snaps[k < c.n_snap ? k : c.n_snap - 1];
    uint32_t lo = S.tab_off, hi = S.tab_off + S.tab_n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (c.snap_tab[mid].vpn < vpn) lo = mid + 1; else hi = mid;
    }
    return lo < S.tab_off + S.tab_n && c.snap_tab[lo].vpn == vpn;
}
__global__ void fi_forward_kernel(const fi_site *sites, uint64_t n, FwdCtx c, uint64_t *keys, uint64_t *eff) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const fi_site s = sites[i];
    uint64_t f = s.inst;
    if (s.target >= 1 && s.target <= 31 && s.inst < (1ULL << 29)) {
        const uint32_t key = (uint32_t)(4 * s.inst);   // (2t) << 1: before both events of numInst t
        uint32_t lo = c.reg_off[s.target], hi = c.reg_off[s.target + 1];
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (c.reg_ev[mid] < key) lo = mid + 1; else hi = mid;
        }
        f = (lo == c.reg_off[s.target + 1] || !(c.reg_ev[lo] & 1u)) ? kFwDead : (uint64_t)(c.reg_ev[lo] >> 2);
    } else if (s.target == FI_T_MEM && c.mw_n && !(s.addr < c.text_hi && s.addr + 8 > c.text_lo) &&
               fw_mapped(c, s.addr >> 12, s.inst)) {
        uint32_t fb = 0;
        for (int b = 0; b < 8; b++) fb |= ((s.mask >> (8 * b)) & 0xFF) ? (1u << b) : 0u;
        uint32_t lo = 0, hi = c.mw_n;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (c.mw_addr[mid] < s.addr) lo = mid + 1; else hi = mid;
        }
        if (lo < c.mw_n && c.mw_addr[lo] == s.addr) {
            uint32_t a = c.mw_off[lo], b = c.mw_off[lo + 1];
            const uint32_t e = b;
            while (a < b) {   // first event at numInst >= t
                const uint32_t mid = (a + b) >> 1;
                if ((c.mw_ev[mid] >> 16) < s.inst) a = mid + 1; else b = mid;
            }
            for (; a < e; a++) {
                const uint64_t ev = c.mw_ev[a];
                if (((ev >> 8) | ev) & fb & 0xFF) { f = ev >> 16; break; }
            }
        }
    }
    eff[i] = f;
    keys[i] = f == kFwDead ? 0 : f;
}

// ------------------------------------------------------------------ predecode
// One entry per halfword of [text_lo, text_hi).  Fetch follows
// Decoder::moreBytes (src/arch/riscv/decoder.cc:63-116): a 4-byte word at
// pc & ~3; pc % 4 != 0 takes its upper half; a 32-bit instruction starting in
// an upper half needs a second fetch tick (the "straddle").  Odd PCs behave
// like pc | 2 of the same word (handled by the caller's key computation).
__global__ void fi_predecode_kernel(const uint8_t *text, uint64_t code_off, uint64_t code_end, uint64_t nhalf,
                                    PreInst *pre) {
    const uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= nhalf) return;
    const uint64_t off = h * 2;
    const uint64_t bytes = nhalf * 2;
    PreInst p;
    p.flags = 0; p.aux = 0; p.raw = 0; p.op = OP_UNKNOWN; p.rd = p.rs1 = p.rs2 = 0; p.imm = 0; p.len = 2;
    uint32_t raw;
    bool straddle = false, ok = true;
    if ((off & 3) == 0) {
        raw = (uint32_t)text[off] | ((uint32_t)text[off + 1] << 8) | ((uint32_t)text[off + 2] << 16) |
              ((uint32_t)text[off + 3] << 24);
    } else {
        raw = (uint32_t)text[off] | ((uint32_t)text[off + 1] << 8);
        if ((raw & 3) == 3) {
            straddle = true;
            if (off + 4 > bytes) ok = false;   // second word outside the pre-decoded text
            else raw |= ((uint32_t)text[off + 2] << 16) | ((uint32_t)text[off + 3] << 24);
        }
    }
    // only instructions whose bytes lie inside the executable segments: a
    // lane's stores elsewhere in the text pages do not invalidate the table
    if (off < code_off || off + ((raw & 3) == 3 ? 4 : 2) > code_end) ok = false;
    if (ok) {
        Dec d = rv_decode(raw);
        const uint16_t u = uop_of(d);   // may normalise d.imm (c.zext.b/h, c.not)
        p.raw = d.raw; p.op = d.op; p.rd = d.rd; p.rs1 = d.rs1; p.rs2 = d.rs2; p.imm = d.imm; p.len = d.len;
        p.aux = u;
        p.flags = (uint8_t)(kPreValid | (straddle ? kPreStraddle : 0) | d.flags);
    }
    pre[h] = p;
}

// dispatch busy spans (DevCtx::span): every slot's min at ~0 (its max is zeroed by a memset)
__global__ void fi_span_init_kernel(unsigned long long *span, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) span[2 * i] = ~0ULL;
}
__global__ void fi_debug_decode_kernel(const uint32_t *raws, uint64_t n, PreInst *out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Dec d = rv_decode(raws[i]);
    PreInst p;
    p.raw = d.raw; p.op = d.op; p.rd = d.rd; p.rs1 = d.rs1; p.rs2 = d.rs2; p.imm = d.imm; p.len = d.len;
    p.aux = d.aux; p.flags = d.flags;
    out[i] = p;
}

// ------------------------------------------------------------------ histogram
// One trial per lane.  The [structure][bit][class] bins are scattered, so each
// lane adds its own bin; everything else is reduced in the wave first: the
// crash / escape sub-codes by ballot + popcount (one wave-uniform count per
// code), the trial and instruction totals by a DPP/shuffle sum, then one
// atomic per wave and counter.
__global__ void __launch_bounds__(256) fi_hist_kernel(const fi_site *sites, const fi_outcome *out, uint64_t n,
                                                      fi_histogram *h) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool v = i < n;
    uint32_t cls = FI_N_CLASS, sub = 0;
    uint64_t ninst = 0;
    if (v) {
        const fi_site s = sites[i];
        const fi_outcome o = out[i];
        const uint32_t t = s.target < FI_N_STRUCT ? s.target : 0;
        const uint32_t bit = s.mask ? (uint32_t)__builtin_ctzll(s.mask) : 0;
        cls = o.cls < FI_N_CLASS ? o.cls : FI_ESCAPE;
        sub = o.sub;
        ninst = o.ninst;
        atomicAdd((unsigned long long *)&h->counts[t][bit][cls], 1ULL);
    }
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t crash = __ballot(cls == FI_CRASH), esc = __ballot(cls == FI_ESCAPE);
    if (crash) {
        for (uint32_t k = 0; k < 16; k++) {
            const uint32_t c = (uint32_t)__popcll(crash & __ballot((sub & 15) == k));
            if (c && lane == 0) atomicAdd((unsigned long long *)&h->crash_sub[k], (unsigned long long)c);
        }
    }
    if (esc) {
        for (uint32_t k = 0; k < 8; k++) {
            const uint32_t c = (uint32_t)__popcll(esc & __ballot((sub & 7) == k));
            if (c && lane == 0) atomicAdd((unsigned long long *)&h->escape_sub[k], (unsigned long long)c);
        }
    }
    const uint64_t nt = (uint64_t)__popcll(__ballot(v)), ni = wave_sum64(ninst);
    if (lane == 0 && nt) {
        atomicAdd((unsigned long long *)&h->trials, (unsigned long long)nt);
        atomicAdd((unsigned long long *)&h->guest_insts, (unsigned long long)ni);
    }
}

// Epochs: sort keys of the suspended lanes (their pc: lanes of one loop end
// up in the same wave); entries past the survivor count sort last.
// Survivor sort key: pc offset from the text base (low 32 bits) above the
// low 32 bits of numInst, so that survivors standing at the same pc are
// adjacent and ordered by progress.  With n_odd (a solo-odd launch follows)
// the key is shifted down one bit under a top bit set for odd pcs, so that
// the odd-pc survivors sort last, and they are counted.
// solo != 0: the next epoch runs one trial per wave, where the order only
// decides when a trial starts: trials that rewrote their code (interpreted at
// ~20x the cost of translated code) start first, then the rest longest-first.
// The work-left estimate of a solo trial: the golden run's remaining length
// (the trial follows its path, the usual case: a wrong value carried to the
// end), or, when the trial stands in a counted loop of the golden text, that
// loop's remaining passes times its length if larger (a flipped bound, counter
// or pointer that stretches the loop: profiles/r05tl_solo_timeline_crc32.jsonl,
// the late starters); capped at the hang cap.
__device__ __forceinline__ uint64_t solo_work_left(const LaneSave &s, uint64_t text_lo, uint64_t golden_ninst,
                                                  const LoopEst *loops, uint32_t n_loops, uint64_t hang_cap) {
    uint64_t w = s.ninst < golden_ninst ? golden_ninst - s.ninst : 0;
    const uint64_t off = s.pc - text_lo;
    for (uint32_t i = 0; i < n_loops; i++) {
        const LoopEst L = loops[i];
        if (off < L.lo || off >= L.hi) continue;
        const uint64_t x = s.regs[L.reg] - (L.treg ? s.regs[L.treg] : 0ULL);
        const uint64_t d = L.step < 0 ? x : 0 - x;
        const uint32_t a = (uint32_t)(L.step < 0 ? -L.step : L.step);
        const uint64_t n = (d & (a - 1)) ? ~0ULL : (d / a ? d / a : ~0ULL);   // (fi_trial.hip loop_passes)
        const uint64_t e = n > (hang_cap / (L.m ? L.m : 1)) ? hang_cap : n * L.m;
        w = e > w ? e : w;
        break;
    }
    const uint64_t left = s.ninst < hang_cap ? hang_cap - s.ninst : 0;
    return w < left ? w : left;
}

__global__ void fi_surv_keys_kernel(const LaneSave *save, const uint32_t *list, const uint32_t *cnt, uint64_t cap,
                                    uint64_t text_lo, uint64_t *keys, uint32_t *vals, uint32_t *n_odd,
                                    uint32_t solo, uint64_t golden_ninst, uint32_t nb, const LoopEst *loops,
                                    uint32_t n_loops, uint64_t hang_cap) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cap) return;
    if (i < *cnt) {
        const uint32_t sl = list[i];
        const uint64_t pc = save[sl].pc;
        uint64_t k = ((pc - text_lo) << 32) | (save[sl].ninst & 0xFFFFFFFFu);
        // solo epoch: code-rewriting survivors and those already past the
        // golden run's end first (the first are interpreted, the second went
        // somewhere the golden run did not -- a re-run of the program, a loop
        // to the hang cap: profiles/r04v_solo_timeline_crc32.jsonl), then
        // longest-first -- the fewest committed instructions have the most
        // left to run (golden suffix or hang cap); one survivor per wave, so
        // no pc grouping (profiles/r03k_ab_lpt.jsonl: crc32 +4 %, intmix +5 %)
        if (solo) {
            const bool first = ((save[sl].flags >> 3) & 1) || save[sl].ninst > golden_ninst;
            // (solo bit 1: survivors not yet injected -- their outcome still
            // unknown -- form a tier of their own after the first)
            const bool uninj = (solo & 2u) && ((save[sl].flags >> 1) & 3) == 0;
            // (nb: the bits of the hang cap, above every survivor's numInst --
            // the key then sorts in nb + 2 (+ 1 odd) bits: fewer radix passes)
            // (tier 2: the most work left first, by the estimate below the cap)
            const uint64_t low = (first || uninj || !n_loops)
                                     ? save[sl].ninst
                                     : ((1ULL << nb) - 1) - solo_work_left(save[sl], text_lo, golden_ninst, loops,
                                                                          n_loops, hang_cap);
            k = ((uint64_t)(first ? 0 : uninj ? 1 : 2) << nb) | low;
        }
        if (n_odd) {
            k = solo ? (((pc & 1) << (nb + 2)) | k) : (((pc & 1) << 63) | (k >> 1));
            if (pc & 1) atomicAdd(n_odd, 1u);
        }
        keys[i] = k;
        vals[i] = sl;
    } else {
        keys[i] = ~0ULL;
        vals[i] = 0;
    }
}

// The solo kernel's share of a sorted survivor list whose odd-pc survivors
// come last: all but the last min(n_odd, grid), which the solo-odd kernel's
// grid takes.
__global__ void fi_odd_split_kernel(const uint32_t *cnt, const uint32_t *n_odd, uint32_t *split, uint32_t grid) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const uint32_t o = *n_odd < grid ? *n_odd : grid;
        *split = *cnt - o;
    }
}

// Packed resume: a wave starts at every sorted survivor whose pc differs from
// its predecessor's, and at every 64th position; it ends at the next start.
// Waves are numbered in atomic order (any order is correct: waves are
// independent).
__global__ void fi_pack_runs_kernel(const uint64_t *keys, const uint32_t *cnt, uint64_t cap, uint32_t *wrange,
                                    uint32_t *n_waves) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = *cnt;
    if (i >= n) return;
    const uint32_t pc = (uint32_t)(keys[i] >> 32);
    if (i != 0 && (i & 63) != 0 && (uint32_t)(keys[i - 1] >> 32) == pc) return;
    uint32_t e = (uint32_t)i + 1;
    while (e < n && (e & 63) != 0 && (uint32_t)(keys[e] >> 32) == pc) e++;
    const uint32_t w = atomicAdd(n_waves, 1u);
    wrange[2 * w] = (uint32_t)i;
    wrange[2 * w + 1] = e;
}

// Second pass of the trials that ran out of private pages (fi_engine.cpp
// chunk_begin / chunk_end): list them, gather their sites densely, scatter the new outcomes.
// (A resource escape with exit code 1 hit a table bound -- the VMA list, the
// getrandom stream -- that more pages would not lift: fi_trial.hip kEscTable.)
__global__ void fi_redo_collect_kernel(const fi_outcome *out, uint64_t n, uint32_t *idx, uint32_t *cnt,
                                       unsigned long long *stats) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const fi_outcome o = out[i];
    if (o.cls == FI_ESCAPE && o.sub == FI_ESC_RESOURCE && o.exit_code == 0) {
        idx[atomicAdd(cnt, 1u)] = (uint32_t)i;
        atomicAdd(&stats[30], 1ull);
    }
}
__global__ void fi_redo_gather_kernel(const fi_site *sites, const uint32_t *idx, uint64_t n, fi_site *rsites,
                                      uint64_t *keys, uint32_t *perm) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const fi_site s = sites[idx[j]];
    rsites[j] = s;
    keys[j] = s.inst;
    perm[j] = (uint32_t)j;
}
__global__ void fi_redo_scatter_kernel(const uint32_t *idx, uint64_t n, const fi_outcome *rout, fi_outcome *out) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) out[idx[j]] = rout[j];
}

__global__ void fi_hist_stats_kernel(const unsigned long long *stats, fi_histogram *h) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        h->fetch_bytes += stats[0];
        h->data_bytes += stats[1];
        h->cow_pages += stats[2];
        h->device_insts += stats[23];
    }
}

// ------------------------------------------------------------------ launch wrappers (host side)
static inline unsigned nblk(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

hipError_t launch_sample(const SampleCtx &c, uint64_t n, fi_site *sites, uint64_t *keys, uint32_t *perm,
                         hipStream_t st) {
    hipLaunchKernelGGL(fi_sample_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, c, n, sites, keys, perm);
    return hipGetLastError();
}
hipError_t launch_forward(const fi_site *sites, uint64_t n, const FwdCtx &c, uint64_t *keys, uint64_t *eff,
                          hipStream_t st) {
    hipLaunchKernelGGL(fi_forward_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, sites, n, c, keys, eff);
    return hipGetLastError();
}
hipError_t launch_keys(const fi_site *sites, uint64_t n, uint64_t *keys, uint32_t *perm, hipStream_t st) {
    hipLaunchKernelGGL(fi_keys_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, sites, n, keys, perm);
    return hipGetLastError();
}
hipError_t launch_predecode(const uint8_t *text, uint64_t code_off, uint64_t code_end, uint64_t nhalf, PreInst *pre,
                           hipStream_t st) {
    hipLaunchKernelGGL(fi_predecode_kernel, dim3(nblk(nhalf, 256)), dim3(256), 0, st, text, code_off, code_end, nhalf,
                       pre);
    return hipGetLastError();
}
hipError_t launch_span_init(unsigned long long *span, uint64_t n, hipStream_t st) {
    hipLaunchKernelGGL(fi_span_init_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, span, n);
    return hipGetLastError();
}
hipError_t launch_debug_decode(const uint32_t *raws, uint64_t n, PreInst *out, hipStream_t st) {
    hipLaunchKernelGGL(fi_debug_decode_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, raws, n, out);
    return hipGetLastError();
}
hipError_t launch_hist(const fi_site *sites, const fi_outcome *out, uint64_t n, fi_histogram *h,
                       const unsigned long long *stats, hipStream_t st) {
    hipLaunchKernelGGL(fi_hist_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, sites, out, n, h);
    if (stats) hipLaunchKernelGGL(fi_hist_stats_kernel, dim3(1), dim3(64), 0, st, stats, h);
    return hipGetLastError();
}
hipError_t launch_hist_stats(const unsigned long long *stats, fi_histogram *h, hipStream_t st) {
    hipLaunchKernelGGL(fi_hist_stats_kernel, dim3(1), dim3(64), 0, st, stats, h);
    return hipGetLastError();
}
hipError_t launch_redo_collect(const fi_outcome *out, uint64_t n, uint32_t *idx, uint32_t *cnt,
                               unsigned long long *stats, hipStream_t st) {
    hipLaunchKernelGGL(fi_redo_collect_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, out, n, idx, cnt, stats);
    return hipGetLastError();
}
hipError_t launch_redo_gather(const fi_site *sites, const uint32_t *idx, uint64_t n, fi_site *rsites, uint64_t *keys,
                              uint32_t *perm, hipStream_t st) {
    hipLaunchKernelGGL(fi_redo_gather_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, sites, idx, n, rsites, keys, perm);
    return hipGetLastError();
}
hipError_t launch_redo_scatter(const uint32_t *idx, uint64_t n, const fi_outcome *rout, fi_outcome *out,
                               hipStream_t st) {
    hipLaunchKernelGGL(fi_redo_scatter_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, idx, n, rout, out);
    return hipGetLastError();
}
hipError_t launch_surv_keys(const LaneSave *save, const uint32_t *list, const uint32_t *cnt, uint64_t cap,
                            uint64_t text_lo, uint64_t *keys, uint32_t *vals, uint32_t *n_odd, uint32_t solo,
                            uint64_t golden_ninst, uint32_t nb, const LoopEst *loops, uint32_t n_loops,
                            uint64_t hang_cap, hipStream_t st) {
    hipLaunchKernelGGL(fi_surv_keys_kernel, dim3(nblk(cap, 256)), dim3(256), 0, st, save, list, cnt, cap, text_lo,
                       keys, vals, n_odd, solo, golden_ninst, nb, loops, n_loops, hang_cap);
    return hipGetLastError();
}
hipError_t launch_odd_split(const uint32_t *cnt, const uint32_t *n_odd, uint32_t *split, uint32_t grid,
                            hipStream_t st) {
    hipLaunchKernelGGL(fi_odd_split_kernel, dim3(1), dim3(64), 0, st, cnt, n_odd, split, grid);
    return hipGetLastError();
}
hipError_t launch_pack_runs(const uint64_t *keys, const uint32_t *cnt, uint64_t cap, uint32_t *wrange,
                            uint32_t *n_waves, hipStream_t st) {
    hipLaunchKernelGGL(fi_pack_runs_kernel, dim3(nblk(cap, 256)), dim3(256), 0, st, keys, cnt, cap, wrange, n_waves);
    return hipGetLastError();
}
hipError_t sort_pairs_bytes(uint64_t n, size_t &bytes) {
    bytes = 0;
    return hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                              (const uint32_t *)nullptr, (uint32_t *)nullptr, (int)n);
}
hipError_t sort_pairs(void *tmp, size_t bytes, const uint64_t *kin, uint64_t *kout, const uint32_t *vin,
                      uint32_t *vout, uint64_t n, int end_bit, hipStream_t st) {
    return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, kin, kout, vin, vout, (int)n, 0, end_bit, st);
}

}  // namespace fi

// ------------------------------------------------------------------ FP port
// The engine's IEEE arithmetic (fi_softfp.h) run on vectors of operands, on
// the host or on the device, for the pinning tests against the reference's
// SoftFloat (tests/test_softfp.py).
namespace fi {
__global__ void softfp_kernel(int op, int fmt, int rm, const uint64_t *a, const uint64_t *b, const uint64_t *c,
                              uint64_t n, uint64_t *out, uint32_t *fl) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t f = 0;
    out[i] = sf::op(op, fmt, rm, a[i], b[i], c[i], f);
    fl[i] = f;
}
}  // namespace fi

extern "C" fi_status fi_debug_softfp(int op, int fmt, int rm, const uint64_t *a, const uint64_t *b,
                                     const uint64_t *c, uint64_t n, uint64_t *out, uint32_t *fl, int on_device) {
    if (op < 0 || op >= fi::sf::OP_COUNT || fmt < 0 || fmt > 2 || rm < 0 || rm > 4 || !a || !b || !c || !out || !fl)
        return FI_E_ARG;
    if (!on_device) {
        for (uint64_t i = 0; i < n; i++) {
            uint32_t f = 0;
            out[i] = fi::sf::op(op, fmt, rm, a[i], b[i], c[i], f);
            fl[i] = f;
        }
        return FI_OK;
    }
    if (!n) return FI_OK;
    uint64_t *d = nullptr;
    if (hipMalloc(&d, n * 8 * 4 + n * 4) != hipSuccess) return FI_E_HIP;
    uint64_t *da = d, *db = d + n, *dc = d + 2 * n, *dout = d + 3 * n;
    uint32_t *dfl = (uint32_t *)(d + 4 * n);
    hipError_t err = hipMemcpy(da, a, n * 8, hipMemcpyHostToDevice);
    if (err == hipSuccess) err = hipMemcpy(db, b, n * 8, hipMemcpyHostToDevice);
    if (err == hipSuccess) err = hipMemcpy(dc, c, n * 8, hipMemcpyHostToDevice);
    if (err == hipSuccess) {
        hipLaunchKernelGGL(fi::softfp_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, op, fmt, rm, da, db,
                           dc, n, dout, dfl);
        err = hipGetLastError();
    }
    if (err == hipSuccess) err = hipDeviceSynchronize();
    if (err == hipSuccess) err = hipMemcpy(out, dout, n * 8, hipMemcpyDeviceToHost);
    if (err == hipSuccess) err = hipMemcpy(fl, dfl, n * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return err == hipSuccess ? FI_OK : FI_E_HIP;
}

// ------------------------------------------------------------- crypto port
// The engine's scalar-crypto port (fi_crypto.h) over operand vectors, on the
// host or on the device, for the pinning test against the reference's rvk.hh
// (tests/test_crypto.py).
namespace fi {
__global__ void crypto_kernel(int fn, const uint64_t *a, const uint64_t *b, uint64_t n, uint64_t *out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = rvk::exec(fn, a[i], b[i]);
}
}  // namespace fi

extern "C" fi_status fi_debug_crypto(int fn, const uint64_t *a, const uint64_t *b, uint64_t n, uint64_t *out,
                                     int on_device) {
    if ((fn & 0xFF) > 21 || !a || !b || !out) return FI_E_ARG;
    if (!on_device) {
        for (uint64_t i = 0; i < n; i++) out[i] = fi::rvk::exec(fn, a[i], b[i]);
        return FI_OK;
    }
    if (!n) return FI_OK;
    uint64_t *d = nullptr;
    if (hipMalloc(&d, n * 8 * 3) != hipSuccess) return FI_E_HIP;
    hipError_t err = hipMemcpy(d, a, n * 8, hipMemcpyHostToDevice);
    if (err == hipSuccess) err = hipMemcpy(d + n, b, n * 8, hipMemcpyHostToDevice);
    if (err == hipSuccess) {
        hipLaunchKernelGGL(fi::crypto_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, fn, d, d + n, n,
                           d + 2 * n);
        err = hipGetLastError();
    }
    if (err == hipSuccess) err = hipDeviceSynchronize();
    if (err == hipSuccess) err = hipMemcpy(out, d + 2 * n, n * 8, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return err == hipSuccess ? FI_OK : FI_E_HIP;
}
