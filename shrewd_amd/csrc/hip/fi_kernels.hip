// fi_kernels.hip -- CDNA4 (gfx950) kernels of the fault-injection campaign.
//
//   fi_sample_kernel    fault-site sampler: SplitMix64 keyed by (seed, trial)
//   fi_predecode_kernel decodes every halfword of the golden text once
//   fi_trial_kernel     batched RV64 interpreter: one trial per lane, the
//                       AtomicSimpleCPU::tick loop (src/cpu/simple/atomic.cc:
//                       611-739) with the golden trace comparator and outcome
//                       classifier folded into the syscall/exit path
//   fi_hist_kernel      outcome histogram (structure x first-bit x class)
//
// Interpreter layout:
//   * one 64-lane wave = 64 trials sorted by inject time, so they share the
//     golden prefix and stay PC-converged; the wave picks a leader PC each
//     iteration (min-PC when lanes diverge) and executes it for every lane at
//     that PC, so fetch/decode and the op dispatch are wave-uniform (SALU +
//     s_load of a pre-decoded 16-byte entry);
//   * guest integer registers live in LDS as R[reg][lane] (8 B), so a
//     wave-uniform register index is one conflict-free ds_read_b64;
//   * guest memory: read-only golden frames + per-trial copy-on-write pages in
//     HBM, found through a 1-entry per-lane TLB, then a per-trial SoA page list
//     (coalesced), then a binary search of the golden page table; pages are
//     materialised by the whole wave cooperatively (16 B per lane per access).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "../fi_types.h"
#include "rv64_isa.h"

namespace fi {

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, l);
    uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t uni32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    return ((uint64_t)uni32((uint32_t)(v >> 32)) << 32) | uni32((uint32_t)v);
}
__device__ __forceinline__ uint64_t wave_min64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        uint64_t o = (uint64_t)__shfl_xor((unsigned long long)v, off, 64);
        v = o < v ? o : v;
    }
    return v;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += (uint64_t)__shfl_xor((unsigned long long)v, off, 64);
    return v;
}
__device__ __forceinline__ uint64_t sx32(uint64_t v) { return (uint64_t)(int64_t)(int32_t)(uint32_t)v; }
__device__ __forceinline__ int64_t sext64(uint64_t v, int n) { return (int64_t)(v << (64 - n)) >> (64 - n); }

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
    const uint64_t b = __umul64hi(r2, (uint64_t)(65 - c.burst));
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

// ------------------------------------------------------------------ predecode
// One entry per halfword of [text_lo, text_hi).  Fetch follows
// Decoder::moreBytes (src/arch/riscv/decoder.cc:63-116): a 4-byte word at
// pc & ~3; pc % 4 != 0 takes its upper half; a 32-bit instruction starting in
// an upper half needs a second fetch tick (the "straddle").  Odd PCs behave
// like pc | 2 of the same word (handled by the caller's key computation).
__global__ void fi_predecode_kernel(const uint8_t *text, uint64_t text_lo, uint64_t nhalf, PreInst *pre) {
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
    if (ok) {
        Dec d = rv_decode(raw);
        const uint16_t u = uop_of(d);   // may normalise d.imm (c.zext.b/h, c.not)
        p.raw = d.raw; p.op = d.op; p.rd = d.rd; p.rs1 = d.rs1; p.rs2 = d.rs2; p.imm = d.imm; p.len = d.len;
        p.aux = u;
        p.flags = (uint8_t)(kPreValid | (straddle ? kPreStraddle : 0) | d.flags);
    }
    pre[h] = p;
    (void)text_lo;
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

// ------------------------------------------------------------------ memory
struct LaneMem {
    uint64_t stack_min;
    uint64_t tlb_vpn;
    const uint8_t *tlb_page;
    uint64_t req_vpn;            // pending page materialisation, ~0 = none
    const uint8_t *req_src;
    uint32_t n_priv;
    bool tlb_w;
    bool code_dirty;
};

constexpr uint64_t kNone = ~0ULL;

__device__ __forceinline__ uint8_t *priv_frame(const DevCtx &c, uint64_t slot, uint32_t i) {
    return c.priv_frames + ((slot * c.priv_pages + i) << 12);
}

// 0 unmapped, 1 mapped read-only (golden frame or never-written stack page),
// 2 private (writable).  SE translation = EmulationPageTable::translate
// (src/mem/page_table.cc:143-153): the lane's page set is the process-start
// image + its private pages + the stack pages [stack_min, top] that
// MemState::fixupFault (src/sim/mem_state.cc:387-447) has mapped.
__device__ int lookup(const DevCtx &c, LaneMem &m, uint64_t slot, uint64_t vpn, const uint8_t *&page) {
    if (vpn == m.tlb_vpn) { page = m.tlb_page; return m.tlb_w ? 2 : 1; }
    int r = 0;
    for (uint32_t i = 0; i < m.n_priv; i++) {
        if (c.priv_vpn[(uint64_t)i * c.n + slot] == vpn) { page = priv_frame(c, slot, i); r = 2; break; }
    }
    if (!r) {
        uint32_t lo = 0, hi = c.n_base;
        while (lo < hi) {
            uint32_t mid = (lo + hi) >> 1;
            uint64_t v = c.base_vpn[mid];
            if (v < vpn) lo = mid + 1; else hi = mid;
        }
        if (lo < c.n_base && c.base_vpn[lo] == vpn) { page = c.frames + ((uint64_t)c.base_frame[lo] << 12); r = 1; }
    }
    if (!r && vpn >= (m.stack_min >> 12) && vpn <= kStackTopVpn) { page = c.zero_page; r = 1; }
    if (r) { m.tlb_vpn = vpn; m.tlb_page = page; m.tlb_w = (r == 2); }
    return r;
}

enum { F_NONE = 0, F_SYSCALL, F_BREAK, F_ILLEGAL, F_UNKNOWN, F_ESCAPE, F_ESCCSR, F_PGFAULT, F_NEEDPAGE, F_DETECT };

// AtomicSimpleCPU::readMem/writeMem (atomic.cc:331-544): the access is split
// at 64-byte line boundaries, each fragment translated on its own; faults are
// raised in fragment order.  Writes to a read-only (shared) page request a
// copy-on-write page first (not a gem5 event: the tick is retried).
__device__ int mem_access(const DevCtx &c, LaneMem &m, uint64_t slot, uint64_t ea, uint32_t size, bool wr,
                          uint64_t &val, uint64_t &fva) {
    uint32_t n1 = 64 - (uint32_t)(ea & 63);
    if (n1 > size) n1 = size;
    if (ea + n1 - 1 < ea) { fva = ea; return F_PGFAULT; }
    const uint8_t *p1 = nullptr, *p2 = nullptr;
    int k1 = lookup(c, m, slot, ea >> 12, p1);
    if (!k1) { fva = ea; return F_PGFAULT; }
    const uint64_t ea2 = ea + n1;
    int k2 = 2;
    if (n1 < size) {
        if (ea2 + (size - n1) - 1 < ea2) { fva = ea2; return F_PGFAULT; }
        k2 = lookup(c, m, slot, ea2 >> 12, p2);
        if (!k2) { fva = ea2; return F_PGFAULT; }
    }
    const uint32_t off = (uint32_t)(ea & 4095);
    if (wr) {
        if (k1 != 2) { m.req_vpn = ea >> 12; m.req_src = p1; return F_NEEDPAGE; }
        if (k2 != 2) { m.req_vpn = ea2 >> 12; m.req_src = p2; return F_NEEDPAGE; }
        uint8_t *w1 = const_cast<uint8_t *>(p1);
        if (n1 == size && (off & (size - 1)) == 0) {
            switch (size) {
            case 1: w1[off] = (uint8_t)val; break;
            case 2: *(uint16_t *)(w1 + off) = (uint16_t)val; break;
            case 4: *(uint32_t *)(w1 + off) = (uint32_t)val; break;
            default: *(uint64_t *)(w1 + off) = val; break;
            }
        } else {
            uint8_t *w2 = const_cast<uint8_t *>(p2);
            for (uint32_t i = 0; i < size; i++) {
                const uint64_t a = ea + i;
                uint8_t *pg = i < n1 ? w1 : w2;
                pg[a & 4095] = (uint8_t)(val >> (8 * i));
            }
        }
    } else {
        uint64_t v = 0;
        if (n1 == size && (off & (size - 1)) == 0) {
            switch (size) {
            case 1: v = p1[off]; break;
            case 2: v = *(const uint16_t *)(p1 + off); break;
            case 4: v = *(const uint32_t *)(p1 + off); break;
            default: v = *(const uint64_t *)(p1 + off); break;
            }
        } else {
            for (uint32_t i = 0; i < size; i++) {
                const uint64_t a = ea + i;
                const uint8_t *pg = i < n1 ? p1 : p2;
                v |= (uint64_t)pg[a & 4095] << (8 * i);
            }
        }
        val = v;
    }
    return F_NONE;
}

// Fast-path translation: succeeds only if every fragment's page is mapped and,
// for a store, already private -- anything else is left to the general path.
__device__ __forceinline__ bool mem_probe(const DevCtx &c, LaneMem &m, uint64_t slot, uint64_t ea, uint32_t size,
                                          bool wr, const uint8_t *&p1, const uint8_t *&p2, uint32_t &n1) {
    n1 = 64 - (uint32_t)(ea & 63);
    if (n1 > size) n1 = size;
    if (ea + size - 1 < ea) return false;
    const int k1 = lookup(c, m, slot, ea >> 12, p1);
    if (!k1 || (wr && k1 != 2)) return false;
    p2 = p1;
    if (n1 < size) {
        const int k2 = lookup(c, m, slot, (ea + n1) >> 12, p2);
        if (!k2 || (wr && k2 != 2)) return false;
    }
    return true;
}

// Slow-path fetch of one lane: Decoder::moreBytes + setupFetchRequest
// (src/arch/riscv/decoder.cc:63-116, src/cpu/simple/base.cc:304-318).
// Returns 0 ok, or F_PGFAULT with the faulting fetch address and the number of
// ticks consumed (1 if the first word faulted, 2 if the second did).
__device__ int fetch_lane(const DevCtx &c, LaneMem &m, uint64_t slot, uint64_t pc, uint32_t &raw, uint32_t &ticks,
                          uint64_t &fva) {
    const uint64_t w0 = pc & ~3ULL;
    const uint8_t *pg;
    ticks = 1;
    if (!lookup(c, m, slot, w0 >> 12, pg)) { fva = w0; return F_PGFAULT; }
    const uint32_t word = *(const uint32_t *)(pg + (w0 & 4095));
    if ((pc & 3) == 0) {
        raw = ((word & 3) != 3) ? (word & 0xFFFF) : word;
        return F_NONE;
    }
    const uint32_t half = word >> 16;
    if ((half & 3) != 3) { raw = half; return F_NONE; }
    ticks = 2;
    const uint64_t w1 = w0 + 4;
    if (!lookup(c, m, slot, w1 >> 12, pg)) { fva = w1; return F_PGFAULT; }
    const uint32_t word2 = *(const uint32_t *)(pg + (w1 & 4095));
    raw = half | ((word2 & 0xFFFF) << 16);
    return F_NONE;
}

// ------------------------------------------------------------------ syscalls
// RV64 Linux SE syscall table classification (src/arch/riscv/linux/
// se_workload.cc:529-895); 0 absent, 1 unimplemented, 2 ignore, 3 escape,
// 4 modelled.
__device__ int sys_class(int num) {
    if (num == 64 || num == 93 || num == 94 || (num >= 172 && num <= 178)) return 4;
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
    int watch;
    bool out_bad, done;
    uint8_t injected;
    fi_outcome res;
};

__device__ __forceinline__ void finish(Lane &L, int cls, int sub, int code, uint32_t detail) {
    L.done = true;
    L.res.cls = (uint8_t)cls; L.res.sub = (uint8_t)sub; L.res.exit_code = (uint8_t)code;
    L.res.flags = (uint8_t)((L.injected ? 1 : 0) | (L.injected == 2 ? 2 : 0));
    L.res.detail = detail;
    L.res.ninst = L.ninst;
}

#define RREG(r) R[(uint32_t)(r) * 64u + lane]

// Diagnostic build only (-DFI_STAMPS): per-wave cycle accounting of the loop
// segments with s_memtime (never compiled into the shipped library).
#ifdef FI_STAMPS
#define STAMP(k)                                                  \
    do {                                                          \
        __builtin_amdgcn_sched_barrier(0);                        \
        const uint64_t _t = __builtin_amdgcn_s_memtime();         \
        __builtin_amdgcn_s_waitcnt(0xC07F);                       \
        tacc[k] += _t - tlast;                                    \
        tlast = _t;                                               \
        __builtin_amdgcn_sched_barrier(0);                        \
    } while (0)
#else
#define STAMP(k) do { } while (0)
#endif

// The syscall path of one lane: EmuLinux::syscall (se_workload.cc:95-106)
// with the golden-output comparator folded into write().
__device__ __forceinline__ void do_syscall(const DevCtx &c, Lane &L, LaneMem &m, uint64_t slot, uint64_t *R, uint32_t lane) {
    const int num = (int)(uint32_t)RREG(17);
    const int cls = sys_class(num);
    if (cls == 0) { finish(L, FI_CRASH, FI_CRASH_SYSCALL_RANGE, 1, (uint32_t)num); return; }
    if (cls == 1) { finish(L, FI_CRASH, FI_CRASH_SYSCALL_UNIMPL, 1, (uint32_t)num); return; }
    if (cls == 3) { finish(L, FI_ESCAPE, FI_ESC_SYSCALL, 0, (uint32_t)num); return; }
    if (cls == 2) { RREG(10) = 0; return; }
    switch (num) {
    case 93: case 94: {  // exitImpl -> exitSimLoop(status & 0xff), sim/syscall_emul.cc:120-248
        const int code = (int)(uint32_t)RREG(10) & 0xff;
        if (c.record) {
            finish(L, FI_MASKED, 0, code, (uint32_t)L.pc);
            return;
        }
        const bool same = !L.out_bad && L.out_pos == c.gout_len && L.err_pos == c.gerr_len && code == (int)c.gexit;
        finish(L, same ? FI_MASKED : FI_SDC, 0, code, (uint32_t)L.pc);
        return;
    }
    case 172: case 178: RREG(10) = kPid; return;
    case 173: RREG(10) = kPpid; return;
    case 174: case 175: RREG(10) = kUid; return;
    case 176: case 177: RREG(10) = kGid; return;
    default: break;   // 64: write
    }
    // writeFunc (src/sim/syscall_emul.hh:2826-2860): int fd, buffer copied in
    // through a non-allocating proxy (fatal on an unmapped byte), then compared
    // with the golden stream at the current position.
    const int fd = (int)(uint32_t)RREG(10);
    const uint64_t buf = RREG(11), n = RREG(12);
    if (fd < 0 || fd >= 1024) { finish(L, FI_CRASH, FI_CRASH_FD_ASSERT, 134, (uint32_t)L.pc); return; }
    if (fd == 0) { finish(L, FI_ESCAPE, FI_ESC_HOST, 0, (uint32_t)L.pc); return; }
    if (fd > 2) { RREG(10) = (uint64_t)(int64_t)-9; return; }
    if (n > (1ULL << 31)) { finish(L, FI_ESCAPE, FI_ESC_HOST, 0, (uint32_t)L.pc); return; }
    if (n) {
        const uint64_t last = buf + n - 1;
        if (last < buf) { finish(L, FI_CRASH, FI_CRASH_PROXY, 1, (uint32_t)L.pc); return; }
        const uint8_t *pg;
        for (uint64_t v = buf >> 12; v <= (last >> 12); v++) {
            if (!lookup(c, m, slot, v, pg)) { finish(L, FI_CRASH, FI_CRASH_PROXY, 1, (uint32_t)L.pc); return; }
        }
        uint64_t &pos = fd == 1 ? L.out_pos : L.err_pos;
        const uint8_t *gold = fd == 1 ? c.gout : c.gerr;
        const uint64_t glen = fd == 1 ? c.gout_len : c.gerr_len;
        uint8_t *rec = fd == 1 ? c.rec_out : c.rec_err;
        uint64_t cur_vpn = kNone;
        for (uint64_t i = 0; i < n; i++) {
            const uint64_t a = buf + i;
            if ((a >> 12) != cur_vpn) { cur_vpn = a >> 12; lookup(c, m, slot, cur_vpn, pg); }
            const uint8_t ch = pg[a & 4095];
            const uint64_t p = pos + i;
            if (c.record) {
                if (p < c.rec_cap) rec[p] = ch;
            } else if (p >= glen || gold[p] != ch) {
                L.out_bad = true;
            }
        }
        pos += n;
    }
    RREG(10) = n;
}

// ------------------------------------------------------------------ trial kernel
__global__ void __launch_bounds__(64) fi_trial_kernel(DevCtx c) {
    __shared__ uint64_t R[32 * 64];
    const uint32_t lane = threadIdx.x;
    const uint64_t slot = (uint64_t)blockIdx.x * 64 + lane;
    const bool live = slot < c.n;
    fi_site s;
    s.inst = kNone; s.mask = 0; s.addr = 0; s.target = 0; s.trial = 0;
    uint32_t sidx = 0;
    if (live && !c.record) { sidx = c.perm[slot]; s = c.sites[sidx]; }
#pragma unroll
    for (int r = 0; r < 32; r++) RREG(r) = 0;
    RREG(2) = c.sp0;

    Lane L;
    L.pc = c.entry; L.ninst = 0; L.ncyc = 0; L.out_pos = L.err_pos = 0; L.fetch_b = L.data_b = 0;
    L.watch = -1; L.out_bad = false; L.done = !live; L.injected = (c.record || !live) ? 1 : 0;
    L.res.cls = 0; L.res.sub = 0; L.res.exit_code = 0; L.res.flags = 0; L.res.detail = 0; L.res.ninst = 0;
    LaneMem m;
    m.stack_min = c.stack_min0; m.tlb_vpn = kNone; m.tlb_page = nullptr; m.req_vpn = kNone; m.req_src = nullptr;
    m.n_priv = 0; m.tlb_w = false; m.code_dirty = false;
    uint64_t pages_made = 0;
    uint32_t n_iter = 0, n_slow = 0, n_min = 0, n_exec = 0;   // per-wave loop counters (uniform)
#ifdef FI_STAMPS
    uint64_t tacc[6] = {0, 0, 0, 0, 0, 0};
    uint64_t tlast = __builtin_amdgcn_s_memtime();
#endif

    for (;;) {
        // ---- A. materialise requested pages, whole wave cooperating
        uint64_t want = __ballot(!L.done && m.req_vpn != kNone);
        if (want) {
            uint64_t w = want;
            while (w) {
                const int l = __ffsll((unsigned long long)w) - 1;
                w &= w - 1;
                const uint32_t np = (uint32_t)__builtin_amdgcn_readlane((int)m.n_priv, l);
                if (np >= c.priv_pages) continue;
                const uint64_t lslot = readlane64(slot, l);
                const uint4 *src = (const uint4 *)readlane64((uint64_t)m.req_src, l);
                uint4 *dst = (uint4 *)priv_frame(c, lslot, np);
#pragma unroll
                for (int k = 0; k < 4; k++) dst[lane + 64 * k] = src[lane + 64 * k];
            }
            __syncthreads();
            if (!L.done && m.req_vpn != kNone) {
                if (m.n_priv >= c.priv_pages) {
                    finish(L, FI_ESCAPE, FI_ESC_RESOURCE, 0, (uint32_t)L.pc);
                } else {
                    c.priv_vpn[(uint64_t)m.n_priv * c.n + slot] = m.req_vpn;
                    if ((m.req_vpn << 12) >= c.text_lo && (m.req_vpn << 12) < c.text_hi) m.code_dirty = true;
                    m.n_priv++;
                    pages_made++;
                }
                m.req_vpn = kNone;
                m.tlb_vpn = kNone;
            }
        }
        STAMP(0);
        // ---- B. tick-top events: fault injection and the max-insts (hang)
        // exit both fire in serviceInstCountEvents at the first tick with
        // numInst >= n (src/cpu/simple/base.cc:321-325, src/cpu/base.cc:764-770)
        if (!L.done && !L.injected && L.ninst >= s.inst) {
            if (s.target >= 1 && s.target <= 31) {
                RREG(s.target) ^= s.mask;
                if ((c.protect_mask >> s.target) & 1) L.watch = (int)s.target;
                L.injected = 1;
            } else if (s.target == FI_T_PC) {
                L.pc ^= s.mask;
                L.injected = 1;
                if ((c.protect_mask >> 32) & 1) finish(L, FI_DETECTED, 0, 0, (uint32_t)L.pc);
            } else if (s.target == FI_T_MEM) {
                const uint8_t *pg;
                const int k = lookup(c, m, slot, s.addr >> 12, pg);
                if (k == 0) {
                    L.injected = 2;    // page not mapped at t: nothing to flip
                } else if (k == 1) {
                    m.req_vpn = s.addr >> 12; m.req_src = pg;   // copy-on-write first, flip next iteration
                } else {
                    uint64_t *wp = (uint64_t *)(const_cast<uint8_t *>(pg) + (s.addr & 4095));
                    *wp ^= s.mask;
                    L.injected = 1;
                }
            } else {
                L.injected = 1;
            }
        }
        if (!L.done && L.ninst >= c.hang_cap) finish(L, FI_HANG, 1, 0, (uint32_t)L.pc);

        const bool ready = !L.done && m.req_vpn == kNone;
        const uint64_t act = __ballot(ready);
        if (act == 0) {
            if (__ballot(!L.done) == 0) break;
            continue;
        }
        STAMP(1);
        // ---- C. leader PC: first ready lane, or min-PC if the lanes diverged
        const int leader = __ffsll((unsigned long long)act) - 1;
        uint64_t lpc = readlane64(L.pc, leader);
        n_iter++;
        if (__ballot(ready && L.pc == lpc) != act) { lpc = wave_min64(ready ? L.pc : kNone); n_min++; }
        lpc = uni64(lpc);   // wave-uniform: keeps fetch/decode/dispatch on the scalar unit
        bool mine = ready && L.pc == lpc;
        // lanes of other groups wait; the group keeps the wave only while its PC
        // stays below theirs (min-PC order, so groups merge when they meet)
        const uint64_t wait_min = (__ballot(mine) != act) ? uni64(wave_min64((ready && !mine) ? L.pc : kNone)) : kNone;
        // next instruction-count event of this lane (injection or hang cap)
        const uint64_t next_ev = (!L.injected && s.inst < c.hang_cap) ? s.inst : c.hang_cap;

        // ---- FAST PATH: the group is converged on golden text with nothing
        // watched or modified -- run pre-decoded micro-ops with PC, instruction,
        // cycle and byte counts in SGPRs until an event is due, the group
        // diverges, meets another group, or hits something the general path owns
        // (K_SLOW op, fault, page request, syscall).  Nothing commits unless the
        // whole instruction commits for every group lane.
        if (lpc >= c.text_lo && lpc < c.text_hi && __ballot(mine && (m.code_dirty || L.watch > 0)) == 0) {
            const uint64_t gm = __ballot(mine);
            const int glane = __ffsll((unsigned long long)gm) - 1;
            const uint64_t budget = uni64(wave_min64(mine ? next_ev - L.ninst : kNone));
            uint64_t spc = lpc, steps = 0, cyc = 0, fbytes = 0, dbytes = 0;
            bool div = false;
            typedef __attribute__((address_space(4))) const uint32_t const_u32;
            for (;;) {
                spc = uni64(spc);   // keep the guest PC in SGPRs: s_load of the entry, scalar dispatch
                const uint64_t key = (spc & 3) ? ((spc & ~3ULL) | 2) : spc;
                if (key < c.text_lo || key >= c.text_hi) break;
                const const_u32 *q = (const const_u32 *)(uintptr_t)(c.pre + ((key - c.text_lo) >> 1));
                const uint32_t q1 = uni32(q[1]), q2 = uni32(q[2]), q3 = uni32(q[3]);
                const uint32_t aux = q3 >> 16, kind = aux & 63;
                if (!((q3 >> 8) & kPreValid) || kind == K_SLOW) break;
                const uint32_t rd = q1 >> 8 & 0xFF, rs1 = q1 >> 16 & 0xFF, rs2 = q1 >> 24;
                const int64_t imm = (int32_t)q2;
                const uint32_t len = q3 & 0xFF, ticks = ((q3 >> 8) & kPreStraddle) ? 2 : 1;
                const uint64_t a0 = RREG(rs1), b0 = RREG(rs2);
                const uint64_t av = (aux & U_APC) ? spc : a0;
                const uint64_t bv = (aux & U_BIMM) ? (uint64_t)imm : b0;
                const bool w32 = aux & U_W32;
                const uint32_t shm = w32 ? 31 : 63;
                uint64_t v = 0, npc = spc + len;
                uint32_t msz = 0;
                bool wr = true;
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
                case K_NOP: wr = false; break;
                case K_JAL: v = npc; npc = spc + imm; break;
                case K_JALR: {
                    v = npc;
                    const uint64_t t = (a0 + imm) & ~1ULL;
                    const uint64_t t0 = readlane64(t, glane);
                    if (__ballot(mine && t != t0) == 0) npc = uni64(t0);
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
                    const uint64_t tk = __ballot(mine && cnd);
                    if (tk == gm) npc = spc + imm;
                    else if (tk != 0) { div = true; if (mine) L.pc = cnd ? spc + imm : npc; }
                    break;
                }
                default: {   // K_LOAD / K_STORE
                    const bool st = kind == K_STORE;
                    msz = 1u << ((aux >> 12) & 3);
                    const uint64_t ea = a0 + imm;
                    const uint8_t *p1 = nullptr, *p2 = nullptr;
                    uint32_t n1 = 0;
                    bool ok = true;
                    if (mine) ok = mem_probe(c, m, slot, ea, msz, st, p1, p2, n1);
                    if (__ballot(mine && !ok) != 0) { msz = 0xFFFFFFFFu; break; }   // bail: general path
                    if (mine) {
                        const uint32_t off = (uint32_t)(ea & 4095);
                        if (st) {
                            uint8_t *w1 = const_cast<uint8_t *>(p1);
                            if (n1 == msz && (off & (msz - 1)) == 0) {
                                switch (msz) {
                                case 1: w1[off] = (uint8_t)b0; break;
                                case 2: *(uint16_t *)(w1 + off) = (uint16_t)b0; break;
                                case 4: *(uint32_t *)(w1 + off) = (uint32_t)b0; break;
                                default: *(uint64_t *)(w1 + off) = b0; break;
                                }
                            } else {
                                uint8_t *w2 = const_cast<uint8_t *>(p2);
                                for (uint32_t i = 0; i < msz; i++) (i < n1 ? w1 : w2)[(ea + i) & 4095] = (uint8_t)(b0 >> (8 * i));
                            }
                        } else {
                            uint64_t t = 0;
                            if (n1 == msz && (off & (msz - 1)) == 0) {
                                switch (msz) {
                                case 1: t = p1[off]; break;
                                case 2: t = *(const uint16_t *)(p1 + off); break;
                                case 4: t = *(const uint32_t *)(p1 + off); break;
                                default: t = *(const uint64_t *)(p1 + off); break;
                                }
                            } else {
                                for (uint32_t i = 0; i < msz; i++) t |= (uint64_t)(i < n1 ? p1 : p2)[(ea + i) & 4095] << (8 * i);
                            }
                            v = (aux & U_SEXT) ? (uint64_t)sext64(t, 8 * msz) : t;
                        }
                    }
                    if (st) wr = false;
                    break;
                }
                }
                if (msz == 0xFFFFFFFFu) break;            // nothing committed for this instruction
                if (w32) v = sx32(v);
                if (wr && rd && mine) RREG(rd) = v;
                steps++; cyc += ticks; fbytes += len; dbytes += msz;
                if (div) break;
                spc = npc;
                if (steps >= budget || spc >= wait_min) break;
            }
            if (steps) {
                if (mine) {
                    L.ninst += steps; L.ncyc += cyc; L.fetch_b += fbytes; L.data_b += dbytes;
                    if (!div) L.pc = spc;
                }
                n_iter += (uint32_t)steps;
                n_exec += (uint32_t)(steps * __popcll(gm));
                continue;
            }
        }

        // ---- inner loop: one guest instruction per iteration while the group
        // stays converged, with no event due and no page request pending
        for (;;) {
        STAMP(2);
        // ---- D. fetch + decode (wave-uniform)
        Dec d;
        uint32_t ticks = 1;
        bool fast = false;
        const uint64_t key = (lpc & 3) ? ((lpc & ~3ULL) | 2) : lpc;
        if (key >= c.text_lo && key < c.text_hi && __ballot(mine && m.code_dirty) == 0) {
            // one s_load_dwordx4 through the constant address space: the
            // pre-decoded table is read-only for the whole launch
            typedef __attribute__((address_space(4))) const uint32_t const_u32;
            const const_u32 *q = (const const_u32 *)(uintptr_t)(c.pre + ((key - c.text_lo) >> 1));
            const uint32_t q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
            const uint32_t pflags = (q3 >> 8) & 0xFF;
            if (pflags & kPreValid) {
                fast = true;
                d.raw = q0; d.op = (uint8_t)q1; d.rd = (uint8_t)(q1 >> 8); d.rs1 = (uint8_t)(q1 >> 16);
                d.rs2 = (uint8_t)(q1 >> 24); d.imm = (int32_t)q2; d.len = (uint8_t)q3;
                d.flags = (uint8_t)pflags; d.aux = (uint16_t)(q3 >> 16);
                ticks = (pflags & kPreStraddle) ? 2 : 1;
            }
        }
        if (!fast) {
            n_slow++;
            uint32_t raw = 0, t = 1;
            uint64_t fva = 0;
            if (mine) {
                const int fr = fetch_lane(c, m, slot, L.pc, raw, t, fva);
                if (fr) {
                    // the faulting tick(s) count, nothing commits; decoder reset;
                    // GenericPageTableFault::invoke -> fixupFault (sim/faults.cc:95-105)
                    L.ncyc += t;
                    mine = false;
                    if (fva < m.stack_min && fva >= kStackBase - kMaxStack) {
                        const uint64_t nm = fva & ~4095ULL;
                        if (kStackBase - nm > kMaxStack) finish(L, FI_CRASH, FI_CRASH_STACK_LIMIT, 1, (uint32_t)L.pc);
                        else { m.stack_min = nm; m.tlb_vpn = kNone; }
                    } else {
                        finish(L, FI_CRASH, FI_CRASH_PAGE_FAULT, 134, (uint32_t)fva);
                    }
                }
            }
            const uint64_t okm = __ballot(mine);
            if (okm == 0) break;
            const int ld = __ffsll((unsigned long long)okm) - 1;
            const uint32_t lraw = (uint32_t)__builtin_amdgcn_readlane((int)raw, ld);
            const uint32_t lt = (uint32_t)__builtin_amdgcn_readlane((int)t, ld);
            mine = mine && raw == lraw;
            d = rv_decode(lraw);
            ticks = lt;
        }
        // force every decoded field into SGPRs: the op switch below must be a
        // scalar branch tree, never a per-lane waterfall
        d.op = (uint8_t)uni32(d.op); d.rd = (uint8_t)uni32(d.rd); d.rs1 = (uint8_t)uni32(d.rs1);
        d.rs2 = (uint8_t)uni32(d.rs2); d.len = (uint8_t)uni32(d.len); d.flags = (uint8_t)uni32(d.flags);
        d.imm = (int32_t)uni32((uint32_t)d.imm); d.aux = (uint16_t)uni32(d.aux); d.raw = uni32(d.raw);
        ticks = uni32(ticks);
        const uint64_t gmask = __ballot(mine);
        n_exec += (uint32_t)__popcll(gmask);
        STAMP(3);
        int f = F_NONE;
        if (mine) {
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
        // detected-by-replica: the flipped protected register is read before
        // being overwritten (build-defined SHREWD semantics)
        if (L.watch > 0 &&
            (((d.flags & kPreRs1) && d.rs1 == L.watch) || ((d.flags & kPreRs2) && d.rs2 == L.watch) ||
             (d.op == OP_ecall && (L.watch == 17 || (L.watch >= 10 && L.watch <= 15))))) {
            f = F_DETECT;
        } else {
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
            case OP_orc_b: {
                v = 0;
#pragma unroll
                for (int i = 0; i < 8; i++) if ((a >> (8 * i)) & 0xFF) v |= 0xFFULL << (8 * i);
                break;
            }
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
            case OP_clmul: { v = 0; for (int i = 0; i < 64; i++) if ((b >> i) & 1) v ^= a << i; break; }
            case OP_bset: v = a | (1ULL << (b & 63)); break;
            case OP_bclr: v = a & ~(1ULL << (b & 63)); break;
            case OP_rol: { const int sh = (int)(b & 63); v = (a << sh) | (a >> ((64 - sh) & 63)); break; }
            case OP_binv: v = a ^ (1ULL << (b & 63)); break;
            case OP_slt: v = (int64_t)a < (int64_t)b ? 1 : 0; break;
            case OP_mulhsu: v = __umul64hi(a, b) - (((int64_t)a < 0) ? b : 0); break;
            case OP_clmulr: { v = 0; for (int i = 0; i < 64; i++) if ((b >> i) & 1) v ^= a >> (63 - i); break; }
            case OP_sh1add: v = (a << 1) + b; break;
            case OP_sltu: v = a < b ? 1 : 0; break;
            case OP_mulhu: v = __umul64hi(a, b); break;
            case OP_clmulh: { v = 0; for (int i = 1; i < 64; i++) if ((b >> i) & 1) v ^= a >> (64 - i); break; }
            case OP_div_: {
                const int64_t x = (int64_t)a, y = (int64_t)b;
                v = y == 0 ? ~0ULL : (x == INT64_MIN && y == -1) ? (uint64_t)x : (uint64_t)(x / y);
                break;
            }
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
            case OP_rem: {
                const int64_t x = (int64_t)a, y = (int64_t)b;
                v = y == 0 ? a : (x == INT64_MIN && y == -1) ? 0 : (uint64_t)(x % y);
                break;
            }
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
            case OP_rolw: { const uint32_t x = (uint32_t)a; const int sh = (int)(b & 31); v = sx32((x << sh) | (x >> ((32 - sh) & 31))); break; }
            case OP_sh1add_uw: v = ((a & 0xFFFFFFFFULL) << 1) + b; break;
            case OP_divw: {
                const int32_t x = (int32_t)a, y = (int32_t)b;
                const int32_t q = y == 0 ? -1 : (x == INT32_MIN && y == -1) ? x : x / y;
                v = (uint64_t)(int64_t)q;
                break;
            }
            case OP_packw: v = sx32(((b & 0xFFFF) << 16) | (a & 0xFFFF)); break;
            case OP_sh2add_uw: v = ((a & 0xFFFFFFFFULL) << 2) + b; break;
            case OP_srlw: v = sx32((uint32_t)a >> (b & 31)); break;
            case OP_divuw: v = (uint32_t)b == 0 ? ~0ULL : sx32((uint32_t)a / (uint32_t)b); break;
            case OP_sraw: v = (uint64_t)(int64_t)((int32_t)(uint32_t)a >> (b & 31)); break;
            case OP_rorw: { const uint32_t x = (uint32_t)a; const int sh = (int)(b & 31); v = sx32((x >> sh) | (x << ((32 - sh) & 31))); break; }
            case OP_remw: {
                const int32_t x = (int32_t)a, y = (int32_t)b;
                const int32_t r = y == 0 ? x : (x == INT32_MIN && y == -1) ? 0 : x % y;
                v = (uint64_t)(int64_t)r;
                break;
            }
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
            case OP_csr: f = csr_u_accessible(d.raw >> 20) ? F_ESCCSR : F_ILLEGAL; break;
            default: f = F_UNKNOWN; break;
            }
        }
        STAMP(4);
        if (msz && f == F_NONE) {
            t = b;
            f = mem_access(c, m, slot, a + imm, msz, mst, t, fva);
            L.data_b += msz;
            if (!mst) v = mext ? (uint64_t)sext64(t, mext) : t;
        }
        STAMP(5);
        // F_NEEDPAGE: copy-on-write first; the tick is retried (no commit)
        // ---- F. commit: countInst only on NoFault (atomic.cc:687-689), then
        // advancePC (src/cpu/simple/base.cc:493-512)
        if (f != F_NEEDPAGE) {
        L.ncyc += ticks;
        L.fetch_b += d.len;
        if (f == F_NONE) {
            if (wrd && d.rd) RREG(d.rd) = v;
            if (wrd && L.watch > 0 && (d.flags & kPreRd) && d.rd == L.watch) L.watch = -1;
            L.ninst++;
            L.pc = npc;
        } else {
        switch (f) {
        case F_SYSCALL:   // SyscallFault::invokeSE advances the PC first (arch/riscv/faults.cc:325-333)
            L.pc = pc + d.len;
            do_syscall(c, L, m, slot, R, lane);
            break;
        case F_BREAK: finish(L, FI_CRASH, FI_CRASH_SIGTRAP, 133, (uint32_t)pc); break;
        case F_ILLEGAL: finish(L, FI_CRASH, FI_CRASH_ILLEGAL_INST, 134, (uint32_t)pc); break;
        case F_UNKNOWN: finish(L, FI_CRASH, FI_CRASH_UNKNOWN_INST, 134, (uint32_t)pc); break;
        case F_ESCAPE: finish(L, FI_ESCAPE, FI_ESC_INST, 0, d.raw); break;
        case F_ESCCSR: finish(L, FI_ESCAPE, FI_ESC_CSR, 0, d.raw); break;
        case F_DETECT: finish(L, FI_DETECTED, 0, 0, (uint32_t)pc); break;
        case F_PGFAULT:
            if (fva < m.stack_min && fva >= kStackBase - kMaxStack) {
                const uint64_t nm = fva & ~4095ULL;
                if (kStackBase - nm > kMaxStack) finish(L, FI_CRASH, FI_CRASH_STACK_LIMIT, 1, (uint32_t)pc);
                else { m.stack_min = nm; m.tlb_vpn = kNone; }
            } else {
                finish(L, FI_CRASH, FI_CRASH_PAGE_FAULT, 134, (uint32_t)fva);
            }
            break;
        default: break;
        }
        }   // fault disposition
        }   // f != F_NEEDPAGE
        }   // mine
        // ---- stay in the inner loop? every group lane committed, none reached
        // its next event, all at one PC that is still the wave's minimum
        const bool cont = mine && f == F_NONE && L.ninst < next_ev;
        const uint64_t cm = __ballot(cont);
        if (cm != gmask) break;
        const uint64_t npc0 = uni64(readlane64(L.pc, __ffsll((unsigned long long)cm) - 1));
        if (__ballot(cont && L.pc == npc0) != cm || npc0 >= wait_min) break;
        lpc = npc0;
        mine = cont;
        n_iter++;
        }   // inner loop
    }

    if (live) c.out[c.record ? 0 : sidx] = L.res;
    if (c.record && live) {
        c.stats[3] = L.ncyc;
        c.stats[4] = L.out_pos;
        c.stats[5] = L.err_pos;
    }
    const uint64_t fb = wave_sum64(L.fetch_b), db = wave_sum64(L.data_b), pm = wave_sum64(pages_made);
    if (lane == 0) {
        atomicAdd(&c.stats[0], (unsigned long long)fb);
        atomicAdd(&c.stats[1], (unsigned long long)db);
        atomicAdd(&c.stats[2], (unsigned long long)pm);
        atomicAdd(&c.stats[6], (unsigned long long)n_iter);
        atomicAdd(&c.stats[7], (unsigned long long)n_exec);
        atomicAdd(&c.stats[8], (unsigned long long)n_slow);
        atomicAdd(&c.stats[9], (unsigned long long)n_min);
        atomicMax(&c.stats[10], (unsigned long long)n_iter);
#ifdef FI_STAMPS
        for (int k = 0; k < 6; k++) atomicAdd(&c.stats[16 + k], (unsigned long long)tacc[k]);
#endif
    }
}

// ------------------------------------------------------------------ histogram
__global__ void fi_hist_kernel(const fi_site *sites, const fi_outcome *out, uint64_t n, fi_histogram *h) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const fi_site s = sites[i];
    const fi_outcome o = out[i];
    const uint32_t t = s.target < FI_N_STRUCT ? s.target : 0;
    const uint32_t bit = s.mask ? (uint32_t)__builtin_ctzll(s.mask) : 0;
    const uint32_t cls = o.cls < FI_N_CLASS ? o.cls : FI_ESCAPE;
    atomicAdd((unsigned long long *)&h->counts[t][bit][cls], 1ULL);
    if (cls == FI_CRASH) atomicAdd((unsigned long long *)&h->crash_sub[o.sub & 15], 1ULL);
    if (cls == FI_ESCAPE) atomicAdd((unsigned long long *)&h->escape_sub[o.sub & 7], 1ULL);
    atomicAdd((unsigned long long *)&h->trials, 1ULL);
    atomicAdd((unsigned long long *)&h->guest_insts, (unsigned long long)o.ninst);
}

__global__ void fi_hist_stats_kernel(const unsigned long long *stats, fi_histogram *h) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        h->fetch_bytes += stats[0];
        h->data_bytes += stats[1];
        h->cow_pages += stats[2];
    }
}

// ------------------------------------------------------------------ launch wrappers (host side)
static inline unsigned nblk(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

hipError_t launch_sample(const SampleCtx &c, uint64_t n, fi_site *sites, uint64_t *keys, uint32_t *perm,
                         hipStream_t st) {
    hipLaunchKernelGGL(fi_sample_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, c, n, sites, keys, perm);
    return hipGetLastError();
}
hipError_t launch_keys(const fi_site *sites, uint64_t n, uint64_t *keys, uint32_t *perm, hipStream_t st) {
    hipLaunchKernelGGL(fi_keys_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, sites, n, keys, perm);
    return hipGetLastError();
}
hipError_t launch_predecode(const uint8_t *text, uint64_t text_lo, uint64_t nhalf, PreInst *pre, hipStream_t st) {
    hipLaunchKernelGGL(fi_predecode_kernel, dim3(nblk(nhalf, 256)), dim3(256), 0, st, text, text_lo, nhalf, pre);
    return hipGetLastError();
}
hipError_t launch_debug_decode(const uint32_t *raws, uint64_t n, PreInst *out, hipStream_t st) {
    hipLaunchKernelGGL(fi_debug_decode_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, raws, n, out);
    return hipGetLastError();
}
hipError_t launch_trials(const DevCtx &c, hipStream_t st) {
    hipLaunchKernelGGL(fi_trial_kernel, dim3(nblk(c.n, 64)), dim3(64), 0, st, c);
    return hipGetLastError();
}
hipError_t launch_hist(const fi_site *sites, const fi_outcome *out, uint64_t n, fi_histogram *h,
                       const unsigned long long *stats, hipStream_t st) {
    hipLaunchKernelGGL(fi_hist_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, sites, out, n, h);
    hipLaunchKernelGGL(fi_hist_stats_kernel, dim3(1), dim3(64), 0, st, stats, h);
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
