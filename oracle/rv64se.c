/*
 * rv64se.c -- TEST INFRASTRUCTURE ONLY (see rv64se.h).
 *
 * Plain-C restatement of gem5's RISC-V AtomicSimpleCPU in SE mode, limited to
 * what a fault-injection trial of a static RV64 Linux binary exercises.  The
 * per-tick loop, decoder state machine, instruction semantics, SE memory
 * fixups, syscall subset and fault disposition each cite the reference
 * location they follow.  Everything outside the modelled subset is reported as
 * an explicit ESCAPE outcome, never guessed.
 */
#define _GNU_SOURCE
#include "rv64se.h"
#include "timing_se.h"
#include "../shrewd_amd/csrc/gem5_decode_table.h"
#include "../shrewd_amd/csrc/gem5_opclass_table.h"

#include <errno.h>
#include <pthread.h>
#include <sys/stat.h>
#include <zlib.h>
#include <stdbool.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* Zkn/Zks: the reference's scalar-crypto helpers (oracle/rvk_ref.cc over
 * src/arch/riscv/rvk.hh, oracle/rvk_ref.mk), linked when present (OR_RVK). */
#ifdef OR_RVK
uint64_t or_rvk_ref(int fn, uint64_t a, uint64_t b);   /* oracle/rvk_ref.cc: the reference's rvk.hh */
#endif

#ifdef OR_RVK
int or_has_rvk(void) { return 1; }
void or_rvk(int fn, const uint64_t *a, const uint64_t *b, uint64_t n, uint64_t *out) {
    for (uint64_t i = 0; i < n; i++) out[i] = or_rvk_ref(fn, a[i], b[i]);
}
#else
int or_has_rvk(void) { return 0; }
void or_rvk(int fn, const uint64_t *a, const uint64_t *b, uint64_t n, uint64_t *out) {
    (void)fn; (void)a; (void)b;
    memset(out, 0, n * sizeof *out);
}
#endif

/* ------------------------------------------------------------- SoftFloat */
/* F/D/Zfh arithmetic is the reference's own SoftFloat (gem5 ext/softfloat,
 * RISC-V specialization), compiled from its sources into oracle/_ref by
 * oracle/softfloat_ref.mk and linked when present (OR_SOFTFLOAT).  The
 * prototypes below restate its C interface (ext/softfloat/softfloat.h): each
 * floatN_t is a struct of one uintN_t, the rounding mode and the exception
 * flags are per-thread globals. */
#ifdef OR_SOFTFLOAT
typedef struct { uint16_t v; } sf16_t;
typedef struct { uint32_t v; } sf32_t;
typedef struct { uint64_t v; } sf64_t;
extern __thread uint_fast8_t softfloat_roundingMode, softfloat_exceptionFlags;
#define SF_DECL(T, p)                                                                                         \
    T p##_add(T, T); T p##_sub(T, T); T p##_mul(T, T); T p##_div(T, T); T p##_sqrt(T); T p##_mulAdd(T, T, T); \
    bool p##_eq(T, T); bool p##_lt(T, T); bool p##_le(T, T); bool p##_lt_quiet(T, T); bool p##_le_quiet(T, T); \
    int_fast32_t p##_to_i32(T, uint_fast8_t, bool); uint_fast32_t p##_to_ui32(T, uint_fast8_t, bool);        \
    int_fast64_t p##_to_i64(T, uint_fast8_t, bool); uint_fast64_t p##_to_ui64(T, uint_fast8_t, bool);        \
    T i32_to_##p(int32_t); T ui32_to_##p(uint32_t); T i64_to_##p(int64_t); T ui64_to_##p(uint64_t);          \
    T p##_roundToInt(T, uint_fast8_t, bool);
SF_DECL(sf16_t, f16)
SF_DECL(sf32_t, f32)
SF_DECL(sf64_t, f64)
sf32_t f16_to_f32(sf16_t); sf64_t f16_to_f64(sf16_t); sf16_t f32_to_f16(sf32_t); sf64_t f32_to_f64(sf32_t);
sf16_t f64_to_f16(sf64_t); sf32_t f64_to_f32(sf64_t);

/* one operation by code (the op / fmt codes of shrewd_amd/csrc/hip/fi_softfp.h) */
#define SF_OPS(T, p, W)                                                                                        \
    static u64 sf_##p(int op, int rm, u64 a, u64 b, u64 c) {                                                   \
        T x = {(W)a}, y = {(W)b}, z = {(W)c};                                                                   \
        switch (op) {                                                                                          \
        case 0: return p##_add(x, y).v; case 1: return p##_sub(x, y).v; case 2: return p##_mul(x, y).v;        \
        case 3: return p##_div(x, y).v; case 4: return p##_sqrt(x).v; case 5: return p##_mulAdd(x, y, z).v;    \
        case 6: return p##_eq(x, y); case 7: return p##_lt(x, y); case 8: return p##_le(x, y);                 \
        case 9: return p##_lt_quiet(x, y); case 10: return p##_le_quiet(x, y);                                  \
        case 11: return (u64)(s64)p##_to_i32(x, rm, true); case 12: return (u64)p##_to_ui32(x, rm, true);      \
        case 13: return (u64)p##_to_i64(x, rm, true); case 14: return (u64)p##_to_ui64(x, rm, true);           \
        case 15: return i32_to_##p((int32_t)a).v; case 16: return ui32_to_##p((uint32_t)a).v;                  \
        case 17: return i64_to_##p((int64_t)a).v; case 18: return ui64_to_##p(a).v;                           \
        case 22: return p##_roundToInt(x, rm, false).v; case 23: return p##_roundToInt(x, rm, true).v;         \
        default: return 0;                                                                                     \
        }                                                                                                      \
    }
typedef uint64_t u64;
typedef int64_t s64;
SF_OPS(sf16_t, f16, uint16_t)
SF_OPS(sf32_t, f32, uint32_t)
SF_OPS(sf64_t, f64, uint64_t)
static u64 sf_ref(int op, int fmt, int rm, u64 a, u64 b, u64 c, uint32_t *fl) {
    softfloat_roundingMode = (uint_fast8_t)rm;
    softfloat_exceptionFlags = 0;
    u64 r;
    if (op >= 19 && op <= 21) {   /* conversions between formats */
        const int to = op - 19;
        if (fmt == to) r = a;
        else if (fmt == 0) r = to == 1 ? f16_to_f32((sf16_t){(uint16_t)a}).v : f16_to_f64((sf16_t){(uint16_t)a}).v;
        else if (fmt == 1) r = to == 0 ? f32_to_f16((sf32_t){(uint32_t)a}).v : f32_to_f64((sf32_t){(uint32_t)a}).v;
        else r = to == 0 ? f64_to_f16((sf64_t){a}).v : f64_to_f32((sf64_t){a}).v;
    } else {
        r = fmt == 0 ? sf_f16(op, rm, a, b, c) : fmt == 1 ? sf_f32(op, rm, a, b, c) : sf_f64(op, rm, a, b, c);
    }
    *fl = softfloat_exceptionFlags;
    return r;
}
int or_has_softfloat(void) { return 1; }
void or_sf_ref(int op, int fmt, int rm, const uint64_t *a, const uint64_t *b, const uint64_t *c, uint64_t n,
               uint64_t *out, uint32_t *fl) {
    for (uint64_t i = 0; i < n; i++) out[i] = sf_ref(op, fmt, rm, a[i], b[i], c[i], &fl[i]);
}
#else
int or_has_softfloat(void) { return 0; }
void or_sf_ref(int op, int fmt, int rm, const uint64_t *a, const uint64_t *b, const uint64_t *c, uint64_t n,
               uint64_t *out, uint32_t *fl) {
    (void)op; (void)fmt; (void)rm; (void)a; (void)b; (void)c; (void)n; (void)out; (void)fl;
}
#endif

#define PAGE 4096ULL
#define OR_NONE (~0ULL)
#define PAGE_MASK (~(PAGE - 1))
/* RiscvProcess64 ctor, arch/riscv/process.cc:71-82 */
#define STACK_BASE 0x7FFFFFFFFFFFFFFFULL
#define MAX_STACK (8ULL * 1024 * 1024)
/* Process params defaults, sim/Process.py:61-67 */
#define PID 100
#define PPID 0
#define UID 100
#define GID 100

typedef uint64_t u64;
typedef int64_t s64;
typedef uint32_t u32;
typedef int32_t s32;

/* ------------------------------------------------------------------ pages */
typedef struct {
    u64 vpn;     /* page number; UINT64_MAX = empty */
    uint8_t *data;
    int owned;   /* 1 = private copy, 0 = shared image page */
} pte_t;

typedef struct {
    pte_t *tab;
    u64 cap, n;
} pmap_t;

static u64 hash_vpn(u64 v) { v ^= v >> 29; v *= 0xBF58476D1CE4E5B9ULL; v ^= v >> 32; return v; }

static void pm_init(pmap_t *m, u64 cap) {
    m->cap = cap; m->n = 0;
    m->tab = (pte_t *)malloc(sizeof(pte_t) * cap);
    for (u64 i = 0; i < cap; i++) { m->tab[i].vpn = UINT64_MAX; m->tab[i].data = NULL; m->tab[i].owned = 0; }
}
static pte_t *pm_find(pmap_t *m, u64 vpn) {
    u64 i = hash_vpn(vpn) & (m->cap - 1);
    for (;;) {
        if (m->tab[i].vpn == vpn) return &m->tab[i];
        if (m->tab[i].vpn == UINT64_MAX) return NULL;
        i = (i + 1) & (m->cap - 1);
    }
}
static pte_t *pm_insert(pmap_t *m, u64 vpn, uint8_t *data, int owned);
static void pm_grow(pmap_t *m) {
    pmap_t n2; pm_init(&n2, m->cap * 2);
    for (u64 i = 0; i < m->cap; i++)
        if (m->tab[i].vpn != UINT64_MAX) pm_insert(&n2, m->tab[i].vpn, m->tab[i].data, m->tab[i].owned);
    free(m->tab); *m = n2;
}
static pte_t *pm_insert(pmap_t *m, u64 vpn, uint8_t *data, int owned) {
    if ((m->n + 1) * 2 > m->cap) pm_grow(m);
    u64 i = hash_vpn(vpn) & (m->cap - 1);
    while (m->tab[i].vpn != UINT64_MAX && m->tab[i].vpn != vpn) i = (i + 1) & (m->cap - 1);
    if (m->tab[i].vpn == UINT64_MAX) m->n++;
    m->tab[i].vpn = vpn; m->tab[i].data = data; m->tab[i].owned = owned;
    return &m->tab[i];
}
static void pm_free(pmap_t *m) {
    for (u64 i = 0; i < m->cap; i++)
        if (m->tab[i].vpn != UINT64_MAX && m->tab[i].owned) free(m->tab[i].data);
    free(m->tab);
}

/* ------------------------------------------------------------- campaign */
typedef struct { uint8_t *buf; u64 len, cap; } bytes_t;
static void by_push(bytes_t *b, const uint8_t *p, u64 n) {
    if (b->len + n > b->cap) {
        u64 nc = b->cap ? b->cap : 256;
        while (nc < b->len + n) nc *= 2;
        b->buf = (uint8_t *)realloc(b->buf, nc); b->cap = nc;
    }
    memcpy(b->buf + b->len, p, n); b->len += n;
}

struct or_campaign {
    pmap_t image;          /* initial process image pages (shared, read-only) */
    u64 *alloc_vpn; u64 n_alloc, cap_alloc;   /* image pages in the order the image write allocated them */
    struct tkgold *tk;     /* tick-domain injection (or_tick_setup): the golden run's requests and ticks */
    u64 entry, sp0, stack_min0;
    u64 regs0[32], pc0;    /* initial architectural state (process start or a checkpoint) */
    u64 text_lo, text_hi;  /* page-aligned executable range (PT_LOAD with PF_X) */
    u64 stack_vma_lo, stack_vma_hi;  /* the "stack" VMA created by argsInit */
    u64 brk0;
    /* the rest of the initial machine (process start: zero / the stack VMA;
     * a checkpoint: what it holds) */
    u64 f0[32]; u32 fflags0, frm0;   /* FP registers, MISCREG_FFLAGS / MISCREG_FRM */
    struct { u64 lo, hi; } vma0[64]; /* MemState VMA list */
    int nvma0;
    u64 mmap_end0;
    u64 tick0;                       /* curTick at the start ([Globals] curTick of a checkpoint) */
    struct { u64 lo, hi; int w; } seg[32];   /* PT_LOAD page ranges, w = PF_W */
    int nseg;
    u64 clk_period;        /* ticks per CPU cycle (1 ps ticks; 500 = 2 GHz) */
    char exe_path[4096];   /* realpath of the process' executable ("" unknown): readlinkat /proc/self/exe */
    uint8_t *in_data;      /* Process.input as a file: its bytes (NULL: "cin", the host's stdin) */
    u64 in_len;
    u64 rnd_seed;          /* gem5 Random::globalSeed (base/random.cc:79) */
    u64 *mem_pages;        /* writable pages at process start (memory fault candidates) */
    u64 n_mem_pages;
    u64 protect_opc;       /* SHREWD replication: OpClass mask (bit = FuncUnit.py enum value) */
    uint8_t *shadow;       /* issue model on: shadow issued per golden numInst index (NULL: off) */
    u64 n_shadow;
    or_issue_stats_t issue_stats;
    /* golden */
    int have_golden;
    or_golden_t golden;
    int gsub;                        /* the golden run's end sub-code (OR_END_*) */
    bytes_t gout, gerr;
    char err[256];
};

const char *or_error(or_campaign_t *c) { return c ? c->err : "null campaign"; }

/* ---------------------------------------------------------------- machine */
typedef struct {
    u64 x[32];
    u64 f[32];            /* FP registers (raw bits; zero at process start) */
    u32 fflags, frm;      /* MISCREG_FFLAGS / MISCREG_FRM (zero at process start) */
    u64 pc, npc;
    u64 num_inst, num_cycles;
    /* decoder state machine, arch/riscv/decoder.cc:54-116 */
    int mid; u32 emi; int inst_done;
    u64 fetch_offset; int stay_at_pc;
    pmap_t mem;
    u64 stack_min;
    bytes_t out, err;
    /* fault injection */
    const or_site_t *site; int injected; int watch; /* watch = protected flipped reg, -1 none */
    int rarm, wrote;      /* result fault armed (OR_T_RESULT); the executing instruction wrote x[rd] */
    u64 rmask;            /* the armed result fault's mask */
    /* golden trace recording for the issue model (or_set_issue_model) */
    or_issue_op_t *rec; u64 rec_n, rec_cap;
    /* LR/SC: the ISA's load reservation (isa.cc:1006-1064) and this context's
     * lock record in memory (abstract_mem.cc:258-345), as virtual addresses
     * (the SE page mapping is a per-page bijection); OR_NONE = none */
    u64 resv, lock;
    /* SE memory map (MemState, sim/mem_state.cc): the VMA list as disjoint
     * [lo, hi) page ranges (only their union matters: names and file backing
     * are not modelled), the break point and the mmap end; plus the fd table
     * entries 0..2 closed (fdc bit fd) and set_tid_address's childClearTID */
    struct { u64 lo, hi; } vma[64];
    int nvma;
    u64 brk, mmap_end, ctid;
    u32 fdc;
    /* getrandom's generator (syscall_emul.hh:3222-3236: one mt19937_64 per
     * process, created at the first call from the global seed) */
    u64 *mt; int mt_i;
    u64 rnd_pos;          /* bytes drawn (the engine's table holds OR_RND_CAP) */
    u64 in_pos;           /* fd 0's file offset (Process.input a file); a checkpoint restart starts at 0 */
    u64 protect_mask;
    /* termination */
    int done; or_outcome_t res;
    /* counters for the roofline bookkeeping */
    u64 fetch_bytes, data_bytes;
    /* diagnostics (or_debug_trace): committed pcs, store addresses into the text */
    u64 *dbg_pc, dbg_pc_n, dbg_pc_cap, *dbg_wr, dbg_wr_n, dbg_wr_cap;
    int dbg_raw;   /* or_debug_trace_raw: pc | instruction word << 32 */
    int m5x, m5code;   /* an M5 op that ends the run after it commits: 1 m5_exit, 2 m5_fail, 3 quiesce */
    /* the vector configuration of the PC state (riscv/pcstate.hh: _vtype, _vl)
     * as VCFG(vtype, vl) -- 0 is the process start (vtype = vill, vl = 0) */
    u32 vcfg;
    /* tick-domain injection (TimingSimpleCPU, include/fi_engine.h "Tick-domain
     * injection"): tkr records the golden run's requests, tki applies a trial's
     * flip inside the instruction in flight; fo = the next fetch reads fo_addr
     * (a request sent before a pc flip); tk_cpu = a CPU access is executing */
    struct tkrec *tkr;
    const struct tkinj *tki;
    int fo, tk_cpu; u64 fo_addr;
    const or_campaign_t *c;
} mach_t;
/* vcfg <-> (vtype, vl): a vtype that getNewVtype produces is vill alone, a
 * legal vtype8, or (vsetvl's register) a legal vtype8 with bit 63 set */
#define VILL (1ULL << 63)
static u32 vcfg_of(u64 vtype, u32 vl) { return ((u32)(vtype & 0xFF) | (u32)(vtype >> 63) << 8 | vl << 9) ^ 0x100u; }
static u64 vcfg_vtype(u32 vcfg) { vcfg ^= 0x100u; return (u64)(vcfg & 0xFF) | (u64)((vcfg >> 8) & 1) << 63; }
static u32 vcfg_vl(u32 vcfg) { return vcfg >> 9; }

enum { F_NONE = 0, F_SYSCALL = 1, F_BREAK = 2, F_ILLEGAL = 3, F_UNKNOWN = 4, F_ESCAPE = 5, F_PGFAULT = 6, F_AMOLINE = 7,
       F_SCLINE = 8, F_M5PANIC = 9, F_UNDEF = 10, F_VSEW = 11, F_TKCLOCK = 12 };

/* -------------------------------------------------------------- decode */
/* Op ids.  Names follow gem5's mnemonics (arch/riscv/isa/decoder.isa). */
#define OPS(X) \
    X(UNKNOWN) X(ESC_FP) X(ESC_VEC) X(ESC_AMO) X(ESC_SYS) X(ESC_CRYPTO) X(ESC_CBO) X(ESC_CMP) X(ESC_M5) X(ESC_HYP) \
    X(c_addi4spn) X(c_lw) X(c_ld) X(c_lbu) X(c_lhu) X(c_lh) X(c_sb) X(c_sh) X(c_sw) X(c_sd) \
    X(c_addi) X(c_addiw) X(c_li) X(c_addi16sp) X(c_lui) X(c_srli) X(c_srai) X(c_andi) \
    X(c_sub) X(c_xor) X(c_or) X(c_and) X(c_subw) X(c_addw) X(c_mul) \
    X(c_zext_b) X(c_sext_b) X(c_zext_h) X(c_sext_h) X(c_zext_w) X(c_not) \
    X(c_j) X(c_beqz) X(c_bnez) X(c_slli) X(c_lwsp) X(c_ldsp) X(c_jr) X(c_mv) X(c_ebreak) X(c_jalr) X(c_add) \
    X(c_swsp) X(c_sdsp) \
    X(lb) X(lh) X(lw) X(ld) X(lbu) X(lhu) X(lwu) X(fence) X(fence_i) \
    X(slli) X(bseti) X(bclri) X(binvi) X(clz) X(ctz) X(cpop) X(sext_b) X(sext_h) \
    X(addi) X(slti) X(sltiu) X(xori) X(srli) X(orc_b) X(srai) X(bexti) X(rori) X(rev8) \
    X(prefetch_i) X(prefetch_r) X(prefetch_w) X(ori_hint) X(ori) X(andi) X(auipc) \
    X(addiw) X(slliw) X(slli_uw) X(clzw) X(ctzw) X(cpopw) X(srliw) X(sraiw) X(roriw) \
    X(sb) X(sh) X(sw) X(sd) \
    X(add) X(sub) X(mul) X(sll) X(mulh) X(clmul) X(bset) X(bclr) X(rol) X(binv) \
    X(slt) X(mulhsu) X(clmulr) X(sh1add) X(sltu) X(mulhu) X(clmulh) \
    X(xor_) X(div_) X(pack) X(min_) X(sh2add) X(xnor) \
    X(srl) X(divu) X(czero_eqz) X(sra) X(minu) X(bext) X(ror) \
    X(or_) X(rem) X(max_) X(sh3add) X(orn) \
    X(and_) X(remu) X(packh) X(maxu) X(czero_nez) X(andn) \
    X(lui) X(addw) X(mulw) X(add_uw) X(subw) X(sllw) X(rolw) X(sh1add_uw) \
    X(divw) X(packw) X(sh2add_uw) X(srlw) X(divuw) X(sraw) X(rorw) X(remw) X(sh3add_uw) X(remuw) \
    X(beq) X(bne) X(blt) X(bge) X(bltu) X(bgeu) X(jalr) X(jal) \
    X(ecall) X(ebreak) X(csr) \
    X(flh) X(flw) X(fld) X(fsh) X(fsw) X(fsd) X(c_fld) X(c_fsd) X(c_fldsp) X(c_fsdsp) \
    X(fmv_x_w) X(fmv_x_d) X(fmv_x_h) X(fmv_w_x) X(fmv_d_x) X(fmv_h_x) \
    X(fsgnj_s) X(fsgnjn_s) X(fsgnjx_s) X(fsgnj_d) X(fsgnjn_d) X(fsgnjx_d) X(fsgnj_h) X(fsgnjn_h) X(fsgnjx_h) \
    X(fclass_s) X(fclass_d) X(fclass_h) \
    X(amoadd_w) X(amoswap_w) X(amoxor_w) X(amoor_w) X(amoand_w) X(amomin_w) X(amomax_w) X(amominu_w) X(amomaxu_w) \
    X(amoadd_d) X(amoswap_d) X(amoxor_d) X(amoor_d) X(amoand_d) X(amomin_d) X(amomax_d) X(amominu_d) X(amomaxu_d) \
    X(lr_w) X(sc_w) X(lr_d) X(sc_d) \
    X(fadd) X(fsub) X(fmul) X(fdiv) X(fsqrt) X(fmin) X(fmax) X(fmadd) X(fmsub) X(fnmsub) X(fnmadd) \
    X(feq) X(flt) X(fle) X(fcvt_f2i) X(fcvt_i2f) X(fcvt_f2f) \
    X(priv) X(cbo) X(m5op) X(crypto) X(fli) X(fround) X(fcvtmod) X(vec) X(vset)

enum {
#define X(n) OP_##n,
    OPS(X)
#undef X
    OP_COUNT
};
static const char *op_names[] = {
#define X(n) #n,
    OPS(X)
#undef X
};

typedef struct {
    u32 raw; u32 len;
    int op;
    int rd, rs1, rs2;     /* integer registers, -1 = not used */
    int frd, frs1, frs2;  /* floating-point registers, -1 = not used */
    s64 imm;
    u32 csr, funct3;
} dec_t;

static inline u32 bits(u32 v, int hi, int lo) { return (v >> lo) & ((hi - lo == 31) ? 0xFFFFFFFFu : ((1u << (hi - lo + 1)) - 1)); }
static inline s64 sext(u64 v, int n) { return (s64)(v << (64 - n)) >> (64 - n); }

/* Decode one instruction (16- or 32-bit in the low bits of raw) following the
 * decode tree of arch/riscv/isa/decoder.isa for rv_type=RV64, enable_zcd=1
 * (RiscvISA.py:95,121-127).  Field definitions: isa/bitfields.isa:36-130. */
static void decode_tree(u32 raw, dec_t *d);
/* Which 32-bit encodings of the non-executed opcode groups (FP, vector, AMO,
 * privileged SYSTEM) gem5 decodes to a real instruction rather than Unknown:
 * first-match rows generated from decoder.isa by
 * tools/oracle/gen_decode_vectors.py (shrewd_amd/csrc/gem5_decode_table.h). */
typedef struct { u32 mask, match; uint8_t known; } dec_row_t;
#define ROW(m, v, k) {m, v, k},
static const dec_row_t gem5_rows[FI_GEM5_DEC_ROWS] = { FI_GEM5_DEC_TABLE(ROW) };
#undef ROW
static int gem5_known(u32 raw) {
    u32 op5 = (raw >> 2) & 31;
#define IDX(o, first, cnt) \
    if (op5 == (o)) { for (int i = (first); i < (first) + (cnt); i++) \
                          if ((raw & gem5_rows[i].mask) == gem5_rows[i].match) return gem5_rows[i].known; \
                      return 0; }
    FI_GEM5_DEC_INDEX(IDX)
#undef IDX
    return 1;
}
/* RVV in a process that has not executed a vset* (vtype = vill, vl = 0:
 * decoder.hh:68-69): the row's action (gem5_decode_table.h, generated by
 * tools/oracle/gen_vector_actions.py from the reference's micro-op code)
 * becomes op `vec`, imm = 2 no-op, 3 no-op of two ticks, 4 IllegalInst
 * ("VILL is set", isa.cc:1400-1402), 5 undefined in gem5 (GEM5_UNREACHABLE
 * at the SEW = 8 decode), 6 needs vector state (vset*, whole-register). */
enum { VEC_NOP = 2, VEC_NOP2 = 3, VEC_ILLEGAL = 4, VEC_UNDEF = 5, VEC_STATE = 6 };
/* Unknown and escape encodings read and write no registers. */
static void refine_fp_amo(u32 raw, dec_t *d);
/* The gem5-known members of the privileged SYSTEM, hypervisor load/store,
 * cache-block, M5 pseudo-op and scalar-crypto groups, which the SE process
 * executes deterministically (registers: the source operands the generated
 * execute() reads first, exec-ns.cc.inc of the reference's ISA parser).
 *   priv   imm 0: IllegalInstFault in PRV_U (SE runs the process in PRV_U,
 *          arch/riscv/process.cc:105; privilege set MSU, no RVH, no Smrnmi,
 *          RiscvISA.py:108,129): sret / wfi / sfence_vma / hfence_vvma / mret /
 *          hfence_gvma / mnret (decoder.isa:5966-6233) and every hlv* / hsv*
 *          (formats/mem.isa:364-376,461-473, after reading Rs1 [, Rs2]);
 *          imm 1: warn-only no-ops sinval_vvma / sfence_w_inval /
 *          sfence_inval_ir / hinval_vvma / hinval_gvma (:6070-6090,6112,6236).
 *   cbo    imm = FUNCT12 (0 inval, 1 clean, 2 flush, 4 zero): a 64-byte
 *          request at Rs1 & ~63 (CacheBlockBasedStoreExecute, formats/
 *          mem.isa:244-268: the body's privilege checks are not part of
 *          execute); zero writes 64 zero bytes (CACHE_BLOCK_ZERO ->
 *          WriteReq), the others only translate (CleanShared / CleanInvalid /
 *          InvalidateReq: AbstractMemory::access leaves memory alone).
 *   m5op   imm = M5FUNC (bitfields.isa:135); a0 = result, a1 = 0.
 *   crypto imm = function (see crypto_fn) | RNUM or BS << 8. */
static const char *const crypto_names[22] = {
    "sha256sum0", "sha256sum1", "sha256sig0", "sha256sig1", "sha512sum0", "sha512sum1", "sha512sig0", "sha512sig1",
    "sm3p0", "sm3p1", "aes64im", "aes64ks1i", "brev8", "sm4ed", "sm4ks", "aes64es", "aes64esm", "aes64ds", "aes64dsm",
    "aes64ks2", "xperm4", "xperm8"};
static void refine_misc(u32 raw, dec_t *d) {
    const u32 f3 = bits(raw, 14, 12), f7 = bits(raw, 31, 25);
    const int rd = (int)bits(raw, 11, 7), rs1 = (int)bits(raw, 19, 15), rs2 = (int)bits(raw, 24, 20);
    switch (d->op) {
    case OP_ESC_SYS:
        d->op = OP_priv;
        d->imm = (f7 == 0x0b || f7 == 0x0c || f7 == 0x13 || f7 == 0x33) ? 1 : 0;
        if (f7 == 0x09 || f7 == 0x11 || f7 == 0x31) { d->rs1 = rs1; d->rs2 = rs2; }   /* demapPage(Rs1, Rs2) */
        return;
    case OP_ESC_HYP:
        d->op = OP_priv; d->imm = 0; d->rs1 = rs1;
        if (f7 & 1) d->rs2 = rs2;   /* hsv_*: FUNCT7 0x31 / 0x33 / 0x35 / 0x37 */
        return;
    case OP_ESC_CBO: d->op = OP_cbo; d->rs1 = rs1; d->imm = bits(raw, 31, 20); return;
    case OP_ESC_M5: d->op = OP_m5op; d->rd = 10; d->imm = f7; return;
    case OP_ESC_CRYPTO: {
        const u32 opc = bits(raw, 6, 2), kf5 = bits(raw, 29, 25), bs = bits(raw, 31, 30);
        int fn = -1;
        if (opc == 0x04 && f3 == 1) {
            if (bits(raw, 31, 27) == 0x02) fn = rs2;                            /* sha256* sha512* sm3p*: 0..9 */
            else fn = bits(raw, 24, 24) ? 11 | (int)(bits(raw, 23, 20) << 8) : 10;   /* aes64ks1i / aes64im */
        } else if (opc == 0x04) {
            fn = 12;                                                            /* brev8 */
        } else if (opc == 0x0c && f3 == 0) {
            switch (kf5) {
            case 0x18: fn = 13 | (int)(bs << 8); break;                         /* sm4ed */
            case 0x1a: fn = 14 | (int)(bs << 8); break;                         /* sm4ks */
            case 0x19: fn = 15; break; case 0x1b: fn = 16; break; case 0x1d: fn = 17; break;
            case 0x1f: fn = bs ? 19 : 18; break;                                /* aes64dsm / aes64ks2 */
            }
        } else if (opc == 0x0c) {
            fn = f3 == 2 ? 20 : 21;                                             /* xperm4 / xperm8 */
        }
        if (fn < 0) return;
        d->op = OP_crypto; d->imm = fn; d->rd = rd; d->rs1 = rs1;
        if ((fn & 0xFF) >= 13) d->rs2 = rs2;
        return;
    }
    default: return;
    }
}
static void decode(u32 raw, dec_t *d) {
    decode_tree(raw, d);
    if ((raw & 3) == 3 && (d->op == OP_ESC_FP || d->op == OP_ESC_VEC || d->op == OP_ESC_AMO ||
                           d->op == OP_ESC_SYS || d->op == OP_ESC_HYP)) {
        const int k = gem5_known(raw);
        if (!k) d->op = OP_UNKNOWN;
        else if (k >= VEC_NOP) { d->op = OP_vec; d->imm = k; }
    }
    if ((raw & 3) == 3 && (d->op == OP_ESC_FP || d->op == OP_ESC_AMO)) refine_fp_amo(raw, d);
    if (d->op < OP_c_addi4spn) d->rd = d->rs1 = d->rs2 = d->frd = d->frs1 = d->frs2 = -1;
    if ((raw & 3) == 3) refine_misc(raw, d);
    if (d->op == OP_vec && d->imm == VEC_STATE && bits(raw, 6, 0) == 0x57 && bits(raw, 14, 12) == 7) {
        /* vsetvli / vsetvl / vsetivli (decoder.isa:5838-5886): imm = the
         * requested vtype's immediate | form << 16 (0 vsetvli, 1 vsetvl: vtype
         * from Rs2, 2 vsetivli: its uimm << 20); Rd written, Rs1 (and Rs2) read */
        const int form = bits(raw, 31, 31) ? (bits(raw, 30, 30) ? 2 : 1) : 0;
        d->op = OP_vset;
        d->rd = (int)bits(raw, 11, 7);
        d->rs1 = form == 2 ? -1 : (int)bits(raw, 19, 15);
        d->rs2 = form == 1 ? (int)bits(raw, 24, 20) : -1;
        d->imm = (form == 0 ? (s64)bits(raw, 30, 20) : form == 2 ? (s64)bits(raw, 29, 20) : 0) | ((s64)form << 16) |
                 (form == 2 ? (s64)bits(raw, 19, 15) << 20 : 0);
    }
}
/* The executed members of the LOAD-FP / STORE-FP / OP-FP / AMO groups, among
 * the encodings gem5 decodes to a known class (decoder.isa:567-591 flh/flw/fld,
 * :1741-1763 fsh/fsw/fsd, :2067-2283 AMOs, :2896-2942 fsgnj*, :3500-3544
 * fmv.x.* / fclass.*, :3545-3548 fmv.w.x, :3593-3598 fmv.d.x, :3648-3652
 * fmv.h.x).  Everything else in those groups stays an escape. */
#ifdef OR_SOFTFLOAT
/* F/D/Zfh arithmetic (decoder.isa:2694-2810 FMADD group, 2811-3440 OP-FP):
 * one op per operation, the format and operand details packed into imm as
 * rm | fmt << 3 | sub << 5 | rs3 << 8 (fmt 0 binary16, 1 binary32, 2 binary64;
 * sub: fmin/fmax 1 = the Zfa minimumNumber variant, flt/fle 1 = quiet (Zfa),
 * fcvt to/from integer the kind w/wu/l/lu, fcvt between formats the source
 * format).  Zfa's fli / fround / froundnx / fcvtmod stay escapes. */
static int fp_fmt(u32 f) { return f == 0 ? 1 : f == 1 ? 2 : f == 2 ? 0 : -1; }
static int refine_fp_arith(u32 raw, dec_t *d) {
    u32 opc = bits(raw, 6, 2), f3 = bits(raw, 14, 12), f7 = bits(raw, 31, 25);
    int rd = (int)bits(raw, 11, 7), rs1 = (int)bits(raw, 19, 15), rs2 = (int)bits(raw, 24, 20);
    int fmt = fp_fmt(f7 & 3), op = -1, sub = 0;
#define FP_SET(o, s_) do { op = (o); sub = (s_); } while (0)
    if (opc >= 0x10 && opc <= 0x13) {
        fmt = fp_fmt(bits(raw, 26, 25));
        if (fmt < 0) return 0;
        d->op = OP_fmadd + (int)(opc - 0x10);
        d->frd = rd; d->frs1 = rs1; d->frs2 = rs2;
        d->imm = f3 | ((u32)fmt << 3) | (bits(raw, 31, 27) << 8);
        return 1;
    }
    if (opc != 0x14 || fmt < 0) return 0;
    switch (f7 >> 2) {
    case 0x00: op = OP_fadd; break;
    case 0x01: op = OP_fsub; break;
    case 0x02: op = OP_fmul; break;
    case 0x03: op = OP_fdiv; break;
    case 0x0b: op = OP_fsqrt; break;
    case 0x05:   /* fmin / fmax / fminm / fmaxm (binary16: fminm at 3, fmaxm at 4) */
        if (f3 == 0) FP_SET(OP_fmin, 0);
        else if (f3 == 1) FP_SET(OP_fmax, 0);
        else if (f3 == (fmt == 0 ? 3u : 2u)) FP_SET(OP_fmin, 1);
        else if (f3 == (fmt == 0 ? 4u : 3u)) FP_SET(OP_fmax, 1);
        else return 0;
        break;
    case 0x14:
        if (f3 == 0) FP_SET(OP_fle, 0);
        else if (f3 == 1) FP_SET(OP_flt, 0);
        else if (f3 == 2) FP_SET(OP_feq, 0);
        else if (f3 == 4) FP_SET(OP_fle, 1);
        else if (f3 == 5) FP_SET(OP_flt, 1);
        else return 0;
        d->op = op; d->rd = rd; d->frs1 = rs1; d->frs2 = rs2;
        d->imm = f3 | ((u32)fmt << 3) | ((u32)sub << 5);
        return 1;
    case 0x18:
        if (rs2 == 8 && fmt == 2) {   /* Zfa fcvtmod.w.d (decoder.isa:3320) */
            d->op = OP_fcvtmod; d->rd = rd; d->frs1 = rs1; d->imm = f3 | (2u << 3);
            return 1;
        }
        if (rs2 > 3) return 0;
        d->op = OP_fcvt_f2i; d->rd = rd; d->frs1 = rs1;
        d->imm = f3 | ((u32)fmt << 3) | ((u32)rs2 << 5);
        return 1;
    case 0x1a:
        if (rs2 > 3) return 0;
        d->op = OP_fcvt_i2f; d->frd = rd; d->rs1 = rs1;
        d->imm = f3 | ((u32)fmt << 3) | ((u32)rs2 << 5);
        return 1;
    case 0x08: {
        if (rs2 == 4 || rs2 == 5) {   /* Zfa fround / froundnx (decoder.isa:3105-3170) */
            d->op = OP_fround; d->frd = rd; d->frs1 = rs1;
            d->imm = f3 | ((u32)fmt << 3) | ((u32)(rs2 == 5) << 5);
            return 1;
        }
        const int src = fp_fmt((u32)rs2);
        if (rs2 > 2 || src < 0 || src == fmt) return 0;
        d->op = OP_fcvt_f2f; d->frd = rd; d->frs1 = rs1;
        d->imm = f3 | ((u32)fmt << 3) | ((u32)src << 5);
        return 1;
    }
    default: return 0;
    }
#undef FP_SET
    d->op = op; d->frd = rd; d->frs1 = rs1; d->frs2 = rs2;
    d->imm = f3 | ((u32)fmt << 3) | ((u32)sub << 5);
    return 1;
}
#endif
static void refine_fp_amo(u32 raw, dec_t *d) {
    u32 opc = bits(raw, 6, 2), f3 = bits(raw, 14, 12), f7 = bits(raw, 31, 25);
    int rd = (int)bits(raw, 11, 7), rs1 = (int)bits(raw, 19, 15), rs2 = (int)bits(raw, 24, 20);
    s64 imm_i = sext(bits(raw, 31, 20), 12), imm_s = sext((bits(raw, 31, 25) << 5) | bits(raw, 11, 7), 12);
    if (opc == 0x01 && f3 >= 1 && f3 <= 3) {
        d->op = OP_flh + (int)(f3 - 1); d->frd = rd; d->rs1 = rs1; d->imm = imm_i; return;
    }
    if (opc == 0x09 && f3 >= 1 && f3 <= 3) {
        d->op = OP_fsh + (int)(f3 - 1); d->frs2 = rs2; d->rs1 = rs1; d->imm = imm_s; return;
    }
    if (opc == 0x0b && (f3 == 2 || f3 == 3)) {
        static const int w[32] = {[0x00] = OP_amoadd_w, [0x01] = OP_amoswap_w, [0x04] = OP_amoxor_w,
                                  [0x08] = OP_amoor_w, [0x0c] = OP_amoand_w, [0x10] = OP_amomin_w,
                                  [0x14] = OP_amomax_w, [0x18] = OP_amominu_w, [0x1c] = OP_amomaxu_w};
        u32 f5 = bits(raw, 31, 27);
        if (f5 == 0x02 || f5 == 0x03) {   /* lr / sc (decoder.isa:2069-2075, 2175-2181) */
            d->op = f5 == 0x02 ? (f3 == 2 ? OP_lr_w : OP_lr_d) : (f3 == 2 ? OP_sc_w : OP_sc_d);
            d->rd = rd; d->rs1 = rs1; d->rs2 = f5 == 0x03 ? rs2 : -1; d->imm = 0;
            d->funct3 = bits(raw, 26, 25);   /* aq << 1 | rl */
            return;
        }
        int o = w[f5];
        if (!o) return;
        d->op = f3 == 2 ? o : o + (OP_amoadd_d - OP_amoadd_w);
        d->rd = rd; d->rs1 = rs1; d->rs2 = rs2; d->imm = 0;
        d->funct3 = bits(raw, 26, 25);   /* aq << 1 | rl: the macro-op's fence micro-ops */
        return;
    }
#ifdef OR_SOFTFLOAT
    if (refine_fp_arith(raw, d)) return;
#endif
    if (opc != 0x14) return;
    if ((f7 == 0x10 || f7 == 0x11 || f7 == 0x12) && f3 <= 2) {
        d->op = (f7 == 0x10 ? OP_fsgnj_s : f7 == 0x11 ? OP_fsgnj_d : OP_fsgnj_h) + (int)f3;
        d->frd = rd; d->frs1 = rs1; d->frs2 = rs2; return;
    }
    if (f7 == 0x70 && f3 <= 1) { d->op = f3 ? OP_fclass_s : OP_fmv_x_w; d->rd = rd; d->frs1 = rs1; return; }
    if (f7 == 0x71 && f3 == 1) { d->op = OP_fclass_d; d->rd = rd; d->frs1 = rs1; return; }
    if (f7 == 0x71 && f3 == 0 && rs2 == 0) { d->op = OP_fmv_x_d; d->rd = rd; d->frs1 = rs1; return; }
    if (f7 == 0x72 && f3 <= 1) { d->op = f3 ? OP_fclass_h : OP_fmv_x_h; d->rd = rd; d->frs1 = rs1; return; }
    if (f7 == 0x78 && f3 == 0 && rs2 == 0) { d->op = OP_fmv_w_x; d->frd = rd; d->rs1 = rs1; return; }
    /* Zfa fli.s / fli.d / fli.h (decoder.isa:3550,3600,3653): rs1 is the table index */
    if ((f7 == 0x78 && f3 == 0 && rs2 == 1) || ((f7 == 0x79 || f7 == 0x7a) && rs2 == 1)) {
        d->op = OP_fli; d->frd = rd; d->imm = ((u32)rs1 << 8) | ((u32)(f7 == 0x78 ? 1 : f7 == 0x79 ? 2 : 0) << 3);
        return;
    }
    if (f7 == 0x79 && rs2 == 0) { d->op = OP_fmv_d_x; d->frd = rd; d->rs1 = rs1; return; }
    if (f7 == 0x7a && rs2 == 0) { d->op = OP_fmv_h_x; d->frd = rd; d->rs1 = rs1; return; }
}
static void decode_tree(u32 raw, dec_t *d) {
    memset(d, 0, sizeof(*d));
    d->raw = raw; d->rd = d->rs1 = d->rs2 = -1; d->frd = d->frs1 = d->frs2 = -1; d->op = OP_UNKNOWN;
    u32 q = raw & 3;
    if (q != 3) {  /* compressed: decoder.isa:43-536 */
        raw &= 0xFFFF; d->raw = raw; d->len = 2;
        u32 cop = bits(raw, 15, 13);
        u32 rp1 = 8 + bits(raw, 9, 7), rp2 = 8 + bits(raw, 4, 2);
        u32 rc1 = bits(raw, 11, 7), rc2 = bits(raw, 6, 2);
        u32 cimm5 = bits(raw, 6, 2), cimm1 = bits(raw, 12, 12), cimm3 = bits(raw, 12, 10), cimm2 = bits(raw, 6, 5);
        u32 cimm6 = bits(raw, 12, 7), cimm8 = bits(raw, 12, 5);
        if (q == 0) {
            switch (cop) {
            case 0: d->op = OP_c_addi4spn; d->rd = rp2; d->rs1 = 2;
                d->imm = (bits(cimm8, 1, 1) << 2) | (bits(cimm8, 0, 0) << 3) | (bits(cimm8, 7, 6) << 4) | (bits(cimm8, 5, 2) << 6);
                return;
            case 1: d->op = OP_c_fld; d->frd = rp2; d->rs1 = rp1; d->imm = (cimm3 << 3) | (cimm2 << 6); return;  /* :57-68 */
            case 2: d->op = OP_c_lw; d->rd = rp2; d->rs1 = rp1;
                d->imm = (bits(cimm2, 1, 1) << 2) | (cimm3 << 3) | (bits(cimm2, 0, 0) << 6); return;
            case 3: d->op = OP_c_ld; d->rd = rp2; d->rs1 = rp1; d->imm = (cimm3 << 3) | (cimm2 << 6); return;
            case 4:
                switch (bits(raw, 12, 10)) {
                case 0: d->op = OP_c_lbu; d->rd = rp2; d->rs1 = rp1; d->imm = (bits(cimm2, 0, 0) << 1) | bits(cimm2, 1, 1); return;
                case 1: d->op = bits(raw, 6, 6) ? OP_c_lh : OP_c_lhu; d->rd = rp2; d->rs1 = rp1; d->imm = bits(cimm2, 0, 0) << 1; return;
                case 2: d->op = OP_c_sb; d->rs1 = rp1; d->rs2 = rp2; d->imm = (bits(cimm2, 0, 0) << 1) | bits(cimm2, 1, 1); return;
                case 3: d->op = OP_c_sh; d->rs1 = rp1; d->rs2 = rp2; d->imm = bits(cimm2, 0, 0) << 1; return;
                default: return;
                }
            case 5: d->op = OP_c_fsd; d->frs2 = rp2; d->rs1 = rp1; d->imm = (cimm3 << 3) | (cimm2 << 6); return;  /* :146-156 */
            case 6: d->op = OP_c_sw; d->rs1 = rp1; d->rs2 = rp2;
                d->imm = (bits(cimm2, 1, 1) << 2) | (cimm3 << 3) | (bits(cimm2, 0, 0) << 6); return;
            case 7: d->op = OP_c_sd; d->rs1 = rp1; d->rs2 = rp2; d->imm = (cimm3 << 3) | (cimm2 << 6); return;
            }
        } else if (q == 1) {
            switch (cop) {
            case 0: d->op = OP_c_addi; d->rd = d->rs1 = rc1; d->imm = sext(cimm5 | (cimm1 << 5), 6); return;
            case 1: d->op = OP_c_addiw; d->rd = d->rs1 = rc1; d->imm = sext(cimm5 | (cimm1 << 5), 6); return;
            case 2: d->op = OP_c_li; d->rd = rc1; d->imm = sext(cimm5 | (cimm1 << 5), 6); return;
            case 3:
                if (rc1 == 2) {
                    d->op = OP_c_addi16sp; d->rd = d->rs1 = 2;
                    d->imm = sext((bits(cimm5, 4, 4) << 4) | (bits(cimm5, 0, 0) << 5) | (bits(cimm5, 3, 3) << 6) |
                                  (bits(cimm5, 2, 1) << 7) | (cimm1 << 9), 10);
                } else {
                    d->op = OP_c_lui; d->rd = rc1; d->imm = sext(cimm5 | (cimm1 << 5), 6) * 4096;
                }
                return;
            case 4:
                switch (bits(raw, 11, 10)) {
                case 0: d->op = OP_c_srli; d->rd = d->rs1 = rp1; d->imm = cimm5 | (cimm1 << 5); return;
                case 1: d->op = OP_c_srai; d->rd = d->rs1 = rp1; d->imm = cimm5 | (cimm1 << 5); return;
                case 2: d->op = OP_c_andi; d->rd = d->rs1 = rp1; d->imm = sext(cimm5 | (cimm1 << 5), 6); return;
                case 3: {
                    u32 f2 = bits(raw, 6, 5);
                    d->rd = d->rs1 = rp1; d->rs2 = rp2;
                    if (!cimm1) {
                        static const int o[4] = {OP_c_sub, OP_c_xor, OP_c_or, OP_c_and};
                        d->op = o[f2]; return;
                    }
                    switch (f2) {
                    case 0: d->op = OP_c_subw; return;
                    case 1: d->op = OP_c_addw; return;
                    case 2: d->op = OP_c_mul; return;
                    case 3:
                        d->rs2 = -1;
                        switch (bits(raw, 4, 2)) {
                        case 0: d->op = OP_c_zext_b; return;
                        case 1: d->op = OP_c_sext_b; return;
                        case 2: d->op = OP_c_zext_h; return;
                        case 3: d->op = OP_c_sext_h; return;
                        case 4: d->op = OP_c_zext_w; return;
                        case 5: d->op = OP_c_not; return;
                        default: d->rd = d->rs1 = -1; d->op = OP_UNKNOWN; return;
                        }
                    }
                }
                }
                return;
            case 5: d->op = OP_c_j;
                d->imm = sext((bits(raw, 5, 3) << 1) | (bits(raw, 11, 11) << 4) | (bits(raw, 2, 2) << 5) |
                              (bits(raw, 7, 7) << 6) | (bits(raw, 6, 6) << 7) | (bits(raw, 10, 9) << 8) |
                              (bits(raw, 8, 8) << 10) | (bits(raw, 12, 12) << 11), 12);
                return;
            case 6: case 7:
                d->op = cop == 6 ? OP_c_beqz : OP_c_bnez; d->rs1 = rp1;
                d->imm = sext((bits(cimm5, 2, 1) << 1) | (bits(cimm3, 1, 0) << 3) | (bits(cimm5, 0, 0) << 5) |
                              (bits(cimm5, 4, 3) << 6) | (bits(cimm3, 2, 2) << 8), 9);
                return;
            }
        } else { /* q == 2 */
            switch (cop) {
            case 0: d->op = OP_c_slli; d->rd = d->rs1 = rc1; d->imm = cimm5 | (cimm1 << 5); return;
            case 1: d->op = OP_c_fldsp; d->frd = rc1; d->rs1 = 2;                                   /* :372-383 */
                d->imm = (bits(cimm5, 4, 3) << 3) | (cimm1 << 5) | (bits(cimm5, 2, 0) << 6); return;
            case 2: d->op = OP_c_lwsp; d->rd = rc1; d->rs1 = 2;
                d->imm = (bits(cimm5, 4, 2) << 2) | (cimm1 << 5) | (bits(cimm5, 1, 0) << 6); return;
            case 3: d->op = OP_c_ldsp; d->rd = rc1; d->rs1 = 2;
                d->imm = (bits(cimm5, 4, 3) << 3) | (cimm1 << 5) | (bits(cimm5, 2, 0) << 6); return;
            case 4:
                if (!cimm1) {
                    if (rc2 == 0) { d->op = OP_c_jr; d->rs1 = rc1; }
                    else { d->op = OP_c_mv; d->rd = rc1; d->rs2 = rc2; }
                } else {
                    if (rc2 == 0) {
                        if (rc1 == 0) d->op = OP_c_ebreak;
                        else { d->op = OP_c_jalr; d->rd = 1; d->rs1 = rc1; }
                    } else { d->op = OP_c_add; d->rd = d->rs1 = rc1; d->rs2 = rc2; }
                }
                return;
            case 5: d->op = OP_c_fsdsp; d->frs2 = rc2; d->rs1 = 2;                                  /* :493-503 */
                d->imm = (bits(cimm6, 5, 3) << 3) | (bits(cimm6, 2, 0) << 6); return;
            case 6: d->op = OP_c_swsp; d->rs1 = 2; d->rs2 = rc2; d->imm = (bits(cimm6, 5, 2) << 2) | (bits(cimm6, 1, 0) << 6); return;
            case 7: d->op = OP_c_sdsp; d->rs1 = 2; d->rs2 = rc2; d->imm = (bits(cimm6, 5, 3) << 3) | (bits(cimm6, 2, 0) << 6); return;
            }
        }
        return;
    }
    /* 32-bit: decoder.isa:537-6365 */
    d->len = 4;
    u32 opc = bits(raw, 6, 2), f3 = bits(raw, 14, 12), f7 = bits(raw, 31, 25);
    u32 rd = bits(raw, 11, 7), rs1 = bits(raw, 19, 15), rs2 = bits(raw, 24, 20);
    u32 fs3 = bits(raw, 31, 27);   /* FS3 <31:27> */
    s64 imm_i = sext(bits(raw, 31, 20), 12);
    s64 imm_s = sext((bits(raw, 31, 25) << 5) | bits(raw, 11, 7), 12);
    s64 imm_b = sext((bits(raw, 31, 31) << 12) | (bits(raw, 7, 7) << 11) | (bits(raw, 30, 25) << 5) | (bits(raw, 11, 8) << 1), 13);
    s64 imm_j = sext((bits(raw, 31, 31) << 20) | (bits(raw, 19, 12) << 12) | (bits(raw, 20, 20) << 11) | (bits(raw, 30, 21) << 1), 21);
    d->funct3 = f3;
    switch (opc) {
    case 0x00: {  /* LOAD :538-566 */
        static const int o[8] = {OP_lb, OP_lh, OP_lw, OP_ld, OP_lbu, OP_lhu, OP_lwu, OP_UNKNOWN};
        d->op = o[f3];
        if (d->op != OP_UNKNOWN) { d->rd = rd; d->rs1 = rs1; d->imm = imm_i; }
        return;
    }
    case 0x01: d->op = OP_ESC_FP; return;      /* LOAD-FP / vector loads */
    case 0x03:  /* MISC-MEM :1336-1433 */
        if (f3 == 0) { d->op = OP_fence; return; }
        if (f3 == 1) { d->op = OP_fence_i; return; }
        if (f3 == 2 && rd == 0) {
            u32 f12 = bits(raw, 31, 20);
            if (f12 == 0 || f12 == 1 || f12 == 2 || f12 == 4) { d->op = OP_ESC_CBO; return; }
        }
        return;
    case 0x04:  /* OP-IMM :1435-1670 */
        d->rd = rd; d->rs1 = rs1;
        switch (f3) {
        case 0: d->op = OP_addi; d->imm = imm_i; return;
        case 1:
            switch (fs3) {
            case 0x00: d->op = OP_slli; d->imm = bits(raw, 25, 20); return;
            case 0x02:
                if (rs2 <= 9) { d->op = OP_ESC_CRYPTO; return; }   /* sha256/sha512/sm3 */
                break;
            case 0x05: d->op = OP_bseti; d->imm = bits(raw, 25, 20); return;
            case 0x06: d->op = OP_ESC_CRYPTO; return;             /* aes64im / aes64ks1i (RV64) */
            case 0x09: d->op = OP_bclri; d->imm = bits(raw, 25, 20); return;
            case 0x0d: d->op = OP_binvi; d->imm = bits(raw, 25, 20); return;
            case 0x0c:
                switch (rs2) {
                case 0: d->op = OP_clz; return;
                case 1: d->op = OP_ctz; return;
                case 2: d->op = OP_cpop; return;
                case 4: d->op = OP_sext_b; return;
                case 5: d->op = OP_sext_h; return;
                }
                break;
            }
            break;
        case 2: d->op = OP_slti; d->imm = imm_i; return;
        case 3: d->op = OP_sltiu; d->imm = imm_i; return;
        case 4: d->op = OP_xori; d->imm = imm_i; return;
        case 5:
            switch (fs3) {
            case 0x0: d->op = OP_srli; d->imm = bits(raw, 25, 20); return;
            case 0x5: d->op = OP_orc_b; d->imm = bits(raw, 25, 20); return;
            case 0x8: d->op = OP_srai; d->imm = bits(raw, 25, 20); return;
            case 0x9: d->op = OP_bexti; d->imm = bits(raw, 25, 20); return;
            case 0xc: d->op = OP_rori; d->imm = bits(raw, 25, 20); return;
            case 0xd:
                if (rs2 == 0x18) { d->op = OP_rev8; return; }
                if (rs2 == 0x07) { d->op = OP_ESC_CRYPTO; return; }   /* brev8 */
                break;
            }
            break;
        case 6:
            if (rd == 0) {
                if (rs2 == 0) { d->op = OP_prefetch_i; d->rd = -1; d->imm = bits(raw, 31, 25) << 5; return; }
                if (rs2 == 1) { d->op = OP_prefetch_r; d->rd = -1; d->imm = bits(raw, 31, 25) << 5; return; }
                if (rs2 == 3) { d->op = OP_prefetch_w; d->rd = -1; d->imm = bits(raw, 31, 25) << 5; return; }
                d->op = OP_ori_hint; d->imm = imm_i; return;
            }
            d->op = OP_ori; d->imm = imm_i; return;
        case 7: d->op = OP_andi; d->imm = imm_i; return;
        }
        d->rd = d->rs1 = -1; d->op = OP_UNKNOWN; return;
    case 0x05: d->op = OP_auipc; d->rd = rd; d->imm = sext(bits(raw, 31, 12), 20) * 4096; return;
    case 0x06:  /* OP-IMM-32 :1676-1720 */
        d->rd = rd; d->rs1 = rs1;
        if (f3 == 0) { d->op = OP_addiw; d->imm = imm_i; return; }
        if (f3 == 1) {
            if (fs3 == 0x0) { d->op = OP_slliw; d->imm = bits(raw, 24, 20); return; }
            if (fs3 == 0x1) { d->op = OP_slli_uw; d->imm = bits(raw, 25, 20); return; }
            if (fs3 == 0xc) {
                if (rs2 == 0) { d->op = OP_clzw; return; }
                if (rs2 == 1) { d->op = OP_ctzw; return; }
                if (rs2 == 2) { d->op = OP_cpopw; return; }
            }
        }
        if (f3 == 5) {
            if (fs3 == 0x0) { d->op = OP_srliw; d->imm = bits(raw, 24, 20); return; }
            if (fs3 == 0x8) { d->op = OP_sraiw; d->imm = bits(raw, 24, 20); return; }
            if (fs3 == 0xc) { d->op = OP_roriw; d->imm = bits(raw, 24, 20); return; }
        }
        d->rd = d->rs1 = -1; d->op = OP_UNKNOWN; return;
    case 0x08: {  /* STORE :1722-1739 */
        static const int o[8] = {OP_sb, OP_sh, OP_sw, OP_sd, OP_UNKNOWN, OP_UNKNOWN, OP_UNKNOWN, OP_UNKNOWN};
        d->op = o[f3];
        if (d->op != OP_UNKNOWN) { d->rs1 = rs1; d->rs2 = rs2; d->imm = imm_s; }
        return;
    }
    case 0x09: d->op = OP_ESC_FP; return;      /* STORE-FP / vector stores */
    case 0x0b: d->op = OP_ESC_AMO; return;     /* AMO :2067-2283 */
    case 0x0c: {  /* OP :2285-2613 */
        d->rd = rd; d->rs1 = rs1; d->rs2 = rs2;
        u32 kf5 = bits(raw, 29, 25), bs = bits(raw, 31, 30);
        switch (f3) {
        case 0:
            if (kf5 == 0x00) { if (bs == 0) { d->op = OP_add; return; } if (bs == 1) { d->op = OP_sub; return; } break; }
            if (kf5 == 0x01) { if (bs == 0) { d->op = OP_mul; return; } break; }
            if (kf5 == 0x11 || kf5 == 0x13 || kf5 == 0x15 || kf5 == 0x17) break;   /* RV32-only aes32* */
            if (kf5 == 0x08 || kf5 == 0x09 || kf5 == 0x0a || kf5 == 0x0b || kf5 == 0x0e || kf5 == 0x0f) break; /* RV32 sha512 */
            if (kf5 == 0x18 || kf5 == 0x1a) { d->op = OP_ESC_CRYPTO; return; }     /* sm4ed / sm4ks */
            if (kf5 == 0x19 || kf5 == 0x1b || kf5 == 0x1d) { if (bs == 0) { d->op = OP_ESC_CRYPTO; return; } break; }
            if (kf5 == 0x1f) { if (bs <= 1) { d->op = OP_ESC_CRYPTO; return; } break; }
            break;
        case 1:
            switch (f7) { case 0x0: d->op = OP_sll; return; case 0x1: d->op = OP_mulh; return; case 0x5: d->op = OP_clmul; return;
            case 0x14: d->op = OP_bset; return; case 0x24: d->op = OP_bclr; return; case 0x30: d->op = OP_rol; return;
            case 0x34: d->op = OP_binv; return; }
            break;
        case 2:
            switch (f7) { case 0x0: d->op = OP_slt; return; case 0x1: d->op = OP_mulhsu; return; case 0x5: d->op = OP_clmulr; return;
            case 0x10: d->op = OP_sh1add; return; case 0x14: d->op = OP_ESC_CRYPTO; return; }
            break;
        case 3:
            switch (f7) { case 0x0: d->op = OP_sltu; return; case 0x1: d->op = OP_mulhu; return; case 0x5: d->op = OP_clmulh; return; }
            break;
        case 4:
            switch (f7) { case 0x0: d->op = OP_xor_; return; case 0x1: d->op = OP_div_; return; case 0x4: d->op = OP_pack; return;
            case 0x5: d->op = OP_min_; return; case 0x10: d->op = OP_sh2add; return; case 0x14: d->op = OP_ESC_CRYPTO; return;
            case 0x20: d->op = OP_xnor; return; }
            break;
        case 5:
            switch (f7) { case 0x0: d->op = OP_srl; return; case 0x1: d->op = OP_divu; return; case 0x7: d->op = OP_czero_eqz; return;
            case 0x20: d->op = OP_sra; return; case 0x5: d->op = OP_minu; return; case 0x24: d->op = OP_bext; return;
            case 0x30: d->op = OP_ror; return; }
            break;
        case 6:
            switch (f7) { case 0x0: d->op = OP_or_; return; case 0x1: d->op = OP_rem; return; case 0x5: d->op = OP_max_; return;
            case 0x10: d->op = OP_sh3add; return; case 0x20: d->op = OP_orn; return; }
            break;
        case 7:
            switch (f7) { case 0x0: d->op = OP_and_; return; case 0x1: d->op = OP_remu; return; case 0x4: d->op = OP_packh; return;
            case 0x5: d->op = OP_maxu; return; case 0x7: d->op = OP_czero_nez; return; case 0x20: d->op = OP_andn; return; }
            break;
        }
        d->rd = d->rs1 = d->rs2 = -1; d->op = OP_UNKNOWN; return;
    }
    case 0x0d: d->op = OP_lui; d->rd = rd; d->imm = sext(bits(raw, 31, 12), 20) * 4096; return;
    case 0x0e:  /* OP-32 :2620-2692 */
        d->rd = rd; d->rs1 = rs1; d->rs2 = rs2;
        switch (f3) {
        case 0: switch (f7) { case 0x0: d->op = OP_addw; return; case 0x1: d->op = OP_mulw; return;
                case 0x4: d->op = OP_add_uw; return; case 0x20: d->op = OP_subw; return; } break;
        case 1: switch (f7) { case 0x0: d->op = OP_sllw; return; case 0x30: d->op = OP_rolw; return; } break;
        case 2: if (f7 == 0x10) { d->op = OP_sh1add_uw; return; } break;
        case 4: switch (f7) { case 0x1: d->op = OP_divw; return; case 0x4: d->op = OP_packw; return;
                case 0x10: d->op = OP_sh2add_uw; return; } break;
        case 5: switch (f7) { case 0x0: d->op = OP_srlw; return; case 0x1: d->op = OP_divuw; return;
                case 0x20: d->op = OP_sraw; return; case 0x30: d->op = OP_rorw; return; } break;
        case 6: switch (f7) { case 0x1: d->op = OP_remw; return; case 0x10: d->op = OP_sh3add_uw; return; } break;
        case 7: d->op = OP_remuw; return;          /* decoded on FUNCT3 alone (:2687-2689) */
        }
        d->rd = d->rs1 = d->rs2 = -1; d->op = OP_UNKNOWN; return;
    case 0x10: case 0x11: case 0x12: case 0x13: case 0x14: d->op = OP_ESC_FP; return;
    case 0x15: d->op = OP_ESC_VEC; return;
    case 0x18: {  /* BRANCH :5891-5936 */
        static const int o[8] = {OP_beq, OP_bne, OP_UNKNOWN, OP_UNKNOWN, OP_blt, OP_bge, OP_bltu, OP_bgeu};
        d->op = o[f3];
        if (d->op != OP_UNKNOWN) { d->rs1 = rs1; d->rs2 = rs2; d->imm = imm_b; }
        return;
    }
    case 0x19:  /* JALR :5938-5943 */
        if (f3 == 0) { d->op = OP_jalr; d->rd = rd; d->rs1 = rs1; d->imm = imm_i; }
        return;
    case 0x1b: d->op = OP_jal; d->rd = rd; d->imm = imm_j; return;   /* :5945-5948 */
    case 0x1c:  /* SYSTEM :5950-6300 */
        if (f3 == 0) {
            if (f7 == 0) {
                if (rs2 == 0) { d->op = OP_ecall; return; }
                if (rs2 == 1) { d->op = OP_ebreak; return; }
                return;
            }
            d->op = OP_ESC_SYS; return;
        }
        if (f3 == 4) { d->op = OP_ESC_HYP; return; }
        d->op = OP_csr; d->rd = rd; d->rs1 = (f3 >= 5) ? -1 : (int)rs1; d->csr = bits(raw, 31, 20);
        d->imm = rs1;  /* uimm for csrr*i */
        return;
    case 0x1e: d->op = OP_ESC_M5; return;      /* M5Op :6363 */
    default: return;
    }
}

const char *or_mnemonic(u32 inst) {
    dec_t d; decode(inst, &d);
    static __thread char buf[64];
    if (d.op == OP_UNKNOWN) return "unknown";
    if (d.op < OP_c_addi4spn) { snprintf(buf, sizeof buf, "escape:%s", op_names[d.op]); return buf; }
    if (d.op == OP_csr) {
        static const char *cn[8] = {"?", "csrrw", "csrrs", "csrrc", "?", "csrrwi", "csrrsi", "csrrci"};
        return cn[d.funct3];
    }
#ifdef OR_SOFTFLOAT
    if (d.op >= OP_fadd && d.op <= OP_fcvt_f2f) {   /* gem5's per-format mnemonic */
        static const char *fs[3] = {"h", "s", "d"}, *is[4] = {"w", "wu", "l", "lu"};
        const int fmt = (int)((d.imm >> 3) & 3), sub = (int)((d.imm >> 5) & 7);
        if (d.op == OP_fcvt_f2i) snprintf(buf, sizeof buf, "fcvt_%s_%s", is[sub], fs[fmt]);
        else if (d.op == OP_fcvt_i2f) snprintf(buf, sizeof buf, "fcvt_%s_%s", fs[fmt], is[sub]);
        else if (d.op == OP_fcvt_f2f) snprintf(buf, sizeof buf, "fcvt_%s_%s", fs[fmt], fs[sub]);
        else snprintf(buf, sizeof buf, "%s%s_%s", op_names[d.op],
                      !sub ? "" : (d.op == OP_fmin || d.op == OP_fmax) ? "m" : "q", fs[fmt]);
        return buf;
    }
#endif
    if (d.op == OP_priv) {
        const u32 f7 = bits(inst, 31, 25), rs2 = bits(inst, 24, 20);
        if (bits(inst, 14, 12) == 4) {
            static const char *hn[8][4] = {{"hlv_b", "hlv_bu"}, {"hsv_b", "hsv_b", "hsv_b", "hsv_b"},
                                           {"hlv_h", "hlv_hu", 0, "hlvx_hu"}, {"hsv_h", "hsv_h", "hsv_h", "hsv_h"},
                                           {"hlv_w", "hlv_wu", 0, "hlvx_wu"}, {"hsv_w", "hsv_w", "hsv_w", "hsv_w"},
                                           {"hlv_d"}, {"hsv_d", "hsv_d", "hsv_d", "hsv_d"}};
            /* hsv_* and hlv_d are decoded on FUNCT7 alone (decoder.isa:6240-6297) */
            const char *n = ((f7 & 1) || f7 == 0x36) ? hn[f7 - 0x30][0] : rs2 < 4 ? hn[f7 - 0x30][rs2] : 0;
            return n ? n : "?";
        }
        switch (f7) {
        case 0x08: return rs2 == 2 ? "sret" : "wfi";
        case 0x09: return "sfence_vma";
        case 0x0b: return "sinval_vvma";
        case 0x0c: return rs2 ? "sfence_inval_ir" : "sfence_w_inval";
        case 0x11: return "hfence_vvma";
        case 0x13: return "hinval_vvma";
        case 0x18: return "mret";
        case 0x31: return "hfence_gvma";
        case 0x33: return "hinval_gvma";
        case 0x38: return "mnret";
        default: return "?";
        }
    }
    if (d.op == OP_cbo) {
        static const char *cn[5] = {"cbo_inval", "cbo_clean", "cbo_flush", "?", "cbo_zero"};
        return d.imm <= 4 ? cn[d.imm] : "?";
    }
    if (d.op == OP_m5op) return "M5Op";
    if (d.op == OP_vec) { snprintf(buf, sizeof buf, "vector:%d", (int)d.imm); return buf; }
    if (d.op == OP_vset) {
        static const char *vn[3] = {"vsetvli", "vsetvl", "vsetivli"};
        return vn[(d.imm >> 16) & 3];
    }
    if (d.op == OP_fli || d.op == OP_fround || d.op == OP_fcvtmod) {
        static const char *fs[3] = {"h", "s", "d"};
        const int fmt = (int)((d.imm >> 3) & 3);
        if (d.op == OP_fcvtmod) return "fcvtmod_w_d";
        snprintf(buf, sizeof buf, "%s_%s", d.op == OP_fli ? "fli" : (d.imm >> 5) & 1 ? "froundnx" : "fround", fs[fmt]);
        return buf;
    }
    if (d.op == OP_crypto) return crypto_names[d.imm & 0xFF];
    const char *n = op_names[d.op];
    size_t l = strlen(n);
    if (l && n[l - 1] == '_') { snprintf(buf, sizeof buf, "%.*s", (int)(l - 1), n); return buf; }
    return n;
}

/* ------------------------------------------------- tick-domain hooks (decl) */
static void tk_page(mach_t *m, u64 vpn);
static void tk_frag(mach_t *m, u64 addr, unsigned size, int cmd);
static void tk_unsupported(mach_t *m, const char *why);
static void tk_fetch(mach_t *m, u64 fetch_pc);

/* ---------------------------------------------------------- memory access */
/* SE translation: arch/riscv/tlb.cc:573-604 -> EmulationPageTable::translate
 * (mem/page_table.cc:143-153).  Returns page data or NULL (page-table fault). */
static uint8_t *translate(mach_t *m, u64 vaddr) {
    pte_t *p = pm_find(&m->mem, vaddr >> 12);
    return p ? p->data : NULL;
}
static uint8_t *translate_w(mach_t *m, u64 vaddr) {
    pte_t *p = pm_find(&m->mem, vaddr >> 12);
    if (!p) return NULL;
    if (!p->owned) {
        uint8_t *n = (uint8_t *)malloc(PAGE);
        memcpy(n, p->data, PAGE);
        p->data = n; p->owned = 1;
    }
    return p->data;
}

/* Process::allocateMem for one page, zero-filled (sim/process.cc:318-343). */
static void alloc_page(mach_t *m, u64 vaddr) {
    u64 vpn = vaddr >> 12;
    if (pm_find(&m->mem, vpn)) return;
    uint8_t *n = (uint8_t *)calloc(1, PAGE);
    pm_insert(&m->mem, vpn, n, 1);
    if (m->tkr) tk_page(m, vpn);   /* seWorkload->allocPhysPages: the next free frame */
}

/* MemState::fixupFault, sim/mem_state.cc:387-447.  Returns 1 handled, 0 not
 * handled (panic), -1 fatal("Maximum stack size exceeded"). */
static int fixup_fault(mach_t *m, u64 vaddr) {
    const or_campaign_t *c = m->c;
    for (int i = 0; i < m->nvma; i++)
        if (vaddr >= m->vma[i].lo && vaddr < m->vma[i].hi) { alloc_page(m, vaddr & PAGE_MASK); return 1; }
    (void)c;
    if (vaddr >= m->stack_min && vaddr < STACK_BASE) { alloc_page(m, vaddr & PAGE_MASK); return 1; }
    if (vaddr < m->stack_min && vaddr >= STACK_BASE - MAX_STACK) {
        while (vaddr < m->stack_min) {
            m->stack_min -= PAGE;
            if (STACK_BASE - m->stack_min > MAX_STACK) return -1;
            alloc_page(m, m->stack_min);
        }
        return 1;
    }
    return 0;
}

/* AtomicSimpleCPU::readMem: fragments split at 64-byte lines, each translated
 * separately; the first fragment that faults aborts the access
 * (cpu/simple/atomic.cc:331-434).  fault_va receives the faulting fragment. */
static int mem_read(mach_t *m, u64 addr, unsigned size, u64 *val, u64 *fault_va) {
    uint8_t buf[8];
    unsigned done = 0;
    u64 a = addr;
    while (done < size) {
        unsigned frag = 64 - (unsigned)(a & 63);
        if (frag > size - done) frag = size - done;
        if (a + frag - 1 < a) { *fault_va = a; return F_PGFAULT; }   /* tlb.cc:589-590 */
        uint8_t *pg = translate(m, a);
        if (!pg) { *fault_va = a; return F_PGFAULT; }
        for (unsigned i = 0; i < frag; i++) {
            u64 b = a + i;   /* fragment lies within one page (64-byte line) */
            buf[done + i] = pg[b & (PAGE - 1)];
        }
        if (m->tkr) tk_frag(m, a, frag, OR_TCMD_READ);
        done += frag; a += frag;
    }
    u64 v = 0;
    for (unsigned i = 0; i < size; i++) v |= (u64)buf[i] << (8 * i);
    *val = v;
    m->data_bytes += size;
    return F_NONE;
}
/* AtomicSimpleCPU::writeMem (atomic.cc:437-544): fragments written in order,
 * a faulting second fragment leaves the first one written. */
static int mem_write(mach_t *m, u64 addr, unsigned size, u64 val, u64 *fault_va) {
    unsigned done = 0;
    u64 a = addr;
    while (done < size) {
        unsigned frag = 64 - (unsigned)(a & 63);
        if (frag > size - done) frag = size - done;
        if (a + frag - 1 < a) { *fault_va = a; return F_PGFAULT; }
        uint8_t *pg = translate_w(m, a);
        if (!pg) { *fault_va = a; return F_PGFAULT; }
        for (unsigned i = 0; i < frag; i++) pg[(a + i) & (PAGE - 1)] = (uint8_t)(val >> (8 * (done + i)));
        if (m->tkr) tk_frag(m, a, frag, OR_TCMD_WRITE);
        /* AbstractMemory::checkLockedAddrList: a store erases the lock records
         * of its fragment's 16-byte granule (abstract_mem.cc:290-345) */
        if (m->lock == (a & ~0xFULL)) m->lock = OR_NONE;
        if (m->dbg_wr && a < m->c->text_hi && a + frag > m->c->text_lo) {
            if (m->dbg_wr_n < m->dbg_wr_cap) m->dbg_wr[m->dbg_wr_n] = a;
            m->dbg_wr_n++;
        }
        done += frag; a += frag;
    }
    m->data_bytes += size;
    return F_NONE;
}

/* cbo.zero: AtomicSimpleCPU::writeMem(nullptr data -> zero_array, 64 bytes at
 * a 64-byte-aligned address: one fragment, atomic.cc:437-449) */
static int mem_write_zero64(mach_t *m, u64 ea, u64 *fault_va) {
    uint8_t *pg = translate_w(m, ea);
    if (!pg) { *fault_va = ea; return F_PGFAULT; }
    memset(pg + (ea & (PAGE - 1)), 0, 64);
    if (m->tkr) tk_frag(m, ea, 64, OR_TCMD_WRITE);
    if (m->lock == ea) m->lock = OR_NONE;
    m->data_bytes += 64;
    return F_NONE;
}

/* ------------------------------------------------------------- terminate */
static void finish(mach_t *m, int cls, int sub, int exit_code) {
    m->done = 1;
    m->res.cls = (uint8_t)cls; m->res.sub = (uint8_t)sub; m->res.exit_code = (uint8_t)exit_code;
    m->res.flags = (uint8_t)((m->injected ? 1 : 0) | (m->injected == 2 ? 2 : 0));
    m->res.detail = (u32)m->pc;
    m->res.ninst = m->num_inst;
}

/* ------------------------------------------------------------- memory map */
static int vma_intersects(const mach_t *m, u64 lo, u64 hi) {
    for (int i = 0; i < m->nvma; i++)
        if (m->vma[i].lo < hi && lo < m->vma[i].hi) return 1;
    return 0;
}
/* the page-table half of MemState::isUnmapped (mem_state.cc:84-106) */
static int pt_intersects(const mach_t *m, u64 lo, u64 hi) {
    for (u64 i = 0; i < m->mem.cap; i++) {
        const u64 v = m->mem.tab[i].vpn;
        if (v != UINT64_MAX && (v << 12) >= lo && (v << 12) < hi) return 1;
    }
    return 0;
}
/* MemState::isUnmapped: 1 unmapped, 0 a VMA intersects, -1 panic ("Someone
 * allocated physical memory at VA %p without creating a VMA!") */
static int is_unmapped(const mach_t *m, u64 s, u64 len) {
    if (vma_intersects(m, s, s + len)) return 0;
    if (pt_intersects(m, s, s + len)) return -1;
    return 1;
}
/* MemState::mapRegion (mem_state.cc:172-189): 0 if the list is full (the
 * engine's capacity, not gem5's: the trial escapes) */
static int vma_add(mach_t *m, u64 lo, u64 hi) {
    if (lo >= hi) return 1;
    if (m->nvma == (int)(sizeof(m->vma) / sizeof(m->vma[0]))) return 0;
    m->vma[m->nvma].lo = lo; m->vma[m->nvma].hi = hi; m->nvma++;
    return 1;
}
/* MemState::unmapRegion (mem_state.cc:191-266): VMAs lose [lo, hi), then
 * Process::deallocateMem (process.cc:348-382) unmaps the pages that are
 * mapped (zeroed on deallocation: zeroPages=True, Process.py:55-58). */
static int vma_unmap(mach_t *m, u64 lo, u64 hi) {
    int n = m->nvma;
    if (m->tkr) tk_unsupported(m, "the golden run unmaps memory (freed frames are reused)");
    for (int i = 0; i < n; i++) {
        u64 a = m->vma[i].lo, b = m->vma[i].hi;
        if (!(a < hi && lo < b)) continue;
        if (a < lo && b > hi) {            /* strict superset: split */
            m->vma[i].hi = lo;
            if (!vma_add(m, hi, b)) return 0;
        } else if (a >= lo && b <= hi) {   /* subset: gone */
            m->vma[i].lo = m->vma[i].hi = 0;
        } else if (a < lo) {
            m->vma[i].hi = lo;
        } else {
            m->vma[i].lo = hi;
        }
    }
    int k = 0;
    for (int i = 0; i < m->nvma; i++)
        if (m->vma[i].lo < m->vma[i].hi) m->vma[k++] = m->vma[i];
    m->nvma = k;
    pmap_t n2;
    pm_init(&n2, m->mem.cap);
    for (u64 i = 0; i < m->mem.cap; i++) {
        pte_t *e = &m->mem.tab[i];
        if (e->vpn == UINT64_MAX) continue;
        if ((e->vpn << 12) >= lo && (e->vpn << 12) < hi) { if (e->owned) free(e->data); continue; }
        pm_insert(&n2, e->vpn, e->data, e->owned);
    }
    free(m->mem.tab);
    m->mem = n2;
    return 1;
}
/* Are all bytes [a, a + n) mapped (a read through SETranslatingPortProxy:
 * no fixups on reads, mem/se_translating_port_proxy.cc:50-70)? */
static int proxy_readable(mach_t *m, u64 a, u64 n) {
    if (!n) return 1;
    if (a + n - 1 < a) return 0;
    for (u64 v = a >> 12; v <= ((a + n - 1) >> 12); v++)
        if (!pm_find(&m->mem, v)) return 0;
    return 1;
}
/* A write through the proxy (NextPage: fixupFault for each missing page);
 * 0 = fatal, -1 = "Maximum stack size exceeded". */
static int fixup_fault(mach_t *m, u64 vaddr);
static int proxy_writable(mach_t *m, u64 a, u64 n) {
    if (!n) return 1;
    if (a + n - 1 < a) return 0;
    for (u64 v = a >> 12; v <= ((a + n - 1) >> 12); v++) {
        if (pm_find(&m->mem, v)) continue;
        const int h = fixup_fault(m, v << 12 > a ? v << 12 : a);
        if (h != 1) return h;
    }
    return 1;
}
static void proxy_write(mach_t *m, u64 a, const uint8_t *src, u64 n) {
    for (u64 i = 0; i < n; i++) {
        uint8_t *pg = translate_w(m, a + i);
        pg[(a + i) & (PAGE - 1)] = src[i];
    }
}

/* ------------------------------------------------------------- syscalls */
/* Classification of the RV64 Linux syscall table (arch/riscv/linux/
 * se_workload.cc:529-895; pinned by tests/golden/syscalls_rv64.json):
 *   0 absent (fatal "out of range", syscall_desc.hh:204-214)
 *   1 present without a handler (unimplementedFunc -> fatal, syscall_emul.cc:77)
 *   2 ignoreFunc / ignoreWarnOnceFunc (returns 0, syscall_emul.cc:84-104)
 *   3 a real gem5 handler this engine does not model (escape)
 *   4 modelled here (write, exit, exit_group, get*id) */
static const uint16_t sys_impl_escape[] = {
    17, 23, 25, 29, 33, 34, 35, 38, 43, 44, 45, 46, 47, 48, 49, 52, 55, 56, 57, 59, 61, 62, 63, 66, 67, 68,
    78, 79, 80, 96, 98, 113, 114, 121, 123, 131, 153, 154, 160, 163, 165, 166, 168, 169, 179, 198, 199, 200,
    201, 202, 203, 204, 205, 206, 207, 208, 209, 210, 211, 212, 214, 215, 216, 220, 221, 222, 258, 260, 261,
    278, 435, 1024, 1025, 1026, 1027, 1028, 1029, 1030, 1031, 1033, 1034, 1035, 1036, 1037, 1038, 1039, 1040,
    1041, 1044, 1047, 1048, 1049, 1050, 1051, 1052, 1054, 1055, 1056, 1057, 1058, 1060, 1062, 1065, 1067, 1068};
/* modelled: the deterministic handlers (syscall_emul.{cc,hh}, se_workload.cc) */
static int sys_modelled(int num) {
    switch (num) {
    case 29: case 57: case 63: case 64: case 66: case 78: case 93: case 94: case 96: case 113: case 160: case 163:
    case 214: case 215: case 222: case 258: case 261: case 278: case 1058:
        return 1;
    default:
        return num >= 172 && num <= 178;
    }
}
int or_sys_class(int num) {
    if (sys_modelled(num)) return 4;
    int present = (num >= 0 && num <= 64) || (num >= 66 && num <= 243) || num == 258 ||
                  (num >= 260 && num <= 287) || (num >= 424 && num <= 450) || (num >= 1024 && num <= 1079) ||
                  num == 2011;
    if (!present) return 0;
    if (num == 99 || num == 100 || num == 101 || num == 124 || (num >= 133 && num <= 139) || num == 146 ||
        num == 164 || (num >= 226 && num <= 233) || num == 235)
        return 2;
    for (size_t i = 0; i < sizeof(sys_impl_escape) / sizeof(sys_impl_escape[0]); i++)
        if (sys_impl_escape[i] == num) return 3;
    return 1;
}

/* resource escapes here are the bounds the engine shares (the VMA list, the
 * precomputed getrandom stream): exit code 1 marks them, as on the device
 * (fi_trial.hip kEscTable); 0 is the device's private-page exhaustion, which
 * the oracle does not have */
#define ESC_TABLE 1
#define EBADF_ 9
#define EINVAL_ 22
#define ENOTTY_ 25
#define EPERM_ 1
static u64 round_up(u64 v) { return (v + PAGE - 1) & ~(PAGE - 1); }   /* base/intmath.hh roundUp (wraps) */
/* Ranges the VM handlers walk page by page (MemState::isUnmapped, Process::
 * deallocateMem, whose page count is an int) are bounded here: a longer one
 * is a host-side hazard the engine does not model (escape). */
#define VM_MAX_LEN (1ULL << 43)
static void vm_escape(mach_t *m, int num) { finish(m, OR_ESCAPE, OR_ESC_SYSCALL, 0); m->res.detail = (u32)num; }
/* an SE handler panics (e.g. "Accessing null ProxyPtr", MemState::isUnmapped) */
static void se_panic(mach_t *m) { finish(m, OR_CRASH, OR_CRASH_SE_PANIC, 134); }

/* writevFunc<RiscvLinux64> (syscall_emul.hh:1964-1996): the iovecs and their
 * buffers are read through the proxy in order (fatal on an unmapped byte),
 * then host writev() on the target fd */
/* std::mt19937_64 (Matsumoto & Nishimura; the C++ standard's parameters),
 * seeded as gem5's Random(globalSeed) does (gen.seed(uint32 seed)) */
static u64 mt64_next(mach_t *m) {
    enum { N = 312, M = 156 };
    if (!m->mt) {
        m->mt = (u64 *)malloc(N * sizeof(u64));
        m->mt[0] = (u64)(uint32_t)m->c->rnd_seed;
        for (int i = 1; i < N; i++) m->mt[i] = 6364136223846793005ULL * (m->mt[i - 1] ^ (m->mt[i - 1] >> 62)) + (u64)i;
        m->mt_i = N;
    }
    if (m->mt_i >= N) {
        for (int i = 0; i < N; i++) {
            const u64 x = (m->mt[i] & 0xFFFFFFFF80000000ULL) | (m->mt[(i + 1) % N] & 0x7FFFFFFFULL);
            m->mt[i] = m->mt[(i + M) % N] ^ (x >> 1) ^ ((x & 1) ? 0xB5026F5AA96619E9ULL : 0);
        }
        m->mt_i = 0;
    }
    u64 y = m->mt[m->mt_i++];
    y ^= (y >> 29) & 0x5555555555555555ULL;
    y ^= (y << 17) & 0x71D67FFFEDA60000ULL;
    y ^= (y << 37) & 0xFFF7EEE000000000ULL;
    y ^= y >> 43;
    return y;
}

static void sys_writev(mach_t *m) {
    const int fd = (int)(s32)(u32)m->x[10];
    const u64 iov = m->x[11], cnt = m->x[12];
    if (fd < 0 || fd >= 1024) { finish(m, OR_CRASH, OR_CRASH_FD_ASSERT, 134); return; }   /* fd_array.cc:322 */
    if (fd > 2 || ((m->fdc >> fd) & 1)) { m->x[10] = (u64)(s64)-EBADF_; return; }
    if (fd == 0 && !m->c->in_data) { finish(m, OR_ESCAPE, OR_ESC_HOST, 0); return; }   /* host stdin */
    if (cnt > (1u << 20)) { finish(m, OR_ESCAPE, OR_ESC_HOST, 0); return; }    /* host allocation */
    u64 total = 0;
    for (u64 i = 0; i < cnt; i++) {
        const u64 e = iov + 16 * i;
        if (e < iov || !proxy_readable(m, e, 16)) { finish(m, OR_CRASH, OR_CRASH_PROXY, 1); return; }
        u64 base = 0, len = 0;
        for (int k = 0; k < 8; k++) {
            base |= (u64)translate(m, e + k)[(e + k) & (PAGE - 1)] << (8 * k);
            len |= (u64)translate(m, e + 8 + k)[(e + 8 + k) & (PAGE - 1)] << (8 * k);
        }
        if (len > (1ULL << 31)) { finish(m, OR_ESCAPE, OR_ESC_HOST, 0); return; }
        if (!proxy_readable(m, base, len)) { finish(m, OR_CRASH, OR_CRASH_PROXY, 1); return; }
        total += len;
    }
    /* the input file (O_RDONLY): host writev fails with EBADF before it looks at IOV_MAX */
    if (fd == 0) { m->x[10] = (u64)(s64)-EBADF_; return; }
    if (cnt > 1024) { m->x[10] = (u64)(s64)-EINVAL_; return; }   /* host writev: IOV_MAX */
    if (total > (1ULL << 31)) { finish(m, OR_ESCAPE, OR_ESC_HOST, 0); return; }
    bytes_t *dst = fd == 1 ? &m->out : &m->err;
    for (u64 i = 0; i < cnt; i++) {
        const u64 e = iov + 16 * i;
        u64 base = 0, len = 0;
        for (int k = 0; k < 8; k++) {
            base |= (u64)translate(m, e + k)[(e + k) & (PAGE - 1)] << (8 * k);
            len |= (u64)translate(m, e + 8 + k)[(e + 8 + k) & (PAGE - 1)] << (8 * k);
        }
        for (u64 j = 0; j < len; j++) {
            const uint8_t ch = translate(m, base + j)[(base + j) & (PAGE - 1)];
            by_push(dst, &ch, 1);
        }
    }
    m->x[10] = total;
}

/* mmapFunc<RiscvLinux64> (syscall_emul.hh:2002-2126) for anonymous mappings,
 * MemState::extendMmap (mem_state.cc:450-477: the region grows down from
 * mmap_end, RiscvProcess64 mmap_end = 0x4000000000000000, process.cc:79). */
static void sys_mmap(mach_t *m) {
    u64 start = m->x[10], len = m->x[11];
    const int flags = (int)(s32)(u32)m->x[13], fd = (int)(s32)(u32)m->x[14];
    const u64 off = m->x[15];
    if ((start & (PAGE - 1)) || (off & (PAGE - 1)) || ((flags & 2) && (flags & 1)) || (!(flags & 2) && !(flags & 1)) ||
        !len) { m->x[10] = (u64)(s64)-EINVAL_; return; }
    if (len > VM_MAX_LEN) { vm_escape(m, 222); return; }
    len = round_up(len);
    if (!(flags & 0x20)) {   /* file-backed: the fd table entry */
        if (fd < 0 || fd >= 1024) { finish(m, OR_CRASH, OR_CRASH_FD_ASSERT, 134); return; }
        if (fd > 2 || ((m->fdc >> fd) & 1)) { m->x[10] = (u64)(s64)-EBADF_; return; }
        finish(m, OR_ESCAPE, OR_ESC_HOST, 0);   /* a host file mapping */
        return;
    }
    if (start + len < start) { vm_escape(m, 222); return; }
    if (!(flags & 0x10)) {
        int u = 0;
        if (start) {
            u = is_unmapped(m, start, len);
            if (u < 0) { se_panic(m); return; }
        }
        if (!u) {
            u64 s2 = m->mmap_end - len;
            for (;;) {
                if (s2 > m->mmap_end) { vm_escape(m, 222); return; }   /* wrapped below 0 */
                int hit = -1;
                for (int i = 0; i < m->nvma; i++)
                    if (m->vma[i].lo < s2 + len && s2 < m->vma[i].hi) { hit = i; break; }
                if (hit < 0) break;
                s2 = m->vma[hit].lo - len;   /* the page-by-page scan lands right below it */
            }
            if (pt_intersects(m, s2, s2 + len)) { se_panic(m); return; }
            m->mmap_end = s2;
            start = s2;
        }
    } else if (!vma_unmap(m, start, start + len)) {
        finish(m, OR_ESCAPE, OR_ESC_RESOURCE, ESC_TABLE); return;
    }
    if (!vma_add(m, start, start + len)) { finish(m, OR_ESCAPE, OR_ESC_RESOURCE, ESC_TABLE); return; }
    m->x[10] = start;
}

/* readlinkatFunc (syscall_emul.hh:1066-1129): the path string is read through
 * the proxy (an unmapped byte: -EFAULT); a relative path with a dirfd other
 * than AT_FDCWD takes atSyscallPath (:356-374: (*fds)[dirfd] asserts the
 * range, no FileFDEntry -> -EBADF, an open stdio entry prefixes its host file
 * name: host); "/proc/self/exe" answers realpath(progName()) strncpy'd into a
 * BufferArg of bufsiz bytes (NUL-padded) copied out through the proxy, the
 * result min(strlen, bufsiz); any other path reads the host file system. */
#define OR_AT_FDCWD (-100)
static void sys_readlinkat(mach_t *m) {
    const int dirfd = (int)(s32)(u32)m->x[10];
    const u64 pathp = m->x[11], buf = m->x[12], bufsiz = m->x[13];
    char path[4096];
    u64 n = 0;
    for (;; n++) {
        if (n == sizeof path) { finish(m, OR_ESCAPE, OR_ESC_HOST, 0); return; }   /* longer than PATH_MAX */
        const uint8_t *pg = translate(m, pathp + n);
        if (!pg || pathp + n < pathp) { m->x[10] = (u64)(s64)-14; return; }    /* -EFAULT */
        path[n] = (char)pg[(pathp + n) & (PAGE - 1)];
        if (!path[n]) break;
    }
    if (path[0] != '/' && dirfd != OR_AT_FDCWD) {
        if (dirfd < 0 || dirfd >= 1024) { finish(m, OR_CRASH, OR_CRASH_FD_ASSERT, 134); return; }
        if (dirfd > 2 || ((m->fdc >> dirfd) & 1)) { m->x[10] = (u64)(s64)-EBADF_; return; }
        finish(m, OR_ESCAPE, OR_ESC_HOST, 0);
        return;
    }
    if (strcmp(path, "/proc/self/exe") || !m->c->exe_path[0] || bufsiz > (1ULL << 20)) {
        finish(m, OR_ESCAPE, OR_ESC_HOST, 0);
        return;
    }
    const u64 len = strlen(m->c->exe_path);
    uint8_t *tmp = (uint8_t *)calloc(bufsiz ? bufsiz : 1, 1);
    memcpy(tmp, m->c->exe_path, len < bufsiz ? len : bufsiz);
    const int h = proxy_writable(m, buf, bufsiz);
    if (h == 0) { free(tmp); finish(m, OR_CRASH, OR_CRASH_PROXY, 1); return; }
    if (h < 0) { free(tmp); finish(m, OR_CRASH, OR_CRASH_STACK_LIMIT, 1); return; }
    proxy_write(m, buf, tmp, bufsiz);
    free(tmp);
    m->x[10] = len > bufsiz ? bufsiz : len;
}

/* riscvHWProbeFunc (arch/riscv/linux/se_workload.cc:221-527) for one thread
 * context (cpumask_malloc: 8 bytes, CPU 0 online) under the SE ISA (misa
 * IMAFDCV + S/U, mvendorid = marchid = mimpid = 0, isa.cc:359-364).
 * pairs are {int64 key, uint64 value}; BufferArg copyIn / copyOut are
 * readBlob (fatal if unmapped) / writeBlob through the allocating proxy. */
static int hw_read(mach_t *m, u64 a, u64 n, uint8_t *dst) {
    if (!proxy_readable(m, a, n)) return 0;
    for (u64 i = 0; i < n; i++) dst[i] = translate(m, a + i)[(a + i) & (PAGE - 1)];
    return 1;
}
static u64 hw_one(mach_t *m, s64 *key) {
    switch (*key) {
    case 0: case 1: case 2: return 0;                 /* mvendorid / marchid / mimpid */
    case 3: return 1;                                 /* BaseBehavior: ima */
    case 4: return (1ULL << 0) | (1ULL << 1) | (1ULL << 2) | (0x3FFFULL << 3) | (1ULL << 28) | (1ULL << 29) |
                   (1ULL << 31) | (1ULL << 32) | (1ULL << 33) | (1ULL << 36) | (1ULL << 42) | (1ULL << 45) |
                   (1ULL << 46) | (1ULL << 47);      /* IMAExt0 (linux.hh:68-118) */
    case 5: case 9: return 2;                         /* Cpuperf0 / MisalignedScalarPerf: Slow */
    case 6: return 64;                                /* ZicbozBlockSize: cacheLineSize() */
    case 7: return m->mmap_end;                       /* HighestVirtAddress: MemState::getMmapEnd() */
    default: *key = -1; return 0;                     /* unknown (incl. TimeCsrFreq) */
    }
}
static void sys_hwprobe(mach_t *m) {
    const u64 pairs = m->x[10], count = m->x[11], cpus_user = m->x[13];
    u64 cpusetsize = m->x[12];
    const u32 flags = (u32)m->x[14];
    if (count > (1ULL << 16)) { finish(m, OR_ESCAPE, OR_ESC_HOST, 0); return; }   /* BufferArg(int size) */
    const u64 psz = 16 * count;
    uint8_t *pb = (uint8_t *)malloc(psz ? psz : 1);
    uint8_t ub[8] = {0};
    int ret = 0;
    if (flags & 1) {   /* hwprobe_get_cpus */
        if (flags != 1 || cpusetsize == 0 || !cpus_user) { ret = -EINVAL_; goto out; }
        if (cpusetsize > 8) cpusetsize = 8;
        const u64 usz = cpusetsize;
        if (!hw_read(m, cpus_user, usz, ub)) { free(pb); finish(m, OR_CRASH, OR_CRASH_PROXY, 1); return; }
        u64 cpus = 0;
        memcpy(&cpus, ub, usz);
        if (!cpus) { cpus = 1; cpusetsize = 8; }
        cpus &= 1;
        if (!hw_read(m, pairs, psz, pb)) { free(pb); finish(m, OR_CRASH, OR_CRASH_PROXY, 1); return; }
        for (u64 i = 0; i < count; i++) {
            s64 key; u64 val;
            memcpy(&key, pb + 16 * i, 8); memcpy(&val, pb + 16 * i + 8, 8);
            if (key < 0 || key > 9) {
                key = -1; val = 0;
                memcpy(pb + 16 * i, &key, 8); memcpy(pb + 16 * i + 8, &val, 8);
                /* memset(cpus_user_buf, 0, cpusetsize): past the buffer when the size grew */
                if (cpusetsize > usz) { free(pb); finish(m, OR_ESCAPE, OR_ESC_UNDEF, 0); return; }
                memset(ub, 0, cpusetsize);
                break;
            }
            /* cpumask_test_cpu reads bits[cpu / 8]: beyond the one-word mask
             * (undefined) once the loop passes cpu 7 */
            if (cpusetsize > 1) { free(pb); finish(m, OR_ESCAPE, OR_ESC_UNDEF, 0); return; }
            if (cpus & 1) {
                s64 k2 = key;
                const u64 v2 = hw_one(m, &k2);
                const int bitmask = key == 3 || key == 4 || key == 5;
                const int match = k2 == key && (bitmask ? (v2 & val) == val : v2 == val);
                if (!match) cpus &= ~1ULL;
            }
        }
        const int h = proxy_writable(m, pairs, psz);
        if (h == 0) { free(pb); finish(m, OR_CRASH, OR_CRASH_PROXY, 1); return; }
        if (h < 0) { free(pb); finish(m, OR_CRASH, OR_CRASH_STACK_LIMIT, 1); return; }
        proxy_write(m, pairs, pb, psz);
        const int h2 = proxy_writable(m, cpus_user, usz);
        if (h2 == 0) { free(pb); finish(m, OR_CRASH, OR_CRASH_PROXY, 1); return; }
        if (h2 < 0) { free(pb); finish(m, OR_CRASH, OR_CRASH_STACK_LIMIT, 1); return; }
        proxy_write(m, cpus_user, ub, usz);
        goto out;
    }
    /* hwprobe_get_values */
    if (flags != 0) { ret = -EINVAL_; goto out; }
    if (cpusetsize > 8) cpusetsize = 8;
    if (!(cpusetsize == 0 && !cpus_user)) {
        if (!hw_read(m, cpus_user, cpusetsize, ub)) { free(pb); finish(m, OR_CRASH, OR_CRASH_PROXY, 1); return; }
        u64 cpus = 0;
        memcpy(&cpus, ub, cpusetsize);
        /* cpumask_and / cpumask_empty walk cpusetsize / 8 words */
        if (cpusetsize < 8 || !(cpus & 1)) { ret = -EINVAL_; goto out; }
    }
    if (!hw_read(m, pairs, psz, pb)) { free(pb); finish(m, OR_CRASH, OR_CRASH_PROXY, 1); return; }
    for (u64 i = 0; i < count; i++) {
        s64 key;
        memcpy(&key, pb + 16 * i, 8);
        const u64 val = hw_one(m, &key);
        memcpy(pb + 16 * i, &key, 8); memcpy(pb + 16 * i + 8, &val, 8);
    }
    {
        const int h = proxy_writable(m, pairs, psz);
        if (h == 0) { free(pb); finish(m, OR_CRASH, OR_CRASH_PROXY, 1); return; }
        if (h < 0) { free(pb); finish(m, OR_CRASH, OR_CRASH_STACK_LIMIT, 1); return; }
        proxy_write(m, pairs, pb, psz);
    }
out:
    free(pb);
    m->x[10] = (u64)(s64)ret;
}

static void do_syscall(mach_t *m) {
    /* EmuLinux::syscall: num = (int) a7 (se_workload.cc:95-106, syscall_desc.hh:204) */
    int num = (int)(s32)(u32)m->x[17];
    int cls = or_sys_class(num);
    if (cls == 0) { finish(m, OR_CRASH, OR_CRASH_SYSCALL_RANGE, 1); m->res.detail = (u32)num; return; }
    if (cls == 1) { finish(m, OR_CRASH, OR_CRASH_SYSCALL_UNIMPL, 1); m->res.detail = (u32)num; return; }
    if (cls == 3) { finish(m, OR_ESCAPE, OR_ESC_SYSCALL, 0); m->res.detail = (u32)num; return; }
    if (cls == 2) { m->x[10] = 0; return; }
    switch (num) {
    case 93: case 94: {   /* exitImpl -> exitSimLoop(status & 0xff) (syscall_emul.cc:120-248) */
        int status = (int)(s32)(u32)m->x[10];
        if (m->ctid) {   /* exitFutexWake: clear *childClearTID through the proxy (syscall_emul.cc:106-117) */
            const int h = proxy_writable(m, m->ctid, 8);
            if (h == 0) { finish(m, OR_CRASH, OR_CRASH_PROXY, 1); return; }
            if (h < 0) { finish(m, OR_CRASH, OR_CRASH_STACK_LIMIT, 1); return; }
        }
        int code = status & 0xff;
        const or_campaign_t *c = m->c;
        /* masked: the golden output and exit code, ended the way the golden run ended */
        int same = c->have_golden && code == (int)c->golden.exit_code && c->gsub == OR_END_EXIT &&
                   m->out.len == c->gout.len && m->err.len == c->gerr.len &&
                   (m->out.len == 0 || !memcmp(m->out.buf, c->gout.buf, m->out.len)) &&
                   (m->err.len == 0 || !memcmp(m->err.buf, c->gerr.buf, m->err.len));
        finish(m, same ? OR_MASKED : OR_SDC, 0, code);
        return;
    }
    case 172: m->x[10] = PID; return;     /* getpid -> tgid (syscall_emul.cc:822-826) */
    case 173: m->x[10] = PPID; return;
    case 174: case 175: m->x[10] = UID; return;
    case 176: case 177: m->x[10] = GID; return;
    case 178: m->x[10] = PID; return;     /* gettid -> pid */
    case 96: m->ctid = m->x[10]; m->x[10] = PID; return;   /* setTidAddressFunc (syscall_emul.cc:292-299) */
    case 57: {   /* closeFunc -> FDArray::closeFDEntry (fd_array.cc:334-352): 0 for any fd in range */
        const int fd = (int)(s32)(u32)m->x[10];
        if (fd < 0 || fd >= 1024) { m->x[10] = (u64)(s64)-EBADF_; return; }
        if (fd <= 2) m->fdc |= 1u << fd;
        m->x[10] = 0;
        return;
    }
    case 29: {   /* ioctlFunc (syscall_emul.hh:743-813): tty requests first, then the fd entry */
        const int fd = (int)(s32)(u32)m->x[10];
        const u32 req = (u32)m->x[11];
        if (req == 0x5401 || req == 0x5405 || req == 0x5407 || req == 0x541B) { m->x[10] = (u64)(s64)-ENOTTY_; return; }
        if (fd < 0 || fd >= 1024) { finish(m, OR_CRASH, OR_CRASH_FD_ASSERT, 134); return; }
        m->x[10] = (u64)(s64)-ENOTTY_;   /* not a device or socket entry */
        return;
    }
    case 66: sys_writev(m); return;
    case 222: case 1058: sys_mmap(m); return;
    case 215: {   /* munmapFunc (syscall_emul.hh:3140-3156) */
        const u64 st = m->x[10];
        u64 len = m->x[11];
        if (st & (PAGE - 1)) { m->x[10] = (u64)(s64)-EINVAL_; return; }
        if (len > VM_MAX_LEN) { vm_escape(m, 215); return; }
        len = round_up(len);
        if (st + len < st) { vm_escape(m, 215); return; }
        if (!vma_unmap(m, st, st + len)) { finish(m, OR_ESCAPE, OR_ESC_RESOURCE, ESC_TABLE); return; }
        m->x[10] = 0;
        return;
    }
    case 214: {   /* brkFunc (syscall_emul.cc:268-289), MemState::updateBrkRegion (mem_state.cc:107-170) */
        const u64 nb = m->x[10], ob = m->brk;
        if (nb == 0 || nb == ob) { m->x[10] = ob; return; }
        const u64 na = round_up(nb), oa = round_up(ob);
        if ((na > oa ? na - oa : oa - na) > VM_MAX_LEN) { vm_escape(m, 214); return; }
        if (nb < ob) {
            if (oa - na > 0 && !vma_unmap(m, na, oa)) { finish(m, OR_ESCAPE, OR_ESC_RESOURCE, ESC_TABLE); return; }
            m->brk = nb;
            m->x[10] = nb;
            return;
        }
        if (na > oa) {
            const int u = is_unmapped(m, oa, na - oa);
            if (u < 0) { se_panic(m); return; }
            if (!u) { m->x[10] = ob; return; }   /* existing mappings impede the heap */
            if (!vma_add(m, oa, na)) { finish(m, OR_ESCAPE, OR_ESC_RESOURCE, ESC_TABLE); return; }
        }
        m->brk = nb;
        m->x[10] = nb;
        return;
    }
    case 163: case 261: {   /* getrlimitFunc / prlimitFunc (syscall_emul.hh:2197-2265) */
        const u64 rlp = num == 163 ? m->x[11] : m->x[13];
        if (rlp && !proxy_readable(m, rlp, 16)) { finish(m, OR_CRASH, OR_CRASH_PROXY, 1); return; }   /* VPtr load */
        if (num == 261 && (int)(s32)(u32)m->x[10] != 0) { m->x[10] = (u64)(s64)-EPERM_; return; }
        if (num == 261 && !rlp) { m->x[10] = 0; return; }
        const s64 res = num == 163 ? (s64)(u32)m->x[10] : (s64)(s32)(u32)m->x[11];
        u64 lim;
        if (res == 3) lim = 8ULL << 20;                     /* RLIMIT_STACK */
        else if (res == 2) lim = 256ULL << 20;              /* RLIMIT_DATA */
        else if (res == 6 && num == 163) lim = 1;           /* RLIMIT_NPROC: system thread contexts (1) */
        else { m->x[10] = (u64)(s64)-EINVAL_; return; }
        if (!rlp) { se_panic(m); return; }                  /* null ProxyPtr */
        uint8_t b[16];
        for (int k = 0; k < 8; k++) b[k] = b[8 + k] = (uint8_t)(lim >> (8 * k));
        proxy_write(m, rlp, b, 16);
        m->x[10] = 0;
        return;
    }
    case 278: {   /* getrandomFunc (syscall_emul.hh:3222-3236): count bytes of gen() % 255 */
        const u64 buf = m->x[10], cnt = m->x[11];
        if (cnt > (1ULL << 31)) { finish(m, OR_ESCAPE, OR_ESC_HOST, 0); return; }   /* host buffer */
        /* the engine precomputes the first 1 MiB of the stream: beyond it, a
         * resource escape on both sides */
        if (m->rnd_pos + cnt > (1ULL << 20)) { finish(m, OR_ESCAPE, OR_ESC_RESOURCE, ESC_TABLE); return; }
        m->rnd_pos += cnt;
        uint8_t *tmp = (uint8_t *)malloc(cnt ? cnt : 1);
        for (u64 i = 0; i < cnt; i++) tmp[i] = (uint8_t)(mt64_next(m) % 255);
        const int h = proxy_writable(m, buf, cnt);
        if (h == 0) { free(tmp); finish(m, OR_CRASH, OR_CRASH_PROXY, 1); return; }
        if (h < 0) { free(tmp); finish(m, OR_CRASH, OR_CRASH_STACK_LIMIT, 1); return; }
        proxy_write(m, buf, tmp, cnt);
        free(tmp);
        m->x[10] = cnt;
        return;
    }
    case 113: {   /* clock_gettimeFunc (syscall_emul.hh:2266-2278): curTick() / 1000 ns since the
                   * first tick (tick = (cycles so far - 1) x period) + seconds_since_epoch (1e9) */
        const u64 tp = m->x[11];
        if (!tp) { se_panic(m); return; }
        if (!proxy_readable(m, tp, 16)) { finish(m, OR_CRASH, OR_CRASH_PROXY, 1); return; }
        if (m->tkr) tk_unsupported(m, "the golden run reads curTick (clock_gettime)");
        if (m->tki) { finish(m, OR_ESCAPE, OR_ESC_TIMING, OR_TK_CLOCK); return; }
        const u64 ns = (m->c->tick0 + (m->num_cycles - 1) * m->c->clk_period) / 1000;
        const u64 sec = ns / 1000000000ULL + 1000000000ULL, nsec = ns % 1000000000ULL;
        uint8_t b[16];
        for (int k = 0; k < 8; k++) { b[k] = (uint8_t)(sec >> (8 * k)); b[8 + k] = (uint8_t)(nsec >> (8 * k)); }
        proxy_write(m, tp, b, 16);
        m->x[10] = 0;
        return;
    }
    case 160: {   /* unameFunc64 (arch/riscv/linux/se_workload.cc:109-122), Linux::utsname = 5 x 65 chars */
        const u64 p = m->x[10];
        if (!p) { se_panic(m); return; }
        if (!proxy_readable(m, p, 325)) { finish(m, OR_CRASH, OR_CRASH_PROXY, 1); return; }
        static const char *f[5] = {"Linux", "sim.gem5.org", "5.1.0", "#1 Mon Aug 18 11:32:15 EDT 2003", "riscv64"};
        for (int k = 0; k < 5; k++) proxy_write(m, p + 65 * k, (const uint8_t *)f[k], strlen(f[k]) + 1);
        m->x[10] = 0;
        return;
    }
    case 63: {  /* readFunc (syscall_emul.hh:2798-2822): (*fds)[fd] asserts 0 <= fd < 1024 (fd_array.cc:322);
                 * an fd without a host-backed entry reads as -EBADF; the open stdio entries read host files */
        int fd = (int)(s32)(u32)m->x[10];
        if (fd < 0 || fd >= 1024) { finish(m, OR_CRASH, OR_CRASH_FD_ASSERT, 134); return; }
        if (fd > 2 || ((m->fdc >> fd) & 1)) { m->x[10] = (u64)(s64)-EBADF_; return; }
        if (fd != 0 || !m->c->in_data) { finish(m, OR_ESCAPE, OR_ESC_HOST, 0); return; }   /* host stdin/stdout */
        /* Process.input is a file (fd_array.cc:69-75): poll() on a regular
         * file is ready (no retry); read() takes min(n, left) bytes at the
         * file offset; BufferArg (zero-filled, syscall_emul_buf.hh:55-85)
         * copies all n bytes out when the read returned any */
        const u64 buf = m->x[11], n = m->x[12];
        if (n > (1ULL << 31)) { finish(m, OR_ESCAPE, OR_ESC_HOST, 0); return; }   /* host buffer */
        const u64 left = m->c->in_len - m->in_pos, k = n < left ? n : left;
        if (k) {
            const int h = proxy_writable(m, buf, n);
            if (h == 0) { finish(m, OR_CRASH, OR_CRASH_PROXY, 1); return; }
            if (h < 0) { finish(m, OR_CRASH, OR_CRASH_STACK_LIMIT, 1); return; }
            proxy_write(m, buf, m->c->in_data + m->in_pos, k);
            static const uint8_t zero[256];
            for (u64 i = k; i < n; i += sizeof zero) proxy_write(m, buf + i, zero, n - i < sizeof zero ? n - i : sizeof zero);
        }
        m->in_pos += k;
        m->x[10] = k;
        return;
    }
    case 78: sys_readlinkat(m); return;
    case 258: sys_hwprobe(m); return;
    case 64: {  /* writeFunc<RiscvLinux64>(int fd, VPtr buf, size_t n) syscall_emul.hh:2826-2860 */
        int fd = (int)(s32)(u32)m->x[10];
        u64 buf = m->x[11], n = m->x[12];
        if (fd < 0 || fd >= 1024) { finish(m, OR_CRASH, OR_CRASH_FD_ASSERT, 134); return; }  /* fd_array.cc:322 */
        if (fd > 2 || ((m->fdc >> fd) & 1)) { m->x[10] = (u64)(s64)-9; return; }   /* no entry: -EBADF */
        if (fd == 0 && !m->c->in_data) { finish(m, OR_ESCAPE, OR_ESC_HOST, 0); return; }   /* host stdin poll/write */
        if (n > (1ULL << 31)) { finish(m, OR_ESCAPE, OR_ESC_HOST, 0); return; } /* host allocation */
        /* BufferArg::copyIn -> readBlob: fatal if any byte is unmapped (no fixup on reads) */
        if (n) {
            u64 last = buf + n - 1;
            if (last < buf) { finish(m, OR_CRASH, OR_CRASH_PROXY, 1); return; }
            for (u64 v = buf >> 12; v <= (last >> 12); v++)
                if (!pm_find(&m->mem, v)) { finish(m, OR_CRASH, OR_CRASH_PROXY, 1); return; }
        }
        /* fd 0 is the input file, opened O_RDONLY (fd_array.cc:69-75): the
         * host write() fails with EBADF (a regular file polls writable) */
        if (fd == 0) { m->x[10] = (u64)(s64)-EBADF_; return; }
        bytes_t *dst = fd == 1 ? &m->out : &m->err;
        for (u64 i = 0; i < n; i++) {
            uint8_t *pg = translate(m, buf + i);
            uint8_t ch = pg[(buf + i) & (PAGE - 1)];
            by_push(dst, &ch, 1);
        }
        m->x[10] = n;
        return;
    }
    }
}

/* ------------------------------------------------------------ execute */
static inline u64 rdreg(mach_t *m, int r) { return r <= 0 ? 0 : m->x[r]; }
static inline void wrreg(mach_t *m, int r, u64 v) { if (r > 0) m->x[r] = v; }

static inline u64 mulhu64(u64 a, u64 b) { return (u64)(((unsigned __int128)a * b) >> 64); }
static inline s64 mulh64(s64 a, s64 b) { return (s64)(((__int128)a * b) >> 64); }
static inline s64 mulhsu64(s64 a, u64 b) { return (s64)(((__int128)a * (__int128)b) >> 64); }
static inline s64 div64(s64 a, s64 b) { if (b == 0) return -1; if (a == INT64_MIN && b == -1) return INT64_MIN; return a / b; }
static inline u64 divu64(u64 a, u64 b) { return b == 0 ? UINT64_MAX : a / b; }
static inline s64 rem64(s64 a, s64 b) { if (b == 0) return a; if (a == INT64_MIN && b == -1) return 0; return a % b; }
static inline u64 remu64(u64 a, u64 b) { return b == 0 ? a : a % b; }
static inline s32 div32(s32 a, s32 b) { if (b == 0) return -1; if (a == INT32_MIN && b == -1) return INT32_MIN; return a / b; }
static inline u32 divu32(u32 a, u32 b) { return b == 0 ? UINT32_MAX : a / b; }
static inline s32 rem32(s32 a, s32 b) { if (b == 0) return a; if (a == INT32_MIN && b == -1) return 0; return a % b; }
static inline u32 remu32(u32 a, u32 b) { return b == 0 ? a : a % b; }
static inline int clz64(u64 v) { return v ? __builtin_clzll(v) : 64; }
static inline int ctz64(u64 v) { return v ? __builtin_ctzll(v) : 64; }
static inline int clz32(u32 v) { return v ? __builtin_clz(v) : 32; }
static inline int ctz32(u32 v) { return v ? __builtin_ctz(v) : 32; }
static inline u64 sx32(u64 v) { return (u64)(s64)(s32)(u32)v; }

/* U-mode CSR accessibility (formats/standard.isa:325-447, regs/misc.hh:604-1241):
 * returns 1 if the access would reach the CSR data path (escape), 0 if it
 * raises IllegalInstFault. */
/* NaN-boxing, arch/riscv/regs/float.hh:72-94 (RISC-V default NaNs 0x7e00 /
 * 0x7fc00000, ext/softfloat/specialize.h) */
static inline u64 unbox32(u64 v) { return (v >> 32) == 0xFFFFFFFFULL ? (v & 0xFFFFFFFFULL) : 0x7FC00000ULL; }
static inline u64 unbox16(u64 v) { return (v >> 16) == 0xFFFFFFFFFFFFULL ? (v & 0xFFFF) : 0x7E00; }
static inline u64 box32(u64 v) { return 0xFFFFFFFF00000000ULL | (v & 0xFFFFFFFFULL); }
static inline u64 box16(u64 v) { return 0xFFFFFFFFFFFF0000ULL | (v & 0xFFFF); }
/* f16/f32/f64_classify, ext/softfloat/f32_classify.c (same shape for 16/64) */
static u64 fclassify(u64 ui, int ebits, int fbits) {
    u64 emax = (1ULL << ebits) - 1;
    u64 e = (ui >> fbits) & emax, fr = ui & ((1ULL << fbits) - 1);
    int sign = (int)((ui >> (ebits + fbits)) & 1);
    int inf_nan = e == emax, sub_zero = e == 0, frac_zero = fr == 0;
    int is_nan = inf_nan && !frac_zero, is_snan = is_nan && !((fr >> (fbits - 1)) & 1);
    return (u64)(sign && inf_nan && frac_zero) << 0 | (u64)(sign && !inf_nan && !sub_zero) << 1 |
           (u64)(sign && sub_zero && !frac_zero) << 2 | (u64)(sign && sub_zero && frac_zero) << 3 |
           (u64)(!sign && inf_nan && frac_zero) << 7 | (u64)(!sign && !inf_nan && !sub_zero) << 6 |
           (u64)(!sign && sub_zero && !frac_zero) << 5 | (u64)(!sign && sub_zero && frac_zero) << 4 |
           (u64)(is_nan && is_snan) << 8 | (u64)(is_nan && !is_snan) << 9;
}
/* AtomicMemOp RMW (decoder.isa:2067-2283 lambdas), w = 32-bit form */
static u64 amo_apply(int op, u64 mem, u64 src, int w) {
    if (w) { mem &= 0xFFFFFFFFULL; src &= 0xFFFFFFFFULL; }
    s64 sm = w ? (s64)(s32)(u32)mem : (s64)mem, ss = w ? (s64)(s32)(u32)src : (s64)src;
    switch (op) {
    case 0: return mem + src;                       /* add  */
    case 1: return src;                             /* swap */
    case 2: return mem ^ src;                       /* xor  */
    case 3: return mem | src;                       /* or   */
    case 4: return mem & src;                       /* and  */
    case 5: return ss < sm ? src : mem;             /* min  */
    case 6: return ss > sm ? src : mem;             /* max  */
    case 7: return src < mem ? src : mem;           /* minu */
    default: return src > mem ? src : mem;          /* maxu */
    }
}

static int csr_u_accessible(u32 csr) {
    if (bits(csr, 9, 8) != 0) return 0;     /* lowestAllowedMode > U */
    if (csr >= 0x001 && csr <= 0x003) return 1;
    if (csr >= 0x008 && csr <= 0x00A) return 1;
    if (csr == 0x00F || csr == 0x017) return 1;
    if (csr >= 0xC00 && csr <= 0xC1F) return 1;
    if (csr >= 0xC20 && csr <= 0xC22) return 1;
    return 0;                              /* absent from CSRData, or RV32-only *H */
}

/* LR: AtomicSimpleCPU::readMem with an LLSC request (atomic.cc:331-434): each
 * fragment that is read sets the ISA reservation to its address
 * (ISA::handleLockedRead, isa.cc:1006-1013) and makes it this context's lock
 * record (AbstractMemory::trackLoadLocked, abstract_mem.cc:258-283). */
static int lr_read(mach_t *m, u64 addr, unsigned size, u64 *val, u64 *fault_va) {
    u64 v = 0;
    unsigned done = 0;
    u64 a = addr;
    while (done < size) {
        unsigned frag = 64 - (unsigned)(a & 63);
        if (frag > size - done) frag = size - done;
        if (a + frag - 1 < a) { *fault_va = a; return F_PGFAULT; }
        uint8_t *pg = translate(m, a);
        if (!pg) { *fault_va = a; return F_PGFAULT; }
        for (unsigned i = 0; i < frag; i++) v |= (u64)pg[(a + i) & (PAGE - 1)] << (8 * (done + i));
        if (m->tkr) tk_frag(m, a, frag, OR_TCMD_LL);
        m->resv = a;
        m->lock = a & ~0xFULL;
        done += frag; a += frag;
    }
    *val = v;
    m->data_bytes += size;
    return F_NONE;
}
/* SC: AtomicSimpleCPU::writeMem with an LLSC request (atomic.cc:437-544).
 * Per fragment, after translation: the ISA check (ISA::handleLockedWrite,
 * isa.cc:1015-1060) fails when the reservation is empty or in another 64-byte
 * line, and clears it either way; a passing store reaches memory, which
 * performs it only if this context's lock record is the fragment's granule
 * (abstract_mem.cc:290-345) and then erases the record.  A second fragment
 * trips assert(curr_frag_id == 0) after its translation.  *ok = success. */
static int sc_write(mach_t *m, u64 addr, unsigned size, u64 val, int *ok, u64 *fault_va) {
    unsigned frag = 64 - (unsigned)(addr & 63);
    if (frag > size) frag = size;
    if (addr + frag - 1 < addr) { *fault_va = addr; return F_PGFAULT; }
    uint8_t *pg = translate_w(m, addr);
    if (!pg) { *fault_va = addr; return F_PGFAULT; }
    int pass = m->resv != OR_NONE && (m->resv & ~63ULL) == (addr & ~63ULL);
    m->resv = OR_NONE;
    *ok = 0;
    if (pass && m->lock == (addr & ~0xFULL)) {
        for (unsigned i = 0; i < frag; i++) pg[(addr + i) & (PAGE - 1)] = (uint8_t)(val >> (8 * i));
        m->lock = OR_NONE;
        *ok = 1;
    }
    if (frag < size) {
        u64 a2 = addr + frag;
        if (a2 + (size - frag) - 1 < a2 || !translate(m, a2)) { *fault_va = a2; return F_PGFAULT; }
        return F_SCLINE;
    }
    if (m->tkr) {   /* a failed SC: whether it reached memory is not in the golden record */
        if (*ok) tk_frag(m, addr, size, OR_TCMD_SC);
        else tk_unsupported(m, "the golden run has a failed SC");
    }
    if (*ok) m->data_bytes += size;
    return F_NONE;
}

/* Zfa fli: table entry i of format fmt (0 binary16, 1 binary32, 2 binary64).
 * The Zfa list: -1.0, the minimum positive normal, 2^-16, 2^-15, 2^-8, 2^-7,
 * 2^-4, 2^-3, 0.25 .. 0.4375, 0.5 .. 0.875, 1.0 .. 1.75 (steps of 1/4 of the
 * binade), 2.0, 2.5, 3, 4, 8, 16, 2^7, 2^8, 2^15, 2^16, +inf and the
 * canonical NaN; a value beyond the format's range rounds to +inf (binary16
 * 2^16) and one below its normal range is encoded subnormal. */
static u64 fli_bits(int fmt, u32 i) {
    const int mb = fmt == 0 ? 10 : fmt == 1 ? 23 : 52, eb = fmt == 0 ? 5 : fmt == 1 ? 8 : 11;
    const int bias = (1 << (eb - 1)) - 1, emax = (1 << eb) - 1;
    if (i == 30) return (u64)emax << mb;
    if (i == 31) return ((u64)emax << mb) | (1ULL << (mb - 1));
    if (i == 1) return 1ULL << mb;
    static const signed char e2[8] = {-16, -15, -8, -7, -4, -3};
    static const signed char big[8] = {0, 2, 3, 4, 7, 8, 15, 16};   /* i = 22..29: 3, then powers of two */
    u64 num = 1; int e = 0, neg = 0;
    if (i == 0) neg = 1;
    else if (i < 8) e = e2[i - 2];
    else if (i < 22) { num = 4 + (i - 8) % 4; e = (int)((i - 8) / 4) - 4; }
    else if (i == 22) num = 3;
    else e = big[i - 22];
    const int t = num >= 4 ? 2 : num >= 2 ? 1 : 0;
    const int be = e + t + bias;
    u64 r;
    if (be >= emax) r = (u64)emax << mb;
    else if (be <= 0) r = num << (e + bias - 1 + mb);
    else r = ((u64)be << mb) | ((num << (mb - t)) & ((1ULL << mb) - 1));
    return neg ? r | (1ULL << (eb + mb)) : r;
}
/* Zfa fcvtmod.w.d, decoder.isa:3320-3384 */
static u64 fcvtmod_w_d(u64 a, uint32_t *fl) {
    const int sign = (int)(a >> 63), ex = (int)((a >> 52) & 0x7FF);
    u64 frac = a & ((1ULL << 52) - 1);
    int inexact = 0, invalid = 0;
    if (ex == 0) { inexact = frac != 0; frac = 0; }
    else if (ex == 0x7FF) { invalid = 1; frac = 0; }
    else {
        const int true_exp = ex - 1023, shift = true_exp - 52;
        frac |= 1ULL << 52;
        if (shift >= 64) frac = 0;
        else if (shift >= 0) frac <<= shift;
        else if (shift > -64) { inexact = (frac << (64 + shift)) != 0; frac >>= -shift; }
        else { frac = 0; inexact = 1; }
        if (true_exp > 31 || frac > (sign ? 0x80000000ULL : 0x7fffffffULL)) { invalid = 1; inexact = 0; }
        if (sign) frac = -frac;
    }
    *fl = (inexact ? 1u : 0u) | (invalid ? 16u : 0u);
    return (u64)(s64)(int32_t)(u32)frac;
}

/* Execute one decoded instruction (the generated StaticInst::execute bodies of
 * decoder.isa).  Returns a fault kind; on F_NONE the caller commits npc. */
static int execute(mach_t *m, const dec_t *d, u64 *fault_va) {
    u64 pc = m->pc;
    u64 a = rdreg(m, d->rs1), b = rdreg(m, d->rs2);
    s64 imm = d->imm;
    u64 v = 0, t;
    int r;
    /* detected-by-replica: a protected flipped register read before being
     * overwritten (build-defined SHREWD semantics). */
    if (m->watch > 0 && (d->rs1 == m->watch || d->rs2 == m->watch)) return 100;
    if (m->watch > 0 && d->op == OP_ecall && (m->watch == 17 || (m->watch >= 10 && m->watch <= 15))) return 100;
    switch (d->op) {
    case OP_UNKNOWN: return F_UNKNOWN;
    case OP_ESC_FP: case OP_ESC_VEC: case OP_ESC_AMO: case OP_ESC_SYS: case OP_ESC_CRYPTO: case OP_ESC_CBO:
    case OP_ESC_CMP: case OP_ESC_M5: case OP_ESC_HYP:
        return F_ESCAPE;
    /* ---- compressed */
    case OP_c_addi4spn: if (imm == 0) return F_ILLEGAL; v = a + imm; break;
    case OP_c_lw: case OP_lw: case OP_c_lwsp:
        if (d->op == OP_c_lwsp && d->rd == 0) return F_ILLEGAL;
        r = mem_read(m, a + imm, 4, &t, fault_va); if (r) return r; v = sx32(t); break;
    case OP_c_ld: case OP_ld: case OP_c_ldsp:
        if (d->op == OP_c_ldsp && d->rd == 0) return F_ILLEGAL;
        r = mem_read(m, a + imm, 8, &t, fault_va); if (r) return r; v = t; break;
    case OP_c_lbu: case OP_lbu: r = mem_read(m, a + imm, 1, &t, fault_va); if (r) return r; v = t; break;
    case OP_c_lhu: case OP_lhu: r = mem_read(m, a + imm, 2, &t, fault_va); if (r) return r; v = t; break;
    case OP_c_lh: case OP_lh: r = mem_read(m, a + imm, 2, &t, fault_va); if (r) return r; v = (u64)sext(t, 16); break;
    case OP_lb: r = mem_read(m, a + imm, 1, &t, fault_va); if (r) return r; v = (u64)sext(t, 8); break;
    case OP_lwu: r = mem_read(m, a + imm, 4, &t, fault_va); if (r) return r; v = t; break;
    case OP_c_sb: case OP_sb: r = mem_write(m, a + imm, 1, b, fault_va); if (r) return r; goto no_rd;
    case OP_c_sh: case OP_sh: r = mem_write(m, a + imm, 2, b, fault_va); if (r) return r; goto no_rd;
    case OP_c_sw: case OP_sw: case OP_c_swsp: r = mem_write(m, a + imm, 4, b, fault_va); if (r) return r; goto no_rd;
    case OP_c_sd: case OP_sd: case OP_c_sdsp: r = mem_write(m, a + imm, 8, b, fault_va); if (r) return r; goto no_rd;
    case OP_c_addi: case OP_addi: v = a + imm; break;
    case OP_c_addiw: if (d->rd == 0) return F_ILLEGAL; v = sx32(a + imm); break;
    case OP_addiw: v = sx32(a + imm); break;
    case OP_c_li: v = imm; break;
    case OP_c_addi16sp: if (imm == 0) return F_ILLEGAL; v = a + imm; break;
    case OP_c_lui: if (imm == 0) return F_ILLEGAL; v = imm; break;
    case OP_c_srli: case OP_srli: v = a >> imm; break;
    case OP_c_srai: case OP_srai: v = (u64)((s64)a >> imm); break;
    case OP_c_andi: case OP_andi: v = a & (u64)imm; break;
    case OP_c_sub: case OP_sub: v = a - b; break;
    case OP_c_xor: case OP_xor_: v = a ^ b; break;
    case OP_c_or: case OP_or_: v = a | b; break;
    case OP_c_and: case OP_and_: v = a & b; break;
    case OP_c_subw: case OP_subw: v = sx32((u32)a - (u32)b); break;
    case OP_c_addw: case OP_addw: v = sx32((u32)a + (u32)b); break;
    case OP_c_mul: case OP_mul: v = a * b; break;
    case OP_c_zext_b: v = a & 0xFF; break;
    case OP_c_sext_b: case OP_sext_b: v = (u64)sext(a & 0xFF, 8); break;
    case OP_c_zext_h: v = a & 0xFFFF; break;
    case OP_c_sext_h: case OP_sext_h: v = (u64)sext(a & 0xFFFF, 16); break;
    case OP_c_zext_w: v = a & 0xFFFFFFFFULL; break;
    case OP_c_not: v = ~a; break;
    case OP_c_j: m->npc = pc + imm; goto no_rd;
    case OP_c_beqz: if (a == 0) m->npc = pc + imm; goto no_rd;
    case OP_c_bnez: if (a != 0) m->npc = pc + imm; goto no_rd;
    case OP_c_slli: case OP_slli: v = a << imm; break;
    case OP_c_jr: if (d->rs1 == 0) return F_ILLEGAL; m->npc = a & ~1ULL; goto no_rd;
    case OP_c_mv: v = b; break;
    case OP_c_ebreak: case OP_ebreak: return F_BREAK;
    case OP_c_jalr: v = m->npc; m->npc = a & ~1ULL; break;
    case OP_c_add: case OP_add: v = a + b; break;
    /* ---- 32-bit */
    case OP_fence: case OP_fence_i: goto no_rd;
    case OP_bseti: v = a | (1ULL << (imm & 63)); break;
    case OP_bclri: v = a & ~(1ULL << (imm & 63)); break;
    case OP_binvi: v = a ^ (1ULL << (imm & 63)); break;
    case OP_clz: v = clz64(a); break;
    case OP_ctz: v = ctz64(a); break;
    case OP_cpop: v = __builtin_popcountll(a); break;
    case OP_slti: v = (s64)a < imm ? 1 : 0; break;
    case OP_sltiu: v = a < (u64)imm ? 1 : 0; break;
    case OP_xori: v = a ^ (u64)imm; break;
    case OP_orc_b: v = 0; for (int i = 0; i < 8; i++) if ((a >> (8 * i)) & 0xFF) v |= 0xFFULL << (8 * i); break;
    case OP_bexti: v = (a >> (imm & 63)) & 1; break;
    case OP_rori: v = (a >> imm) | (a << ((64 - imm) & 63)); break;
    case OP_rev8: v = __builtin_bswap64(a); break;
    case OP_prefetch_i: case OP_prefetch_r: case OP_prefetch_w: goto no_rd;   /* faults suppressed (atomic.cc:604) */
    case OP_ori_hint: case OP_ori: v = a | (u64)imm; break;
    case OP_auipc: v = pc + imm; break;
    case OP_slliw: v = sx32((u32)a << imm); break;
    case OP_slli_uw: v = (a & 0xFFFFFFFFULL) << imm; break;
    case OP_clzw: v = clz32((u32)a); break;
    case OP_ctzw: v = ctz32((u32)a); break;
    case OP_cpopw: v = __builtin_popcount((u32)a); break;
    case OP_srliw: v = sx32((u32)a >> imm); break;
    case OP_sraiw: v = (u64)(s64)((s32)(u32)a >> imm); break;
    case OP_roriw: { u32 x = (u32)a; v = sx32((x >> imm) | (x << ((32 - imm) & 31))); break; }
    case OP_sll: v = a << (b & 63); break;
    case OP_mulh: v = (u64)mulh64((s64)a, (s64)b); break;
    case OP_clmul: v = 0; for (int i = 0; i < 64; i++) if ((b >> i) & 1) v ^= a << i; break;
    case OP_bset: v = a | (1ULL << (b & 63)); break;
    case OP_bclr: v = a & ~(1ULL << (b & 63)); break;
    case OP_rol: { int s = (int)(b & 63); v = (a << s) | (a >> ((64 - s) & 63)); break; }
    case OP_binv: v = a ^ (1ULL << (b & 63)); break;
    case OP_slt: v = (s64)a < (s64)b ? 1 : 0; break;
    case OP_mulhsu: v = (u64)mulhsu64((s64)a, b); break;
    case OP_clmulr: v = 0; for (int i = 0; i < 64; i++) if ((b >> i) & 1) v ^= a >> (64 - i - 1); break;
    case OP_sh1add: v = (a << 1) + b; break;
    case OP_sltu: v = a < b ? 1 : 0; break;
    case OP_mulhu: v = mulhu64(a, b); break;
    case OP_clmulh: v = 0; for (int i = 1; i < 64; i++) if ((b >> i) & 1) v ^= a >> (64 - i); break;
    case OP_div_: v = (u64)div64((s64)a, (s64)b); break;
    case OP_pack: v = (b << 32) | (a & 0xFFFFFFFFULL); break;
    case OP_min_: v = (s64)a < (s64)b ? a : b; break;
    case OP_sh2add: v = (a << 2) + b; break;
    case OP_xnor: v = ~(a ^ b); break;
    case OP_srl: v = a >> (b & 63); break;
    case OP_divu: v = divu64(a, b); break;
    case OP_czero_eqz: v = b == 0 ? 0 : a; break;
    case OP_sra: v = (u64)((s64)a >> (b & 63)); break;
    case OP_minu: v = a < b ? a : b; break;
    case OP_bext: v = (a >> (b & 63)) & 1; break;
    case OP_ror: { int s = (int)(b & 63); v = (a >> s) | (a << ((64 - s) & 63)); break; }
    case OP_rem: v = (u64)rem64((s64)a, (s64)b); break;
    case OP_max_: v = (s64)a > (s64)b ? a : b; break;
    case OP_sh3add: v = (a << 3) + b; break;
    case OP_orn: v = a | ~b; break;
    case OP_remu: v = remu64(a, b); break;
    case OP_packh: v = ((b & 0xFF) << 8) | (a & 0xFF); break;
    case OP_maxu: v = a > b ? a : b; break;
    case OP_czero_nez: v = b != 0 ? 0 : a; break;
    case OP_andn: v = a & ~b; break;
    case OP_lui: v = imm; break;
    case OP_mulw: v = sx32((u32)a * (u32)b); break;
    case OP_add_uw: v = (a & 0xFFFFFFFFULL) + b; break;
    case OP_sllw: v = sx32((u32)a << (b & 31)); break;
    case OP_rolw: { u32 x = (u32)a; int s = (int)(b & 31); v = sx32((x << s) | (x >> ((32 - s) & 31))); break; }
    case OP_sh1add_uw: v = ((a & 0xFFFFFFFFULL) << 1) + b; break;
    case OP_divw: v = (u64)(s64)div32((s32)a, (s32)b); break;
    case OP_packw: v = sx32(((b & 0xFFFF) << 16) | (a & 0xFFFF)); break;
    case OP_sh2add_uw: v = ((a & 0xFFFFFFFFULL) << 2) + b; break;
    case OP_srlw: v = sx32((u32)a >> (b & 31)); break;
    case OP_divuw: v = sx32(divu32((u32)a, (u32)b)); break;
    case OP_sraw: v = (u64)(s64)((s32)(u32)a >> (b & 31)); break;
    case OP_rorw: { u32 x = (u32)a; int s = (int)(b & 31); v = sx32((x >> s) | (x << ((32 - s) & 31))); break; }
    case OP_remw: v = (u64)(s64)rem32((s32)a, (s32)b); break;
    case OP_sh3add_uw: v = ((a & 0xFFFFFFFFULL) << 3) + b; break;
    case OP_remuw: v = sx32(remu32((u32)a, (u32)b)); break;
    case OP_beq: if (a == b) m->npc = pc + imm; goto no_rd;
    case OP_bne: if (a != b) m->npc = pc + imm; goto no_rd;
    case OP_blt: if ((s64)a < (s64)b) m->npc = pc + imm; goto no_rd;
    case OP_bge: if ((s64)a >= (s64)b) m->npc = pc + imm; goto no_rd;
    case OP_bltu: if (a < b) m->npc = pc + imm; goto no_rd;
    case OP_bgeu: if (a >= b) m->npc = pc + imm; goto no_rd;
    case OP_jalr: v = m->npc; m->npc = (a + imm) & ~1ULL; break;
    case OP_jal: v = m->npc; m->npc = pc + imm; break;
    case OP_ecall: return F_SYSCALL;
    case OP_csr:
        if (d->csr >= 1 && d->csr <= 3) {
            /* fflags / frm / fcsr (CSRExecute, formats/standard.isa:325-447; ISA::readCSR /
             * writeCSR, isa.cc:1141-1300): csrrw(i) reads only if rd != 0, csrrs/c(i) write
             * only if rs1 / uimm != 0; masks FFLAGS 0x1f, FRM 0x7 (regs/misc.hh) */
            const u32 f3 = d->funct3;
            const u64 src = f3 >= 5 ? (u64)d->imm : rdreg(m, d->rs1);
            const int rdc = (f3 == 1 || f3 == 5) ? d->rd != 0 : 1;
            const int wrc = (f3 == 1 || f3 == 5) ? 1 : (d->imm != 0);
            u64 data = 0;
            if (rdc) data = d->csr == 1 ? m->fflags : d->csr == 2 ? m->frm : (m->fflags | (m->frm << 5));
            v = data;
            const u64 nd = (f3 & 3) == 1 ? src : (f3 & 3) == 2 ? (data | src) : (data & ~src);
            if (wrc) {
                if (d->csr == 1) m->fflags = (u32)(nd & 0x1F);
                else if (d->csr == 2) m->frm = (u32)(nd & 7);
                else { m->fflags = (u32)(nd & 0x1F); m->frm = (u32)((nd >> 5) & 7); }
            }
            break;
        }
        return csr_u_accessible(d->csr) ? F_ESCAPE + 100 : F_ILLEGAL;
    /* ---- F/D/Zfh loads and stores (Load/Store formats, formats/mem.isa:123-207):
     * the access first, then the FPU-status update (never off in SE: fs is
     * INITIAL from ISA::resetThread, isa.cc:390); loads NaN-box (float.hh:104-107) */
    case OP_flh: case OP_flw: case OP_fld: case OP_c_fld: case OP_c_fldsp: {
        unsigned sz = d->op == OP_flh ? 2 : d->op == OP_flw ? 4 : 8;
        r = mem_read(m, a + imm, sz, &t, fault_va); if (r) return r;
        m->f[d->frd] = sz == 2 ? box16(t) : sz == 4 ? box32(t) : t;
        goto no_rd;
    }
    case OP_fsh: case OP_fsw: case OP_fsd: case OP_c_fsd: case OP_c_fsdsp: {
        unsigned sz = d->op == OP_fsh ? 2 : d->op == OP_fsw ? 4 : 8;
        r = mem_write(m, a + imm, sz, m->f[d->frs2], fault_va); if (r) return r;
        goto no_rd;
    }
    /* ---- moves, sign injection, classify (no rounding, no exception flags) */
    case OP_fmv_x_w: v = sx32(m->f[d->frs1]); break;
    case OP_fmv_x_d: v = m->f[d->frs1]; break;
    case OP_fmv_x_h: v = (u64)sext(m->f[d->frs1] & 0xFFFF, 16); break;
    case OP_fmv_w_x: m->f[d->frd] = box32(a); goto no_rd;
    case OP_fmv_d_x: m->f[d->frd] = a; goto no_rd;
    case OP_fmv_h_x: m->f[d->frd] = box16(a); goto no_rd;
    case OP_fsgnj_s: case OP_fsgnjn_s: case OP_fsgnjx_s: {
        u64 x = unbox32(m->f[d->frs1]), y = unbox32(m->f[d->frs2]);
        u64 sg = d->op == OP_fsgnj_s ? y : d->op == OP_fsgnjn_s ? ~y : (x ^ y);
        m->f[d->frd] = box32((x & 0x7FFFFFFFULL) | (sg & 0x80000000ULL));
        goto no_rd;
    }
    case OP_fsgnj_d: case OP_fsgnjn_d: case OP_fsgnjx_d: {
        u64 x = m->f[d->frs1], y = m->f[d->frs2];
        u64 sg = d->op == OP_fsgnj_d ? y : d->op == OP_fsgnjn_d ? ~y : (x ^ y);
        m->f[d->frd] = (x & 0x7FFFFFFFFFFFFFFFULL) | (sg & 0x8000000000000000ULL);
        goto no_rd;
    }
    case OP_fsgnj_h: case OP_fsgnjn_h: case OP_fsgnjx_h: {
        u64 x = unbox16(m->f[d->frs1]), y = unbox16(m->f[d->frs2]);
        u64 sg = d->op == OP_fsgnj_h ? y : d->op == OP_fsgnjn_h ? ~y : (x ^ y);
        m->f[d->frd] = box16((x & 0x7FFF) | (sg & 0x8000));
        goto no_rd;
    }
    case OP_fclass_s: v = fclassify(unbox32(m->f[d->frs1]), 8, 23); break;
    case OP_fclass_d: v = fclassify(m->f[d->frs1], 11, 52); break;
    case OP_fclass_h: v = fclassify(unbox16(m->f[d->frs1]), 5, 10); break;
#ifdef OR_SOFTFLOAT
    /* ---- F/D/Zfh arithmetic through the reference SoftFloat: FloatExecute
     * (formats/fp.isa:34-56) ORs the raised flags into FFLAGS; RM_REQUIRED
     * (fp_inst.hh:37-44) takes frm for the dynamic mode and faults on 5-7 */
    case OP_fadd: case OP_fsub: case OP_fmul: case OP_fdiv: case OP_fsqrt: case OP_fmadd: case OP_fmsub:
    case OP_fnmsub: case OP_fnmadd: case OP_fmin: case OP_fmax: case OP_feq: case OP_flt: case OP_fle:
    case OP_fcvt_f2i: case OP_fcvt_i2f: case OP_fcvt_f2f: {
        const int fmt = (int)((imm >> 3) & 3), sub = (int)((imm >> 5) & 7);
        const u64 sgn = fmt == 0 ? 0x8000ULL : fmt == 1 ? 0x80000000ULL : 0x8000000000000000ULL;
        const u64 qnan = fmt == 0 ? 0x7E00ULL : fmt == 1 ? 0x7FC00000ULL : 0x7FF8000000000000ULL;
        const int rounds = !(d->op == OP_fmin || d->op == OP_fmax || d->op == OP_feq || d->op == OP_flt ||
                             d->op == OP_fle);
        if (d->op == OP_fsqrt && d->frs2 != 0) return F_ILLEGAL;   /* "source reg x1" */
        int rm = (int)(imm & 7);
        if (rounds) {
            if (rm == 7) rm = (int)m->frm;
            if (rm > 4) return F_ILLEGAL;                           /* "RM fault" */
        }
#define UNBOX(f_, x_) ((f_) == 0 ? unbox16(x_) : (f_) == 1 ? unbox32(x_) : (x_))
#define BOX(f_, x_) ((f_) == 0 ? box16(x_) : (f_) == 1 ? box32(x_) : (x_))
        uint32_t fl = 0, fl2 = 0;
        const u64 x = d->frs1 >= 0 ? UNBOX(d->op == OP_fcvt_f2f ? sub : fmt, m->f[d->frs1]) : 0;
        const u64 y = d->frs2 >= 0 ? UNBOX(fmt, m->f[d->frs2]) : 0;
        const u64 z = UNBOX(fmt, m->f[(imm >> 8) & 31]);
        int to_f = 1;
        u64 r = 0;
        switch (d->op) {
        case OP_fadd: r = sf_ref(0, fmt, rm, x, y, 0, &fl); break;
        case OP_fsub: r = sf_ref(1, fmt, rm, x, y, 0, &fl); break;
        case OP_fmul: r = sf_ref(2, fmt, rm, x, y, 0, &fl); break;
        case OP_fdiv: r = sf_ref(3, fmt, rm, x, y, 0, &fl); break;
        case OP_fsqrt: r = sf_ref(4, fmt, rm, x, 0, 0, &fl); break;
        case OP_fmadd: r = sf_ref(5, fmt, rm, x, y, z, &fl); break;                 /* decoder.isa:2694-2719 */
        case OP_fmsub: r = sf_ref(5, fmt, rm, x, y, z ^ sgn, &fl); break;
        case OP_fnmsub: r = sf_ref(5, fmt, rm, x ^ sgn, y, z, &fl); break;
        case OP_fnmadd: r = sf_ref(5, fmt, rm, x ^ sgn, y, z ^ sgn, &fl); break;
        case OP_fmin: case OP_fmax: {   /* decoder.isa:2944-3120: lt_quiet, then eq */
            const int mx = d->op == OP_fmax;
            const u64 p = mx ? y : x, q = mx ? x : y;   /* fmax compares (fs2, fs1) */
            int pick = (int)sf_ref(9, fmt, rm, p, q, 0, &fl);
            if (!pick) pick = (int)sf_ref(6, fmt, rm, p, q, 0, &fl2) && (p & sgn);
            fl |= fl2;
            const u64 inf = fmt == 0 ? 0x7C00ULL : fmt == 1 ? 0x7F800000ULL : 0x7FF0000000000000ULL;
            const int nx = (x & ~sgn) > inf, ny = (y & ~sgn) > inf;
            if (sub) {   /* fminm / fmaxm: a non-NaN result is written unboxed (Fd_bits = fs.v) */
                if (!(nx || ny)) { m->fflags |= (fl | fl2) & 0x1F; m->f[d->frd] = pick ? x : y; goto no_rd; }
                r = qnan;
            } else {
                r = (nx && ny) ? qnan : ((pick || ny) ? x : y);
            }
            break;
        }
        case OP_feq: v = sf_ref(6, fmt, rm, x, y, 0, &fl); to_f = 0; break;
        case OP_flt: v = sf_ref(sub ? 9 : 7, fmt, rm, x, y, 0, &fl); to_f = 0; break;
        case OP_fle: v = sf_ref(sub ? 10 : 8, fmt, rm, x, y, 0, &fl); to_f = 0; break;
        case OP_fcvt_f2i:   /* decoder.isa:3273-3420: w/wu results sign-extended from 32 bits */
            v = sf_ref(11 + sub, fmt, rm, x, 0, 0, &fl);
            if (sub <= 1) v = sx32(v);
            to_f = 0;
            break;
        case OP_fcvt_i2f: r = sf_ref(15 + sub, fmt, rm, a, 0, 0, &fl); break;
        default: r = sf_ref(19 + fmt, sub, rm, x, 0, 0, &fl); break;   /* fcvt between formats */
        }
        m->fflags |= fl & 0x1F;
        if (to_f) { m->f[d->frd] = BOX(fmt, r); goto no_rd; }
#undef UNBOX
#undef BOX
        break;
    }
#endif
    /* ---- AMOs: AtomicSimpleCPU::amoMem (atomic.cc:546-608) panics on an
     * access that crosses a 64-byte line before translating; no alignment
     * check in SE (tlb.cc:573-604).  Rd = the old value (sign-extended .w). */
    case OP_amoadd_w: case OP_amoswap_w: case OP_amoxor_w: case OP_amoor_w: case OP_amoand_w:
    case OP_amomin_w: case OP_amomax_w: case OP_amominu_w: case OP_amomaxu_w:
    case OP_amoadd_d: case OP_amoswap_d: case OP_amoxor_d: case OP_amoor_d: case OP_amoand_d:
    case OP_amomin_d: case OP_amomax_d: case OP_amominu_d: case OP_amomaxu_d: {
        int w = d->op <= OP_amomaxu_w;
        unsigned sz = w ? 4 : 8;
        u64 ea = a;
        if (((ea + sz - 1) & ~63ULL) > ea) return F_AMOLINE;
        if (ea + sz - 1 < ea) { *fault_va = ea; return F_PGFAULT; }
        uint8_t *pg = translate_w(m, ea);
        if (!pg) { *fault_va = ea; return F_PGFAULT; }
        u64 old = 0;
        for (unsigned i = 0; i < sz; i++) old |= (u64)pg[(ea + i) & (PAGE - 1)] << (8 * i);
        u64 nw = amo_apply(d->op - (w ? OP_amoadd_w : OP_amoadd_d), old, b, w);
        for (unsigned i = 0; i < sz; i++) pg[(ea + i) & (PAGE - 1)] = (uint8_t)(nw >> (8 * i));
        if (m->tkr) tk_frag(m, ea, sz, OR_TCMD_SWAP);
        m->data_bytes += 2 * sz;
        m->num_cycles += (d->funct3 & 1) + (d->funct3 >> 1);   /* rl / aq fence micro-ops: one tick each */
        v = w ? sx32(old) : old;
        break;
    }
    /* ---- LR / SC (formats/amo.isa LoadReserved / StoreCond; rl/aq fence
     * micro-ops are one tick each, like the AMOs) */
    case OP_lr_w: case OP_lr_d: {
        unsigned sz = d->op == OP_lr_w ? 4 : 8;
        r = lr_read(m, a, sz, &t, fault_va); if (r) return r;
        m->num_cycles += (d->funct3 & 1) + (d->funct3 >> 1);
        v = sz == 4 ? sx32(t) : t;
        break;
    }
    case OP_sc_w: case OP_sc_d: {
        unsigned sz = d->op == OP_sc_w ? 4 : 8;
        int ok = 0;
        r = sc_write(m, a, sz, b, &ok, fault_va); if (r) return r;
        m->num_cycles += (d->funct3 & 1) + (d->funct3 >> 1);
        v = ok ? 0 : 1;   /* result = !success (amo.isa StoreCondExecute) */
        break;
    }
    /* ---- Zfa.  fli: the value the 5-bit rs1 field selects from the table the
     * Zfa specification lists (decoder.isa:3550-3700; pinned by
     * tests/golden/fli_rv64.json); no rounding mode, no flags. */
    case OP_fli: {
        const int fmt = (int)((imm >> 3) & 3);
        const u64 x = fli_bits(fmt, (u32)(imm >> 8) & 31);
        m->f[d->frd] = fmt == 0 ? box16(x) : fmt == 1 ? box32(x) : x;
        goto no_rd;
    }
    /* fcvtmod.w.d: RM_REQUIRED (fp_inst.hh:34-41), then the modular
     * truncation of decoder.isa:3320-3384 (flags through FFLAGS_EXE) */
    case OP_fcvtmod: {
        int rm = (int)(imm & 7);
        if (rm == 7) rm = (int)m->frm;
        if (rm > 4) return F_ILLEGAL;
        uint32_t fl = 0;
        v = fcvtmod_w_d(m->f[d->frs1], &fl);
        m->fflags |= fl;
        break;
    }
#ifdef OR_SOFTFLOAT
    /* fround / froundnx: RM_REQUIRED, then f*_roundToInt(fs1, rm, exact) of
     * the reference SoftFloat (decoder.isa:3105-3170) */
    case OP_fround: {
        const int fmt = (int)((imm >> 3) & 3);
        int rm = (int)(imm & 7);
        if (rm == 7) rm = (int)m->frm;
        if (rm > 4) return F_ILLEGAL;
        uint32_t fl = 0;
        const u64 x = fmt == 0 ? unbox16(m->f[d->frs1]) : fmt == 1 ? unbox32(m->f[d->frs1]) : m->f[d->frs1];
        const u64 r2 = sf_ref(22 + (int)((imm >> 5) & 1), fmt, rm, x, 0, 0, &fl);
        m->fflags |= fl & 0x1F;
        m->f[d->frd] = fmt == 0 ? box16(r2) : fmt == 1 ? box32(r2) : r2;
        goto no_rd;
    }
#else
    case OP_fround: return F_ESCAPE;
#endif
    /* ---- RVV before any vset* (decode: op vec) */
    case OP_vec:
        if (m->vcfg) return F_ESCAPE;   /* decoded under another vtype / vl: the vector unit's state */
        switch ((int)imm) {
        case VEC_NOP: goto no_rd;
        case VEC_NOP2: m->num_cycles += 1; goto no_rd;   /* the trailing micro-op's tick */
        case VEC_ILLEGAL: return F_ILLEGAL;
        case VEC_UNDEF: return F_UNDEF;
        default: return F_ESCAPE;
        }
    /* ---- vset*: VConfOp::execute (formats/vector_conf.isa:115-186; the
     * operands at decoder.isa:5838-5886).  getNewVtype: a request other than
     * the current vtype is checked -- getSew asserts vsew <= 3
     * (insts/vector.hh:52-56: gem5.opt aborts); LMUL outside [1/8, 8] (vlmul
     * 4: 1/16), SEW > min(LMUL, 1) x ELEN (ELEN 64, RiscvISA.py:103) or
     * reserved bits 62..8 set give vtype = vill.  VLMAX = VLEN / SEW x LMUL
     * (getVlmax, insts/vector.cc:69-76; VLEN 256, RiscvISA.py:98), 0 under
     * vill.  getNewVL takes the requested vl as uint32_t and picks by the
     * rd / rs1 register indices (vsetivli: rs1 "-1").  rd gets vl; the new
     * configuration is the decoder's from the next instruction on
     * (decoder.cc:155-163). */
    case OP_vset: {
        const int form = (int)((imm >> 16) & 3);
        const u64 req = form == 1 ? b : (u64)(imm & 0xFFFF);
        const u64 old = vcfg_vtype(m->vcfg);
        u64 nt = old;
        if (req != old) {
            const u32 vsew = (u32)(req >> 3) & 7, vlmul = (u32)req & 7;
            if (vsew > 3) return F_VSEW;
            const u32 lim = vlmul <= 3 ? 64 : vlmul == 5 ? 8 : vlmul == 6 ? 16 : vlmul == 7 ? 32 : 0;
            const int illegal = vlmul == 4 || (8u << vsew) > lim || ((req >> 8) & ((1ULL << 55) - 1)) != 0;
            nt = illegal ? VILL : req;
        }
        u32 vlmax = 0;
        if (!(nt >> 63)) {
            const u32 vsew = (u32)(nt >> 3) & 7, vlmul = (u32)nt & 7, per = 32u >> vsew;
            vlmax = vlmul <= 3 ? per << vlmul : per >> (8 - vlmul);
        }
        const u32 rs1_bits = form == 2 ? 1u : (u32)d->rs1, req_vl = form == 2 ? (u32)(imm >> 20) : (u32)a;
        const u32 cur = vcfg_vl(m->vcfg);
        u32 nvl = 0;
        if (vlmax == 0) nvl = 0;
        else if (d->rd == 0 && rs1_bits == 0) nvl = cur > vlmax ? vlmax : cur;
        else if (d->rd != 0 && rs1_bits == 0) nvl = vlmax;
        else nvl = req_vl > vlmax ? vlmax : req_vl;
        m->vcfg = vcfg_of(nt, nvl);
        v = nvl;
        break;
    }
    /* ---- privileged SYSTEM / hypervisor load-store from PRV_U (refine_misc) */
    case OP_priv:
        if (!imm) return F_ILLEGAL;
        goto no_rd;
    /* ---- cache-block operations: one 64-byte request at the line of Rs1 */
    case OP_cbo: {
        const u64 ea = a & ~63ULL;
        if (imm == 4) { r = mem_write_zero64(m, ea, fault_va); if (r) return r; goto no_rd; }
        if (!translate(m, ea)) { *fault_va = ea; return F_PGFAULT; }
        goto no_rd;
    }
    /* ---- M5Op (formats/m5ops.isa:39-57): pseudoInstWork (sim/pseudo_inst.hh)
     * with RegABI64 arguments a0.. (reg_abi.cc:37-40); the generated execute()
     * then writes a0 = rvSext(result) and a1 = 0 (its RV32 branch's second
     * destination, zero-initialised: exec-ns.cc.inc M5Op::execute).  Under the
     * default System / BaseCPU params of an SE run (System.py:120-149,
     * BaseCPU.py:124-129; one thread context, no dist-gem5). */
    case OP_m5op: {
        u64 res = 0;
        switch (imm) {
        case 0x07:   /* rpns: curTick() / ns */
            if (m->tkr) tk_unsupported(m, "the golden run reads curTick (rpns)");
            if (m->tki) return F_TKCLOCK;
            res = (m->c->tick0 + (m->num_cycles - 1) * m->c->clk_period) / 1000;
            break;
        case 0x23:   /* m5sum(a0..a5) */
            if (m->watch >= 10 && m->watch <= 15) return 100;
            for (int k = 10; k <= 15; k++) res += m->x[k];
            break;
        case 0x30: {   /* initParam: the key is the 16 bytes of a0, a1 as a C string */
            if (m->watch == 10 || m->watch == 11) return 100;
            char key[17];
            for (int k = 0; k < 8; k++) { key[k] = (char)(m->x[10] >> (8 * k)); key[8 + k] = (char)(m->x[11] >> (8 * k)); }
            key[16] = 0;
            if (!key[0]) res = 0;                              /* DEFAULT "": System.init_param = 0 */
            else if (!strcmp(key, "dist-rank")) res = 0;       /* DistIface::rankParam, no primary */
            else if (!strcmp(key, "dist-size")) res = 1;       /* DistIface::sizeParam, no primary */
            else return F_M5PANIC;                             /* "Unknown key for initparam" */
            break;
        }
        case 0x51: return F_BREAK;      /* debugbreak: debug::breakpoint() -> SIGTRAP (base/debug.cc:64-70) */
        case 0x54: return F_M5PANIC;    /* M5OP_PANIC */
        /* quiesce: ThreadContext::quiesce suspends the only context
         * (thread_context.cc:167, system.cc:145-151; AtomicSimpleCPU::
         * suspendContext deschedules its tick, atomic.cc:246-269) after this
         * instruction commits, and nothing wakes it: the simulation runs to
         * its tick limit ("simulate() limit reached") -- a hang */
        case 0x01: m->m5x = 3; break;
        /* m5_exit(delay) / m5_fail(delay, code): exitSimLoop at curTick +
         * delay ns (pseudo_inst.cc:178-204); the stdlib run script's default
         * handler for both ends the simulation (simulate/exit_handler.py:551-
         * 557).  delay 0: the exit event fires after this instruction's tick
         * (Sim_Exit_Pri after CPU_Tick_Pri, sim/eventq.hh:207,237); a delayed
         * exit lets more ticks run first -- not modelled (escape) */
        case 0x21: case 0x22:
            if (m->watch == 10 || (imm == 0x22 && m->watch == 11)) return 100;
            if (m->x[10] != 0) return F_ESCAPE;
            m->m5x = imm == 0x21 ? 1 : 2;
            m->m5code = imm == 0x22 ? (int)(m->x[11] & 0xff) : 0;
            break;
        /* m5_checkpoint: the stdlib default saves a checkpoint and continues;
         * switchcpu: switch_generator does nothing for a processor that is not
         * switchable (BaseCPUProcessor) and continues (exit_event_generators.
         * py:72-83, 100-114): no architectural effect, result 0 */
        case 0x43: case 0x52: break;
        /* simulator control or host files: quiesce for a time, writefile,
         * addsymbol, workbegin / workend, togglesync, workload event, hypercall */
        case 0x02: case 0x03: case 0x04: case 0x4f:
        case 0x53: case 0x5a: case 0x5b: case 0x62: case 0x70: case 0x71:
            return F_ESCAPE;
        /* arm (Workload stats), wakeCPU (the only context is active), loadsymbol
         * (symbolfile ""), reset/dump stats (a later stats event only),
         * readfile (readfile ""), reserved and unhandled functions: result 0 */
        default: break;
        }
        wrreg(m, 10, res);
        wrreg(m, 11, 0);
        m->wrote = 1;
        if (m->watch == 10 || m->watch == 11) m->watch = -1;
        return F_NONE;
    }
#ifdef OR_RVK
    /* ---- Zkn / Zks through the reference's own helpers (rvk_ref.cc) */
    case OP_crypto: v = or_rvk_ref((int)imm, a, b); break;
#else
    case OP_crypto: return F_ESCAPE;
#endif
    default: return F_UNKNOWN;
    }
    wrreg(m, d->rd, v);
    m->wrote = d->rd > 0;
    if (m->watch > 0 && d->rd == m->watch) m->watch = -1;   /* overwritten before read */
    return F_NONE;
no_rd:
    return F_NONE;
}

/* --------------------------------------------------------- inject / tick */
static void inject(mach_t *m) {
    const or_site_t *s = m->site;
    m->injected = 1;
    if (s->target >= 1 && s->target <= 31) {
        m->x[s->target] ^= s->mask;
        if ((m->protect_mask >> s->target) & 1) m->watch = (int)s->target;
    } else if (s->target == OR_T_PC) {
        m->pc ^= s->mask;
        if ((m->protect_mask >> 32) & 1) { finish(m, OR_DETECTED, 0, 0); }
    } else if (s->target == OR_T_RESULT) {
        m->rarm = 1;   /* the next instruction that commits is the target */
        m->rmask = s->mask;
    } else if (s->target == OR_T_MEM) {
        /* flip the 8-byte word if its page is mapped at inject time */
        uint8_t *pg = translate_w(m, s->addr);
        if (pg) {
            u64 off = s->addr & (PAGE - 1);
            for (int i = 0; i < 8; i++) pg[off + i] ^= (uint8_t)(s->mask >> (8 * i));
        } else {
            m->injected = 2;
        }
    }
}

/* RiscvFault::invoke / invokeSE dispositions, arch/riscv/faults.cc:286-333 and
 * sim/faults.cc:95-105. */
static void invoke_fault(mach_t *m, int f, u64 fault_va, const dec_t *d) {
    switch (f) {
    case F_SYSCALL:
        /* SyscallFault::invokeSE advances the PC first (faults.cc:325-333) */
        m->pc = m->pc + d->len;
        do_syscall(m);
        return;
    case F_BREAK: finish(m, OR_CRASH, OR_CRASH_SIGTRAP, 133); return;
    case F_TKCLOCK: finish(m, OR_ESCAPE, OR_ESC_TIMING, OR_TK_CLOCK); return;
    case F_ILLEGAL: finish(m, OR_CRASH, OR_CRASH_ILLEGAL_INST, 134); return;
    case F_UNKNOWN: finish(m, OR_CRASH, OR_CRASH_UNKNOWN_INST, 134); return;
    case F_ESCAPE: finish(m, OR_ESCAPE, OR_ESC_INST, 0); m->res.detail = d->raw; return;
    case F_ESCAPE + 100: finish(m, OR_ESCAPE, OR_ESC_CSR, 0); m->res.detail = d->raw; return;
    case F_AMOLINE: finish(m, OR_CRASH, OR_CRASH_AMO_LINE, 134); return;
    case F_SCLINE: finish(m, OR_CRASH, OR_CRASH_SC_LINE, 134); return;
    case F_M5PANIC: finish(m, OR_CRASH, OR_CRASH_M5_PANIC, 134); return;
    case F_VSEW: finish(m, OR_CRASH, OR_CRASH_VSET_SEW, 134); return;
    case F_UNDEF: finish(m, OR_ESCAPE, OR_ESC_UNDEF, 0); m->res.detail = d->raw; return;
    case 100: finish(m, OR_DETECTED, 0, 0); return;
    case F_PGFAULT: {
        int h = fixup_fault(m, fault_va);
        if (h == 1) return;   /* retried next tick */
        if (h == -1) { finish(m, OR_CRASH, OR_CRASH_STACK_LIMIT, 1); return; }
        finish(m, OR_CRASH, OR_CRASH_PAGE_FAULT, 134);
        m->res.detail = (u32)fault_va;
        return;
    }
    }
}

/* gem5 OpClass of an executed op (tests/golden/opclass_rv64.json, generated
 * from the reference's ISA description) */
static int op_class(int op) {
    switch (op) {
#define OPC(n, c) case OP_##n: return c;
    FI_GEM5_OPCLASS(OPC)
#undef OPC
    default: return 0;
    }
}

/* ------------------------------------------------ SHREWD FU contention */
/* The O3 issue stage replayed over the golden run (include/fi_engine.h,
 * "SHREWD functional-unit contention": what is restated from the reference
 * and what is a model).  Written from the reference, independently of
 * shrewd_amd/csrc/fi_issue.cpp: a plain cycle loop over arrays. */
enum { OC_NONE = 0, OC_INTALU = 1, OC_INTMULT = 2, OC_INTDIV = 3, OC_FADD = 4, OC_FCMP = 5, OC_FCVT = 6,
       OC_FMULT = 7, OC_FMULTACC = 8, OC_FDIV = 9, OC_FMISC = 10, OC_FSQRT = 11, OC_MEMREAD = 52,
       OC_MEMWRITE = 53, OC_FMEMREAD = 54, OC_FMEMWRITE = 55, OC_IPR = 56, OC_N = 77 };
/* fu_pool.hh:148-167 */
enum { FU_NOSHADOW = -7, FU_NONEED = -3, FU_NOCAPABLE = -2, FU_NOFREE = -1 };

typedef struct {
    int nunits;
    u64 busy_until[64];           /* unitBusy: busy while busy_until > now */
    int cap_n[OC_N], cap_units[OC_N][16], cap_rr[OC_N];   /* fuPerCapList: FUIdxQueue */
    int capable[OC_N], lat[OC_N], piped[OC_N];           /* capabilityList, maxOpLatencies, pipelined */
} fupool_t;

/* FUPool::FUPool over DefaultFUPool (o3/FUPool.py:52-66) with the counts of
 * FuncUnitConfig.py (IntALU 6, IntMultDiv 2, FP_ALU 4, FP_MultDiv 2,
 * RdWrPort 4, IprPort 1; SIMD/matrix/predicate units serve no scalar class). */
static void fupool_init(fupool_t *P, const or_issue_params_t *p) {
    static const struct { int desc, cls, lat, piped; } opdesc[] = {
        {0, OC_INTALU, 1, 1},                                                    /* IntALU      :45-47 */
        {1, OC_INTMULT, 3, 1}, {1, OC_INTDIV, 20, 0},                            /* IntMultDiv  :50-56 */
        {2, OC_FADD, 2, 1}, {2, OC_FCMP, 2, 1}, {2, OC_FCVT, 2, 1},              /* FP_ALU      :59-65 */
        {3, OC_FMULT, 4, 1}, {3, OC_FMULTACC, 5, 1}, {3, OC_FMISC, 3, 1},
        {3, OC_FDIV, 12, 0}, {3, OC_FSQRT, 24, 0},                               /* FP_MultDiv  :68-76 */
        {4, OC_MEMREAD, 1, 1}, {4, OC_MEMWRITE, 1, 1}, {4, OC_FMEMREAD, 1, 1}, {4, OC_FMEMWRITE, 1, 1},  /* RdWrPort */
        {5, OC_IPR, 3, 0},                                                       /* IprPort     :196-198 */
    };
    memset(P, 0, sizeof *P);
    for (int k = 0; k < OC_N; k++) P->piped[k] = 1;
    for (int d = 0; d < 6; d++) {
        int n = (int)p->fu_count[d];
        if (n <= 0) continue;
        if (n > 8) n = 8;
        for (unsigned j = 0; j < sizeof opdesc / sizeof opdesc[0]; j++) {
            if (opdesc[j].desc != d) continue;
            int c = opdesc[j].cls;
            P->capable[c] = 1;
            for (int k = 0; k < n; k++) P->cap_units[c][P->cap_n[c]++] = P->nunits + k;
            if (opdesc[j].lat > P->lat[c]) P->lat[c] = opdesc[j].lat;
            if (!opdesc[j].piped) P->piped[c] = 0;
        }
        P->nunits += n;
    }
}

/* FUPool::findFreeUnit (fu_pool.cc:155-173) */
static int fu_find(fupool_t *P, int cls, u64 now) {
    if (!P->cap_n[cls]) return FU_NOFREE;
    int *rr = &P->cap_rr[cls];
#define GETFU() (u = P->cap_units[cls][*rr], *rr = (*rr + 1 == P->cap_n[cls]) ? 0 : *rr + 1)
    int u, start;
    GETFU();
    start = u;
    while (P->busy_until[u] > now) {
        GETFU();
        if (u == start) return FU_NOFREE;
    }
#undef GETFU
    return u;
}

/* FUPool::getUnit(capability, is_shadow, approx_capability) (fu_pool.cc:175-301) */
static int fu_get(fupool_t *P, int cap, int is_shadow, int *approx, u64 now) {
    if (!P->capable[cap]) return FU_NOCAPABLE;
    int fu = FU_NOFREE, aux = FU_NOFREE, aux2 = FU_NOFREE;
    *approx = cap;
    if (is_shadow) {
        switch (cap) {
        case OC_INTALU:
            fu = fu_find(P, cap, now); aux = fu_find(P, OC_FADD, now); aux2 = fu_find(P, OC_FCMP, now);
            if (fu == FU_NOFREE) {
                fu = aux; *approx = OC_FADD;
                if (aux == FU_NOFREE) { *approx = OC_FCMP; fu = aux2; }
            }
            break;
        case OC_INTMULT:
            fu = fu_find(P, cap, now); aux = fu_find(P, OC_FMULT, now);
            if (fu == FU_NOFREE) { *approx = OC_FMULT; fu = aux; }
            break;
        case OC_INTDIV:
            fu = fu_find(P, cap, now); aux = fu_find(P, OC_FDIV, now);
            if (fu == FU_NOFREE) { *approx = OC_FDIV; fu = aux; }
            break;
        case OC_FADD: case OC_FMULT: case OC_FDIV: case OC_FSQRT:
            fu = fu_find(P, cap, now); aux = fu_find(P, OC_INTALU, now);
            if (fu == FU_NOFREE) { *approx = OC_INTALU; fu = aux; }
            break;
        case OC_FMULTACC: case OC_FCVT: case OC_FCMP: case OC_FMISC:
            fu = fu_find(P, cap, now);
            break;
        default:
            fu = FU_NOSHADOW;
            break;
        }
    } else {
        fu = fu_find(P, cap, now);
    }
    if (fu == FU_NOSHADOW) return FU_NOSHADOW;
    if (fu == FU_NOFREE) return FU_NOFREE;
    P->busy_until[fu] = ~0ULL;
    return fu;
}

/* InstructionQueue::requestShadow (inst_queue.cc:1082-1181) */
static void request_shadow(fupool_t *P, int idx, int *idx_shadow, int op_class, int *shadow_class, int *has_shadow,
                           u64 *op_latency, u64 now, or_issue_stats_t *st) {
    if (idx != FU_NOFREE && idx != FU_NOCAPABLE) {
        *idx_shadow = fu_get(P, op_class, 1, shadow_class, now);
        if (*idx_shadow != FU_NOSHADOW && idx != FU_NOCAPABLE) {
            if (*idx_shadow != FU_NOFREE) {
                *has_shadow = 1;
                st->shadow_available++;
                if ((u64)P->lat[*shadow_class] > *op_latency) *op_latency = (u64)P->lat[*shadow_class];
                if (op_class == *shadow_class) st->shadow_same_fu++; else st->shadow_not_same_fu++;
            } else {
                st->shadow_not_available++;
            }
            if (op_class >= OC_INTALU && op_class <= OC_FSQRT) {
                if (*has_shadow) st->class_available[op_class]++; else st->class_not_available[op_class]++;
            }
        }
    }
}

int or_issue_model(const or_issue_op_t *ops, uint64_t n, const or_issue_params_t *p, uint8_t *shadow,
                   or_issue_stats_t *stats) {
    if (!p || !p->issue_width || !p->dispatch_width || !p->commit_width || !p->iq_entries || !p->rob_entries ||
        !p->load_latency)
        return -1;
    or_issue_stats_t st; memset(&st, 0, sizeof st);
    st.ops = n;
    fupool_t *P = (fupool_t *)calloc(1, sizeof *P);
    fupool_init(P, p);
    u64 *done = (u64 *)malloc((n + 1) * sizeof(u64));   /* value ready; ~0 = not issued */
    u64 *dcyc = (u64 *)malloc((n + 1) * sizeof(u64));   /* dispatch cycle */
    int32_t (*prod)[8] = (int32_t (*)[8])malloc((n + 1) * sizeof *prod);   /* latest older writer of each source */
    int *in_iq = (int *)calloc(n + 1, sizeof(int));
    for (u64 i = 0; i < n; i++) done[i] = ~0ULL;
    s64 writer[33];
    for (int r = 0; r < 33; r++) writer[r] = -1;
    u64 committed = 0, dispatched = 0, iq_count = 0, cyc = 0, serial_open = 0;
    u64 *grp = (u64 *)malloc((p->issue_width + 1) * sizeof(u64));
    int *grp_idx = (int *)malloc((p->issue_width + 1) * sizeof(int));
    u64 *grp_lat = (u64 *)malloc((p->issue_width + 1) * sizeof(u64));
    while (committed < n) {
        /* memory ops leave the IQ once done */
        for (u64 i = committed; i < dispatched; i++)
            if (in_iq[i] && done[i] <= cyc) { in_iq[i] = 0; iq_count--; }
        /* in-order commit of up to commitWidth completed ops */
        for (u32 k = 0; k < p->commit_width; k++) {
            if (committed >= dispatched || done[committed] > cyc) break;
            if (ops[committed].kind == OR_ISSUE_SERIAL) serial_open--;
            committed++;
        }
        if (committed == n) break;
        /* scheduleReadyInsts: oldest ready first; a class that finds no free
         * unit is passed over for the rest of the cycle */
        int skip[OC_N]; memset(skip, 0, sizeof skip);
        u32 issued = 0, ng = 0;
        for (u64 i = committed; i < dispatched && issued < p->issue_width; i++) {
            if (!in_iq[i] || done[i] != ~0ULL || dcyc[i] >= cyc) continue;
            int oc = ops[i].opclass;
            if (skip[oc]) continue;
            int ok = 1;
            if (ops[i].kind == OR_ISSUE_SERIAL && committed != i) ok = 0;
            for (int r = 0; ok && r < 8; r++)
                if (prod[i][r] >= 0 && done[prod[i][r]] > cyc) ok = 0;
            if (!ok) continue;
            int idx = FU_NONEED, approx = oc;
            u64 op_latency = 1;
            if (oc != OC_NONE) {
                idx = fu_get(P, oc, 0, &approx, cyc);
                if (idx > FU_NOFREE) op_latency = (u64)P->lat[oc];
            }
            int idx_shadow = FU_NONEED, has_shadow = 0, shadow_oc = oc;
            if (p->priority_to_shadow)
                request_shadow(P, idx, &idx_shadow, oc, &shadow_oc, &has_shadow, &op_latency, cyc, &st);
            if (idx > FU_NOFREE || idx == FU_NONEED || idx == FU_NOCAPABLE) {
                if (op_latency == 1) {
                    if (idx >= 0) {
                        P->busy_until[idx] = cyc + 1;                  /* freeUnitNextCycle */
                        if (has_shadow) P->busy_until[idx_shadow] = cyc + 1;
                    }
                } else {
                    P->busy_until[idx] = P->piped[oc] ? cyc + 1 : cyc + op_latency;   /* FUCompletion setFreeFU */
                    if (has_shadow) P->busy_until[idx_shadow] = P->piped[shadow_oc] ? cyc + 1 : cyc + op_latency;
                }
                if (!p->priority_to_shadow) { grp[ng] = i; grp_idx[ng] = idx; grp_lat[ng] = op_latency; ng++; }
                shadow[i] = (uint8_t)has_shadow;
                done[i] = cyc + (ops[i].kind == OR_ISSUE_LOAD ? (u64)p->load_latency : op_latency);
                if (ops[i].kind != OR_ISSUE_LOAD && ops[i].kind != OR_ISSUE_STORE) { in_iq[i] = 0; iq_count--; }
                issued++;
            } else {
                skip[oc] = 1;
            }
        }
        /* !priorityToShadow: shadows for the issued group, in issue order */
        for (u32 g = 0; g < ng; g++) {
            u64 i = grp[g];
            int idx_shadow = FU_NONEED, has_shadow = 0, oc = ops[i].opclass, shadow_oc = oc;
            u64 lat = grp_lat[g];
            request_shadow(P, grp_idx[g], &idx_shadow, oc, &shadow_oc, &has_shadow, &lat, cyc, &st);
            shadow[i] = (uint8_t)has_shadow;
            if (has_shadow) {
                if (lat == 1) { if (idx_shadow >= 0) P->busy_until[idx_shadow] = cyc + 1; }
                else P->busy_until[idx_shadow] = P->piped[shadow_oc] ? cyc + 1 : cyc + lat;
            }
        }
        /* dispatch in program order into IQ + ROB; nothing passes an
         * uncommitted serialising op */
        for (u32 k = 0; k < p->dispatch_width && dispatched < n; k++) {
            if (iq_count >= p->iq_entries || dispatched - committed >= p->rob_entries) break;
            if (serial_open) break;
            u64 i = dispatched++;
            dcyc[i] = cyc;
            int np = 0;
            for (int r = 0; r < 8; r++) prod[i][r] = -1;
            for (int r = 1; r < 33 && np < 8; r++)
                if (((ops[i].src >> r) & 1) && writer[r] >= 0) prod[i][np++] = (int32_t)writer[r];
            if (ops[i].kind == OR_ISSUE_SERIAL) serial_open++;
            for (int r = 1; r < 33; r++) if ((ops[i].dst >> r) & 1) writer[r] = (s64)i;
            in_iq[i] = 1; iq_count++;
        }
        cyc++;
    }
    st.cycles = cyc;
    if (stats) *stats = st;
    free(P); free(done); free(dcyc); free(prod); free(in_iq); free(grp); free(grp_idx); free(grp_lat);
    return 0;
}

/* One trace event of the golden run as a replayed op (restates
 * shrewd_amd/csrc/fi_issue.cpp:issue_ops_from_trace's rule from the oracle's
 * own decode): integer operands x1..x31; ecall reads a0..a7, writes a0 and
 * serialises; FP ops chain through one FP-state register (bit 32). */
static or_issue_op_t issue_op(const dec_t *d, int is_ecall) {
    or_issue_op_t o; memset(&o, 0, sizeof o);
    int oc = op_class(d->op);
    o.opclass = (uint8_t)oc;
    if (is_ecall) { o.src = 0x3FC00ULL; o.dst = 1ULL << 10; o.kind = OR_ISSUE_SERIAL; return o; }
    if (d->rs1 > 0) o.src |= 1ULL << d->rs1;
    if (d->rs2 > 0) o.src |= 1ULL << d->rs2;
    if (d->rd > 0) o.dst |= 1ULL << d->rd;
    if (oc >= OC_FADD && oc <= OC_FSQRT) { o.src |= 1ULL << 32; o.dst |= 1ULL << 32; }
    if (oc == OC_FMEMREAD) o.dst |= 1ULL << 32;
    if (oc == OC_FMEMWRITE) o.src |= 1ULL << 32;
    o.kind = (oc == OC_MEMREAD || oc == OC_FMEMREAD) ? OR_ISSUE_LOAD
           : (oc == OC_MEMWRITE || oc == OC_FMEMWRITE) ? OR_ISSUE_STORE : OR_ISSUE_PLAIN;
    return o;
}

/* SHREWD shadow execution: FUPool::getUnit(cap, is_shadow=true) (cpu/o3/
 * fu_pool.cc:177-301) finds a shadow unit only for IntAlu, IntMult, IntDiv and
 * the scalar Float classes (FloatAdd..FloatSqrt, enum 1..11); every other
 * class returns NoShadowFU.  Without the issue model the shadow is always
 * available; with it (or_set_issue_model), only if the k-th committed golden
 * instruction's shadow found a unit (the target of a result fault at numInst
 * k is that golden instruction: the trial equals the golden run until then). */
static int replicated(const or_campaign_t *c, int cls, u64 k) {
    if (!(cls >= FI_OPC_INTALU && cls <= FI_OPC_FLOATSQRT && ((c->protect_opc >> cls) & 1))) return 0;
    return !c->shadow || k >= c->n_shadow || c->shadow[k];
}

/* Result fault (OR_T_RESULT): applied to the first instruction that commits
 * at or after the inject time.  A replicated instruction's shadow disagrees
 * with the faulty result: detected at its commit (pc = the instruction).
 * Otherwise the value written to x[rd] is flipped; an instruction that writes
 * no integer register leaves nothing to flip.  Returns 1 if the trial ended. */
static int result_fault(mach_t *m, const dec_t *d) {
    m->rarm = 0;
    if (!m->wrote) { m->injected = 2; return 0; }
    if (replicated(m->c, op_class(d->op), m->num_inst - 1)) { finish(m, OR_DETECTED, 0, 0); return 1; }
    m->x[d->rd] ^= m->rmask;
    return 0;
}

/* One AtomicSimpleCPU::tick() with width=1 (cpu/simple/atomic.cc:611-739). */
static void tk_open(mach_t *m, u64 tick_index);
static void tk_close(mach_t *m, int f, const dec_t *d);
static void tk_inject_top(mach_t *m);
static void tk_inject_data(mach_t *m, const dec_t *d);
static int tk_here(const mach_t *m, u64 tick_index, int data);

static void tick(mach_t *m, u64 cap) {
    const u64 tick_index = m->num_cycles;
    m->num_cycles++;
    if (m->tkr) tk_open(m, tick_index);
    if (m->tki && !m->injected && tk_here(m, tick_index, 0)) {
        tk_inject_top(m);
        if (m->done) return;
    }
    /* serviceInstCountEvents (base.cc:321-325): fault injection and the
     * max-insts exit both fire at the top of the first tick with numInst >= n */
    if (m->site && !m->injected && m->num_inst >= m->site->inst) {
        inject(m);
        if (m->done) return;
    }
    /* (a hang's record names no pc: the engine proves some hangs before the
       cap, shrewd_amd/csrc/fi_translate.cpp counted-loop proofs) */
    if (m->num_inst >= cap) { finish(m, OR_HANG, OR_HANG_INSTS, 0); m->res.detail = 0; return; }
    /* setupFetchRequest: 4 bytes at (pc & ~3) + fetchOffset (base.cc:304-318) */
    u64 fetch_pc = (m->pc & ~3ULL) + m->fetch_offset;
    if (m->fo) { fetch_pc = m->fo_addr; m->fo = 0; }   /* a request sent before the pc flip */
    uint8_t *pg = translate(m, fetch_pc);
    if (pg && m->tkr) tk_fetch(m, fetch_pc);
    int f = F_NONE; u64 fva = 0;
    dec_t d; memset(&d, 0, sizeof d);
    int have_inst = 0;
    if (!pg) {
        f = F_PGFAULT; fva = fetch_pc;
    } else {
        const uint8_t *w = pg + (fetch_pc & (PAGE - 1));
        u32 word = (u32)w[0] | ((u32)w[1] << 8) | ((u32)w[2] << 16) | ((u32)w[3] << 24);
        m->fetch_bytes += 4;
        /* Decoder::moreBytes (decoder.cc:63-116) */
        int aligned = (m->pc % 4) == 0;
        if (aligned) {
            m->emi = word;
            if ((word & 3) != 3) m->emi = word & 0xFFFF;
            m->inst_done = 1;
        } else if (m->mid) {
            m->emi = (m->emi & 0xFFFF) | ((word & 0xFFFF) << 16);
            m->mid = 0; m->inst_done = 1;
        } else {
            m->emi = word >> 16;
            m->mid = (m->emi & 3) == 3;
            m->inst_done = !m->mid;
        }
        /* preExecute / Decoder::decode (base.cc:328-409, decoder.cc:135-173) */
        if (m->inst_done) {
            m->inst_done = 0;
            decode(m->emi, &d);
            m->npc = m->pc + d.len;
            m->stay_at_pc = 0;
            have_inst = 1;
        } else {
            m->stay_at_pc = 1;
            m->fetch_offset += 4;
        }
        if (have_inst) {
            m->wrote = 0;
            m->tk_cpu = 1;
            f = execute(m, &d, &fva);
            m->tk_cpu = 0;
            if (m->tki && !m->injected && f == F_NONE && tk_here(m, tick_index, 1)) tk_inject_data(m, &d);
            if (m->rec && (f == F_NONE || f == F_SYSCALL)) {
                if (m->rec_n == m->rec_cap) {
                    m->rec_cap = m->rec_cap ? 2 * m->rec_cap : 4096;
                    m->rec = (or_issue_op_t *)realloc(m->rec, m->rec_cap * sizeof *m->rec);
                }
                m->rec[m->rec_n++] = issue_op(&d, f == F_SYSCALL);
            }
            if (f == F_NONE) {
                m->num_inst++;   /* countInst only on NoFault (atomic.cc:687-689) */
                if (m->dbg_pc && m->dbg_pc_n < m->dbg_pc_cap) m->dbg_pc[m->dbg_pc_n] = m->dbg_raw ? (m->pc & 0xFFFFFFFFULL) | ((u64)d.raw << 32) : m->pc;
                if (m->dbg_pc) m->dbg_pc_n++;
                if (m->rarm && result_fault(m, &d)) return;
            }
        }
    }
    /* advancePC (base.cc:493-512) */
    if (f != F_NONE || !m->stay_at_pc) {
        m->fetch_offset = 0;
        if (f != F_NONE) {
            m->mid = 0; m->inst_done = 0; m->emi = 0;   /* decoder->reset() */
            invoke_fault(m, f, fva, &d);
        } else {
            m->pc = m->npc;
        }
    }
    if (m->m5x && !m->done) {   /* the M5 op that ends the run has committed */
        if (m->tkr) tk_close(m, F_NONE + 100, &d);
        if (m->m5x == 3) {
            finish(m, OR_HANG, OR_HANG_QUIESCE, 0);
        } else {
            const or_campaign_t *c = m->c;
            int same = c->have_golden && m->m5code == (int)c->golden.exit_code &&
                       c->gsub == (m->m5x == 1 ? OR_END_M5_EXIT : OR_END_M5_FAIL) &&
                       m->out.len == c->gout.len && m->err.len == c->gerr.len &&
                       (m->out.len == 0 || !memcmp(m->out.buf, c->gout.buf, m->out.len)) &&
                       (m->err.len == 0 || !memcmp(m->err.buf, c->gerr.buf, m->err.len));
            finish(m, same ? OR_MASKED : OR_SDC, m->m5x == 1 ? OR_END_M5_EXIT : OR_END_M5_FAIL, m->m5code);
        }
    }
    if (m->tkr && (f != F_NONE || !m->stay_at_pc)) tk_close(m, f, &d);
}

/* --------------------------------------------------------- ELF + image */
static int rd16(const uint8_t *p) { return p[0] | (p[1] << 8); }
static u32 rd32(const uint8_t *p) { return (u32)p[0] | ((u32)p[1] << 8) | ((u32)p[2] << 16) | ((u32)p[3] << 24); }
static u64 rd64(const uint8_t *p) { return (u64)rd32(p) | ((u64)rd32(p + 4) << 32); }

static void image_write(or_campaign_t *c, u64 addr, const uint8_t *src, u64 n) {
    /* Process::initState -> image.write through an allocating proxy (process.cc:289-306) */
    for (u64 i = 0; i < n; i++) {
        u64 a = addr + i;
        pte_t *p = pm_find(&c->image, a >> 12);
        if (!p) {
            p = pm_insert(&c->image, a >> 12, (uint8_t *)calloc(1, PAGE), 1);
            /* SETranslatingPortProxy::fixupRange (Always): allocateMem per page
             * in write order, each the next free frame (mem_pool.cc:96-102) */
            if (c->n_alloc == c->cap_alloc) {
                c->cap_alloc = c->cap_alloc ? 2 * c->cap_alloc : 64;
                c->alloc_vpn = (u64 *)realloc(c->alloc_vpn, c->cap_alloc * sizeof(u64));
            }
            c->alloc_vpn[c->n_alloc++] = a >> 12;
        }
        p->data[a & (PAGE - 1)] = src ? src[i] : 0;
    }
}

/* gem5 Random: std::mt19937_64 seeded with the global seed 5489
 * (base/random.hh:211-217, random.cc:79); random(0,0xFF) = gen() % 256. */
typedef struct { u64 mt[312]; int idx; } mt64_t;
static void mt_seed(mt64_t *s, u64 seed) {
    s->mt[0] = seed;
    for (int i = 1; i < 312; i++) s->mt[i] = 6364136223846793005ULL * (s->mt[i - 1] ^ (s->mt[i - 1] >> 62)) + (u64)i;
    s->idx = 312;
}
static u64 mt_next(mt64_t *s) {
    if (s->idx >= 312) {
        for (int i = 0; i < 312; i++) {
            u64 x = (s->mt[i] & 0xFFFFFFFF80000000ULL) | (s->mt[(i + 1) % 312] & 0x7FFFFFFFULL);
            u64 xa = x >> 1;
            if (x & 1) xa ^= 0xB5026F5AA96619E9ULL;
            s->mt[i] = s->mt[(i + 156) % 312] ^ xa;
        }
        s->idx = 0;
    }
    u64 y = s->mt[s->idx++];
    y ^= (y >> 29) & 0x5555555555555555ULL;
    y ^= (y << 17) & 0x71D67FFFEDA60000ULL;
    y ^= (y << 37) & 0xFFF7EEE000000000ULL;
    y ^= y >> 43;
    return y;
}

static void push64(or_campaign_t *c, u64 *sp, u64 v) {
    uint8_t b[8];
    for (int i = 0; i < 8; i++) b[i] = (uint8_t)(v >> (8 * i));
    image_write(c, *sp, b, 8);
    *sp += 8;
}

or_campaign_t *or_create(const uint8_t *elf, size_t len, const char *argv0) {
    or_campaign_t *c = (or_campaign_t *)calloc(1, sizeof(*c));
    pm_init(&c->image, 64);
    if (len < 64 || memcmp(elf, "\x7f" "ELF", 4) || elf[4] != 2 || elf[5] != 1 || rd16(elf + 18) != 243) {
        snprintf(c->err, sizeof c->err, "not an ELF64 LE RISC-V file"); return c;
    }
    c->entry = rd64(elf + 24);
    u64 phoff = rd64(elf + 32);
    int phentsize = rd16(elf + 54), phnum = rd16(elf + 56);
    u64 max_addr = 0, phdr_vaddr = 0;
    u64 wpages[4096]; u64 nw = 0;
    for (int i = 0; i < phnum; i++) {
        const uint8_t *ph = elf + phoff + (u64)i * phentsize;
        if (rd32(ph) != 1) continue;                   /* PT_LOAD */
        u32 flags = rd32(ph + 4);
        u64 off = rd64(ph + 8), vaddr = rd64(ph + 16), paddr = rd64(ph + 24);
        u64 filesz = rd64(ph + 32), memsz = rd64(ph + 40);
        if (memsz == 0) continue;                      /* elf_object.cc:378-381 */
        /* segments are loaded at p_paddr, bss zero-filled (elf_object.cc:383-392) */
        image_write(c, paddr, elf + off, filesz);
        if (memsz > filesz) image_write(c, paddr + filesz, NULL, memsz - filesz);
        if (paddr + memsz > max_addr) max_addr = paddr + memsz;
        if (off <= phoff && off + filesz > phoff) phdr_vaddr = vaddr + (phoff - off);   /* :396-402 */
        if (flags & 2)
            for (u64 pg = paddr & PAGE_MASK; pg < paddr + memsz && nw < 4096; pg += PAGE) wpages[nw++] = pg;
        if (c->nseg < 32) {
            c->seg[c->nseg].lo = paddr & PAGE_MASK;
            c->seg[c->nseg].hi = (paddr + memsz + PAGE - 1) & PAGE_MASK;
            c->seg[c->nseg].w = (flags & 2) != 0;
            c->nseg++;
        }
        if (flags & 1) {
            u64 lo = paddr & PAGE_MASK, hi = (paddr + memsz + PAGE - 1) & PAGE_MASK;
            if (!c->text_hi || lo < c->text_lo) c->text_lo = lo;
            if (hi > c->text_hi) c->text_hi = hi;
        }
    }
    /* RiscvProcess64 ctor: brk = roundUp(image.maxAddr(), 4096) (process.cc:76) */
    c->brk0 = (max_addr + PAGE - 1) & PAGE_MASK;
    c->clk_period = 500;
    c->rnd_seed = 5489;

    /* RiscvProcess::argsInit<uint64_t> (process.cc:134-261), argv = {argv0}, envp = {} */
    const size_t alen = strlen(argv0);
    u64 stack_min = STACK_BASE;
    u64 stack_top = stack_min - 16 - (alen + 1);
    stack_top &= ~7ULL;
    const u64 at_random = stack_top;   /* auxv Random is taken here (process.cc:150-159) */
    const int nauxv = 8;
    stack_top -= (1 + 1) * 8 + (1 + 0) * 8 + 8 + 2 * 8 * nauxv;
    stack_top &= ~15ULL;
    u64 stack_size = STACK_BASE - stack_top;
    c->stack_vma_lo = stack_top & PAGE_MASK;
    c->stack_vma_hi = c->stack_vma_lo + ((stack_size + PAGE - 1) & PAGE_MASK);
    c->vma0[0].lo = c->stack_vma_lo; c->vma0[0].hi = c->stack_vma_hi; c->nvma0 = 1;
    c->mmap_end0 = 0x4000000000000000ULL;   /* RiscvProcess64 (process.cc:79) */
    /* AT_RANDOM */
    stack_min -= 16;
    mt64_t mt; mt_seed(&mt, 5489);
    uint8_t rnd[16];
    for (int i = 0; i < 16; i++) rnd[i] = (uint8_t)(mt_next(&mt) % 256);
    image_write(c, stack_min, rnd, 16);
    /* argv string */
    stack_min -= alen + 1;
    image_write(c, stack_min, (const uint8_t *)argv0, alen + 1);
    u64 argp = stack_min;
    stack_min &= ~7ULL;
    stack_min -= (1 + 1) * 8 + (1 + 0) * 8 + 8 + 2 * 8 * nauxv;
    stack_min &= ~15ULL;
    u64 sp = stack_min;
    push64(c, &sp, 1);            /* argc */
    push64(c, &sp, argp); push64(c, &sp, 0);
    push64(c, &sp, 0);            /* envp terminator */
    const u64 aux[8][2] = {{9, c->entry}, {5, (u64)phnum}, {4, (u64)phentsize}, {3, phdr_vaddr},
                           {6, PAGE}, {23, 0}, {25, at_random}, {0, 0}};
    for (int i = 0; i < nauxv; i++) { push64(c, &sp, aux[i][0]); push64(c, &sp, aux[i][1]); }
    c->sp0 = stack_min;
    c->stack_min0 = stack_min & PAGE_MASK;
    /* writable pages at start: ELF writable segments + initial stack pages */
    for (u64 pg = c->stack_min0; pg != 0 && pg <= (STACK_BASE & PAGE_MASK); pg += PAGE) {
        if (nw < 4096) wpages[nw++] = pg;
        if (pg == (STACK_BASE & PAGE_MASK)) break;
    }
    /* sorted, unique */
    for (u64 i = 1; i < nw; i++)
        for (u64 j = i; j > 0 && wpages[j - 1] > wpages[j]; j--) { u64 t = wpages[j]; wpages[j] = wpages[j - 1]; wpages[j - 1] = t; }
    u64 u = 0;
    for (u64 i = 0; i < nw; i++) if (u == 0 || wpages[u - 1] != wpages[i]) wpages[u++] = wpages[i];
    nw = u;
    c->n_mem_pages = nw;
    c->mem_pages = (u64 *)malloc(sizeof(u64) * (nw ? nw : 1));
    memcpy(c->mem_pages, wpages, sizeof(u64) * nw);
    memset(c->regs0, 0, sizeof c->regs0);
    c->regs0[2] = c->sp0;   /* argsInit: every register 0 but sp, pc = e_entry */
    c->pc0 = c->entry;
    return c;
}

static void tkgold_free(struct tkgold *g);
void or_destroy(or_campaign_t *c) {
    if (!c) return;
    pm_free(&c->image);
    tkgold_free(c->tk);
    free(c->alloc_vpn);
    free(c->mem_pages); free(c->gout.buf); free(c->gerr.buf); free(c->shadow); free(c->in_data);
    free(c);
}

static void mach_init(mach_t *m, const or_campaign_t *c) {
    memset(m, 0, sizeof(*m));
    m->c = c;
    pm_init(&m->mem, 64);
    for (u64 i = 0; i < c->image.cap; i++)
        if (c->image.tab[i].vpn != UINT64_MAX) pm_insert(&m->mem, c->image.tab[i].vpn, c->image.tab[i].data, 0);
    memcpy(m->x, c->regs0, sizeof m->x);
    m->x[0] = 0;
    m->pc = c->pc0;
    m->stack_min = c->stack_min0;
    m->watch = -1;
    m->resv = m->lock = OR_NONE;
    memcpy(m->f, c->f0, sizeof m->f);
    m->fflags = c->fflags0; m->frm = c->frm0;
    memcpy(m->vma, c->vma0, sizeof m->vma);   /* process start: argsInit's "stack" VMA */
    m->nvma = c->nvma0;
    m->brk = c->brk0;
    m->mmap_end = c->mmap_end0;
}
static void mach_free(mach_t *m) { pm_free(&m->mem); free(m->out.buf); free(m->err.buf); free(m->mt); }

static void run(mach_t *m, u64 cap) {
    while (!m->done) tick(m, cap);
}

int or_golden(or_campaign_t *c, u64 max_inst, or_golden_t *out) {
    if (c->err[0]) return -1;
    mach_t m; mach_init(&m, c);
    run(&m, max_inst);
    if (m.res.cls != OR_MASKED && m.res.cls != OR_SDC) {
        snprintf(c->err, sizeof c->err, "golden run did not exit (cls %d sub %d pc %#lx)", m.res.cls, m.res.sub,
                 (unsigned long)m.pc);
        mach_free(&m); return -1;
    }
    c->golden.ninst = m.num_inst; c->golden.ncycles = m.num_cycles;
    c->golden.exit_code = m.res.exit_code; c->golden.cls = 0;
    c->gsub = m.res.sub;   /* how it ended: exit, m5_exit or m5_fail */
    c->golden.stdout_len = m.out.len; c->golden.stderr_len = m.err.len;
    c->golden.fetch_bytes = m.fetch_bytes; c->golden.data_bytes = m.data_bytes;
    free(c->gout.buf); free(c->gerr.buf);
    c->gout = m.out; c->gerr = m.err; m.out.buf = m.err.buf = NULL;
    c->have_golden = 1;
    mach_free(&m);
    if (out) *out = c->golden;
    return 0;
}

uint64_t or_golden_ops(or_campaign_t *c, or_issue_op_t *out, uint64_t cap) {
    if (!c->have_golden) return 0;
    mach_t m; mach_init(&m, c);
    m.rec_cap = 4096;
    m.rec = (or_issue_op_t *)malloc(m.rec_cap * sizeof *m.rec);
    run(&m, c->golden.ninst + 1);
    const u64 n = m.rec_n;
    if (out) memcpy(out, m.rec, (cap < n ? cap : n) * sizeof *out);
    free(m.rec); m.rec = NULL;
    mach_free(&m);
    return n;
}

int or_set_issue_model(or_campaign_t *c, const or_issue_params_t *p) {
    if (!p) { free(c->shadow); c->shadow = NULL; c->n_shadow = 0; return 0; }
    if (!c->have_golden) { snprintf(c->err, sizeof c->err, "or_set_issue_model: no golden run"); return -1; }
    mach_t m; mach_init(&m, c);
    m.rec_cap = 4096;
    m.rec = (or_issue_op_t *)malloc(m.rec_cap * sizeof *m.rec);
    run(&m, c->golden.ninst + 1);
    uint8_t *all = (uint8_t *)calloc(m.rec_n + 1, 1);
    or_issue_stats_t st;
    int rc = or_issue_model(m.rec, m.rec_n, p, all, &st);
    if (rc == 0) {
        free(c->shadow);
        c->shadow = (uint8_t *)calloc(c->golden.ninst + 1, 1);
        u64 k = 0;
        for (u64 i = 0; i < m.rec_n; i++)
            if (m.rec[i].kind != OR_ISSUE_SERIAL && k < c->golden.ninst) c->shadow[k++] = all[i];
        c->n_shadow = k;
        c->issue_stats = st;
        if (k != c->golden.ninst) { snprintf(c->err, sizeof c->err, "issue model: trace length"); rc = -1; }
    } else {
        snprintf(c->err, sizeof c->err, "issue model: invalid parameters");
    }
    free(all); free(m.rec); m.rec = NULL;
    mach_free(&m);
    return rc;
}

uint64_t or_shadow_map(or_campaign_t *c, uint8_t *buf, uint64_t cap, or_issue_stats_t *stats) {
    if (!c->shadow) return 0;
    if (buf && cap) memcpy(buf, c->shadow, cap < c->n_shadow ? cap : c->n_shadow);
    if (stats) *stats = c->issue_stats;
    return c->n_shadow;
}

uint64_t or_golden_stdout(or_campaign_t *c, uint8_t *buf, uint64_t cap) {
    u64 n = c->gout.len < cap ? c->gout.len : cap;
    if (n) memcpy(buf, c->gout.buf, n);
    return c->gout.len;
}

uint64_t or_golden_stderr(or_campaign_t *c, uint8_t *buf, uint64_t cap) {
    u64 n = c->gerr.len < cap ? c->gerr.len : cap;
    if (n) memcpy(buf, c->gerr.buf, n);
    return c->gerr.len;
}

/* ------------------------------------------------------------- sampler */
/* SplitMix64 (Steele et al. 2014); site = f(seed, trial) only, so it is
 * shard-invariant.  Same definition as shrewd_amd/csrc/hip/sampler. */
static u64 splitmix(u64 *s) {
    u64 z = (*s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static u64 mulhi(u64 a, u64 b) { return (u64)(((unsigned __int128)a * b) >> 64); }

int or_sample(or_campaign_t *c, u64 seed, u64 first, u64 n, u64 structures, u32 burst, u64 bits,
              or_site_t *sites) {
    if (!c->have_golden) { snprintf(c->err, sizeof c->err, "golden run required before sampling"); return -1; }
    if (burst < 1 || burst > 64) burst = 1;
    structures &= ~1ULL;                        /* x0 is not a fault site */
    if (c->n_mem_pages == 0) structures &= ~(1ULL << OR_T_MEM);
    int nt = __builtin_popcountll(structures);
    if (nt == 0) { snprintf(c->err, sizeof c->err, "no fault structures"); return -1; }
    for (u64 i = 0; i < n; i++) {
        u64 id = first + i;
        u64 st = seed ^ (id * 0xD6E8FEB86659FD93ULL);
        u64 r0 = splitmix(&st), r1 = splitmix(&st), r2 = splitmix(&st), r3 = splitmix(&st);
        or_site_t *s = &sites[i];
        s->inst = mulhi(r0, c->golden.ninst);
        u64 k = mulhi(r1, (u64)nt);
        u64 m = structures;
        for (u64 j = 0; j < k; j++) m &= m - 1;
        s->target = (u32)__builtin_ctzll(m);
        /* bits: eligible lowest-bit positions (fi_set_bits); all of them = the plain draw */
        const u64 valid = burst == 1 ? ~0ULL : ((2ULL << (64 - burst)) - 1);
        u64 b;
        if ((bits & valid) == valid) {
            b = mulhi(r2, 65 - burst);
        } else {
            u64 mm = bits & valid;
            const u64 kk = mulhi(r2, (u64)__builtin_popcountll(mm));
            for (u64 j = 0; j < kk; j++) mm &= mm - 1;
            b = (u64)__builtin_ctzll(mm);
        }
        s->mask = (burst == 64 ? ~0ULL : ((1ULL << burst) - 1)) << b;
        s->addr = 0;
        if (s->target == OR_T_MEM) {
            u64 w = mulhi(r3, c->n_mem_pages * 512);
            s->addr = c->mem_pages[w / 512] + (w % 512) * 8;
        }
        s->trial = (u32)id;
    }
    return 0;
}

/* ------------------------------------------------------------- trials */
static u64 hang_cap(const or_campaign_t *c, u64 f16) {
    if (f16 == 0) f16 = 32;   /* default cap: 2x golden instructions */
    return (c->golden.ninst * f16) / 16 + 1000;
}

static void run_trial(const or_campaign_t *c, const or_site_t *s, u64 protect, u64 cap, or_outcome_t *o,
                      bytes_t *cap_out) {
    mach_t m; mach_init(&m, c);
    m.site = s; m.protect_mask = protect;
    run(&m, cap);
    *o = m.res;
    if (cap_out) { *cap_out = m.out; m.out.buf = NULL; }
    mach_free(&m);
}

typedef struct {
    const or_campaign_t *c; const or_site_t *sites; u64 n; u64 protect; u64 cap;
    or_outcome_t *out; int tid, nth;
} job_t;

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    for (u64 i = (u64)j->tid; i < j->n; i += (u64)j->nth)
        run_trial(j->c, &j->sites[i], j->protect, j->cap, &j->out[i], NULL);
    return NULL;
}

void or_set_protect_opclasses(or_campaign_t *c, u64 mask) { c->protect_opc = mask; }
void or_set_exe_path(or_campaign_t *c, const char *path) {
    snprintf(c->exe_path, sizeof c->exe_path, "%s", path ? path : "");
}
int or_set_stdin(or_campaign_t *c, const uint8_t *data, u64 len) {
    free(c->in_data);
    c->in_data = NULL; c->in_len = 0;
    if (!data) return 0;
    c->in_data = (uint8_t *)malloc(len ? len : 1);
    if (!c->in_data) return -1;
    memcpy(c->in_data, data, len);
    c->in_len = len;
    return 0;
}
void or_set_clock(or_campaign_t *c, u64 period_ticks, u64 random_seed) {
    c->clk_period = period_ticks;
    c->rnd_seed = random_seed;
}

int or_run_trials(or_campaign_t *c, const or_site_t *sites, u64 n, u64 protect, u64 f16, or_outcome_t *out,
                  int nth) {
    if (!c->have_golden) { snprintf(c->err, sizeof c->err, "golden run required"); return -1; }
    u64 cap = hang_cap(c, f16);
    if (nth <= 1) {
        for (u64 i = 0; i < n; i++) run_trial(c, &sites[i], protect, cap, &out[i], NULL);
        return 0;
    }
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nth);
    job_t *jobs = (job_t *)malloc(sizeof(job_t) * nth);
    for (int t = 0; t < nth; t++) {
        jobs[t] = (job_t){c, sites, n, protect, cap, out, t, nth};
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    for (int t = 0; t < nth; t++) pthread_join(th[t], NULL);
    free(th); free(jobs);
    return 0;
}

int or_run_one_capture(or_campaign_t *c, const or_site_t *site, u64 protect, u64 f16, or_outcome_t *out,
                       uint8_t *buf, u64 capn, u64 *len) {
    if (!c->have_golden && site) { snprintf(c->err, sizeof c->err, "golden run required"); return -1; }
    bytes_t b = {0};
    u64 cap = c->have_golden ? hang_cap(c, f16) : (u64)1 << 40;
    run_trial(c, site, protect, cap, out, &b);
    u64 n = b.len < capn ? b.len : capn;
    if (n) memcpy(buf, b.buf, n);
    *len = b.len;
    free(b.buf);
    return 0;
}

/* Diagnostics: one trial with its committed pcs (first pcap) and the
 * addresses of its stores into the text range (first wcap); *pn / *wn = the
 * totals.  Tooling only (tools/trial_trace.py). */
static int debug_trace(or_campaign_t *c, const or_site_t *site, u64 f16, or_outcome_t *out, u64 *pcs, u64 pcap, u64 *pn,
                       u64 *wrs, u64 wcap, u64 *wn, int raw) {
    if (!c->have_golden) { snprintf(c->err, sizeof c->err, "golden run required"); return -1; }
    mach_t m; mach_init(&m, c);
    m.site = site;
    m.dbg_raw = raw;
    m.dbg_pc = pcs; m.dbg_pc_cap = pcap; m.dbg_wr = wrs; m.dbg_wr_cap = wcap;
    run(&m, hang_cap(c, f16));
    *out = m.res; *pn = m.dbg_pc_n; *wn = m.dbg_wr_n;
    mach_free(&m);
    return 0;
}
int or_debug_trace(or_campaign_t *c, const or_site_t *site, u64 f16, or_outcome_t *out, u64 *pcs, u64 pcap, u64 *pn,
                   u64 *wrs, u64 wcap, u64 *wn) {
    return debug_trace(c, site, f16, out, pcs, pcap, pn, wrs, wcap, wn, 0);
}
/* the same with each committed instruction's word in the high half (the pc's low 32 bits below) */
int or_debug_trace_raw(or_campaign_t *c, const or_site_t *site, u64 f16, or_outcome_t *out, u64 *pcs, u64 pcap,
                       u64 *pn, u64 *wrs, u64 wcap, u64 *wn) {
    return debug_trace(c, site, f16, out, pcs, pcap, pn, wrs, wcap, wn, 1);
}

/* ------------------------------------------------------------- probe */
int or_probe(u32 inst, u64 pc, const u64 regs[32], or_probe_t *o) {
    static or_campaign_t dummy;   /* stack VMA empty: no fixups */
    mach_t m; memset(&m, 0, sizeof m);
    m.c = &dummy;
    pm_init(&m.mem, 64);
    for (int i = 0; i < 32; i++) m.x[i] = regs[i];
    m.x[0] = 0;
    m.pc = pc; m.watch = -1; m.stack_min = STACK_BASE; m.resv = m.lock = OR_NONE;
    dec_t d; decode(inst, &d);
    m.npc = pc + d.len;
    /* memory: every page the access touches is mapped zero (probe semantics) */
    if (d.rs1 >= 0) {
        u64 ea = rdreg(&m, d.rs1) + d.imm;
        alloc_page(&m, ea & PAGE_MASK);
        alloc_page(&m, (ea + 7) & PAGE_MASK);
    }
    u64 fva = 0;
    int f = execute(&m, &d, &fva);
    o->fault = f == F_NONE ? 0 : f == F_SYSCALL ? 1 : f == F_BREAK ? 2 : f == F_ILLEGAL ? 3 :
               f == F_UNKNOWN ? 4 : f == F_PGFAULT ? 6 : f == F_VSEW ? 11 : 5;
    o->rd = d.rd;
    o->rd_value = d.rd > 0 ? m.x[d.rd] : 0;
    if (d.rd < 0 && d.frd >= 0) { o->rd = 32 + d.frd; o->rd_value = m.f[d.frd]; }   /* FP destination: 32 + f */
    o->npc = m.npc;
    o->len = d.len;
    o->op = (u32)d.op;
    pm_free(&m.mem);
    return 0;
}

/* ------------------------------------------------------------ checkpoints */
/* gem5 SE checkpoints (test infrastructure).  The writer produces what
 * gem5's serialization writes for this machine (m5.cpt INI sections and a
 * gzip-compressed physical memory store; formats cited in
 * shrewd_amd/csrc/fi_checkpoint.cpp): thread context [system.cpu.xc.0]
 * (serialize(tc), cpu/thread_context.cc:194-218; 33 integer registers,
 * int.hh:62-80), process [system.cpu.workload] (MemState::serialize,
 * sim/mem_state.hh:189-210), its page table (page_table.cc:186-201) and
 * [system.physmem] (physical.cc:340-405), frames assigned in vpn order.  The
 * reader is the oracle's own restatement of the restore
 * (Process::unserialize, sim/process.cc:427-441). */
/* MiscRegIndex (src/arch/riscv/regs/misc.hh) positions the checkpoint uses */
enum { CPT_MISC_FFLAGS = 120, CPT_MISC_FRM = 121, CPT_NUM_MISC = 193 };

static void cpt_bytes(FILE *f, const char *name, const uint8_t *b, int n) {
    fprintf(f, "%s=", name);
    for (int i = 0; i < n; i++) fprintf(f, i ? " %u" : "%u", b[i]);
    fprintf(f, "\n");
}

int or_write_checkpoint(or_campaign_t *c, uint64_t ninst, const char *dir) {
    if (!c->have_golden || ninst >= c->golden.ninst) {
        snprintf(c->err, sizeof c->err, "or_write_checkpoint: need a golden run longer than %llu",
                 (unsigned long long)ninst);
        return -1;
    }
    mach_t m; mach_init(&m, c);
    while (!m.done && m.num_inst < ninst) tick(&m, UINT64_MAX);
    if (m.done || m.stay_at_pc || m.fetch_offset) { mach_free(&m); snprintf(c->err, sizeof c->err, "not at a boundary"); return -1; }
    if (mkdir(dir, 0755) && errno != EEXIST) { mach_free(&m); snprintf(c->err, sizeof c->err, "mkdir %s", dir); return -1; }
    char path[4096];
    /* pages in vpn order -> frames 0, 1, ... */
    u64 n = 0;
    for (u64 i = 0; i < m.mem.cap; i++) if (m.mem.tab[i].vpn != UINT64_MAX) n++;
    u64 *vpns = (u64 *)malloc(sizeof(u64) * (n ? n : 1));
    uint8_t **data = (uint8_t **)malloc(sizeof(uint8_t *) * (n ? n : 1));
    u64 k = 0;
    for (u64 i = 0; i < m.mem.cap; i++) if (m.mem.tab[i].vpn != UINT64_MAX) { vpns[k] = m.mem.tab[i].vpn; k++; }
    for (u64 i = 1; i < n; i++)
        for (u64 j = i; j > 0 && vpns[j - 1] > vpns[j]; j--) { u64 t = vpns[j]; vpns[j] = vpns[j - 1]; vpns[j - 1] = t; }
    for (u64 i = 0; i < n; i++) data[i] = pm_find(&m.mem, vpns[i])->data;
    snprintf(path, sizeof path, "%s/system.physmem.store0.pmem", dir);
    gzFile gz = gzopen(path, "wb");
    for (u64 i = 0; gz && i < n; i++) gzwrite(gz, data[i], (unsigned)PAGE);
    if (gz) gzclose(gz);
    snprintf(path, sizeof path, "%s/m5.cpt", dir);
    FILE *f = fopen(path, "w");
    if (!gz || !f) { free(vpns); free(data); mach_free(&m); if (f) fclose(f); snprintf(c->err, sizeof c->err, "write %s", dir); return -1; }
    fprintf(f, "## checkpoint generated by oracle/rv64se.c:or_write_checkpoint at numInst %llu\n\n",
            (unsigned long long)ninst);
    fprintf(f, "[Globals]\ncurTick=%llu\n\n", (unsigned long long)(c->tick0 + m.num_cycles * c->clk_period));
    fprintf(f, "[system.cpu.xc.0]\n_status=1\n");
    uint8_t ib[33 * 8], fb[32 * 8];
    memset(ib, 0, sizeof ib);
    for (int r = 1; r < 32; r++) for (int b = 0; b < 8; b++) ib[r * 8 + b] = (uint8_t)(m.x[r] >> (8 * b));
    for (int r = 0; r < 32; r++) for (int b = 0; b < 8; b++) fb[r * 8 + b] = (uint8_t)(m.f[r] >> (8 * b));
    cpt_bytes(f, "regs.integer", ib, 33 * 8);
    cpt_bytes(f, "regs.floating_point", fb, 32 * 8);
    /* PCState (generic/pcstate.hh:141-145, 329-333; riscv/pcstate.hh:146-156): vtype/vl as at
     * process start (vill), the only vector configuration the engine models */
    fprintf(f, "_pc=%llu\n_upc=0\n_npc=%llu\n_nupc=1\n_rvType=1\n_new_vconf=false\n_vtype=%llu\n_vl=0\n"
               "_compressed=false\n_zcmtSecondFetch=false\n_zcmtPc=0\n\n",
            (unsigned long long)m.pc, (unsigned long long)(m.pc + 4), 1ULL << 63);
    /* the ISA's misc registers (ISA::serialize, isa.cc:977-983: miscRegFile,
     * NUM_PHYS_MISCREGS values in MiscRegIndex order, regs/misc.hh); the
     * oracle models fflags and frm (indices in tests/golden/riscv_miscreg.json) */
    fprintf(f, "[system.cpu.isa]\nmiscRegFile=");
    for (int i = 0; i < CPT_NUM_MISC; i++)
        fprintf(f, i ? " %u" : "%u", i == CPT_MISC_FFLAGS ? m.fflags : i == CPT_MISC_FRM ? m.frm : 0u);
    fprintf(f, "\n\n");
    fprintf(f, "[system.cpu.workload]\nbrkPoint=%llu\nstackBase=%llu\nstackSize=%llu\nmaxStackSize=%llu\n"
               "stackMin=%llu\nnextThreadStackBase=%llu\nmmapEnd=%llu\n\n",
            (unsigned long long)m.brk, (unsigned long long)STACK_BASE, (unsigned long long)(STACK_BASE - m.stack_min),
            (unsigned long long)MAX_STACK, (unsigned long long)m.stack_min,
            (unsigned long long)(STACK_BASE - MAX_STACK), (unsigned long long)m.mmap_end);
    fprintf(f, "[system.cpu.workload.vmalist]\nsize=%d\n\n", m.nvma);
    for (int i = 0; i < m.nvma; i++)
        fprintf(f, "[system.cpu.workload.vmalist.Vma%d]\nname=%s\naddrRangeStart=%llu\naddrRangeEnd=%llu\n\n", i,
                (m.vma[i].lo == c->stack_vma_lo && m.vma[i].hi == c->stack_vma_hi) ? "stack" : "anon",
                (unsigned long long)m.vma[i].lo, (unsigned long long)m.vma[i].hi);
    fprintf(f, "[system.cpu.workload.ptable]\nsize=%llu\n\n", (unsigned long long)n);
    for (u64 i = 0; i < n; i++)
        fprintf(f, "[system.cpu.workload.ptable.Entry%llu]\nvaddr=%llu\npaddr=%llu\nflags=0\n\n", (unsigned long long)i,
                (unsigned long long)(vpns[i] << 12), (unsigned long long)(i << 12));
    fprintf(f, "[system.physmem]\nlal_addr=\nlal_cid=\nnbr_of_stores=1\n\n");
    fprintf(f, "[system.physmem.store0]\nstore_id=0\nfilename=system.physmem.store0.pmem\nrange_size=%llu\n",
            (unsigned long long)(n << 12));
    fclose(f);
    free(vpns); free(data);
    mach_free(&m);
    return 0;
}

/* m5.cpt reader: section/key lookup by a linear scan of the file's lines */
typedef struct { char **lines; int n; } cpt_t;
static int cpt_load(cpt_t *t, const char *path) {
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    t->lines = NULL; t->n = 0;
    char *line = NULL; size_t cap = 0; ssize_t len;
    int capn = 0;
    while ((len = getline(&line, &cap, f)) >= 0) {
        while (len > 0 && (line[len - 1] == '\n' || line[len - 1] == '\r')) line[--len] = 0;
        if (t->n == capn) { capn = capn ? 2 * capn : 1024; t->lines = (char **)realloc(t->lines, sizeof(char *) * capn); }
        t->lines[t->n++] = strdup(line);
    }
    free(line);
    fclose(f);
    return 0;
}
static void cpt_free(cpt_t *t) { for (int i = 0; i < t->n; i++) free(t->lines[i]); free(t->lines); }
/* value of key in section sec (NULL if absent) */
static const char *cpt_get(const cpt_t *t, const char *sec, const char *key) {
    int in = 0;
    size_t kl = strlen(key);
    for (int i = 0; i < t->n; i++) {
        const char *l = t->lines[i];
        if (l[0] == '[') { in = strlen(l) == strlen(sec) + 2 && !strncmp(l + 1, sec, strlen(sec)); continue; }
        if (in && !strncmp(l, key, kl) && l[kl] == '=') return l + kl + 1;
    }
    return NULL;
}
/* the first section holding key (copied into out) */
static int cpt_find(const cpt_t *t, const char *key, char *out, size_t cap) {
    const char *sec = NULL;
    size_t kl = strlen(key);
    for (int i = 0; i < t->n; i++) {
        const char *l = t->lines[i];
        if (l[0] == '[') { sec = l; continue; }
        if (sec && !strncmp(l, key, kl) && l[kl] == '=') {
            size_t n = strlen(sec) - 2;
            if (n >= cap) return -1;
            memcpy(out, sec + 1, n); out[n] = 0;
            return 0;
        }
    }
    return -1;
}
static u64 cpt_u64(const cpt_t *t, const char *sec, const char *key, int *ok) {
    const char *v = cpt_get(t, sec, key);
    if (!v) { *ok = 0; return 0; }
    return strtoull(v, NULL, 0);
}

/* Memory-fault candidates of a checkpoint start: as at process start (the
 * ELF's writable segments and the stack), every mapped page that no read-only
 * PT_LOAD segment covers -- writable segments, stack, heap and mmap pages. */
static int cpt_fault_page(const or_campaign_t *c, u64 va) {
    int ro = 0;
    for (int i = 0; i < c->nseg; i++)
        if (va >= c->seg[i].lo && va < c->seg[i].hi) {
            if (c->seg[i].w) return 1;
            ro = 1;
        }
    return !ro;
}

or_campaign_t *or_create_checkpoint(const char *dir, const uint8_t *elf, size_t len) {
    or_campaign_t *c = or_create(elf, len, "checkpoint");
    if (c->err[0]) return c;
    char path[4096], xc[512], ps[512], pm[512], sec[1024];
    snprintf(path, sizeof path, "%s/m5.cpt", dir);
    cpt_t t;
    if (cpt_load(&t, path)) { snprintf(c->err, sizeof c->err, "cannot read %.200s", path); return c; }
    int ok = 1;
    if (cpt_find(&t, "regs.integer", xc, sizeof xc) || cpt_find(&t, "brkPoint", ps, sizeof ps) ||
        cpt_find(&t, "nbr_of_stores", pm, sizeof pm)) {
        snprintf(c->err, sizeof c->err, "m5.cpt lacks a thread context, process or memory"); cpt_free(&t); return c;
    }
    /* registers: 8 bytes each, little-endian, x0 first */
    const char *v = cpt_get(&t, xc, "regs.integer");
    memset(c->regs0, 0, sizeof c->regs0);
    for (int i = 0; i < 32 * 8 && v && *v; i++) {
        char *e;
        unsigned long b = strtoul(v, &e, 10);
        if (e == v) break;
        if (i >= 8) c->regs0[i / 8] |= (u64)(b & 0xFF) << (8 * (i % 8));
        v = e;
    }
    const char *fv = cpt_get(&t, xc, "regs.floating_point");
    memset(c->f0, 0, sizeof c->f0);
    for (int i = 0; i < 32 * 8 && fv && *fv; i++) {
        char *e;
        unsigned long b = strtoul(fv, &e, 10);
        if (e == fv) break;
        c->f0[i / 8] |= (u64)(b & 0xFF) << (8 * (i % 8));
        fv = e;
    }
    /* fflags / frm from the ISA's miscRegFile (absent: zero) */
    c->fflags0 = c->frm0 = 0;
    char isa[512];
    if (!cpt_find(&t, "miscRegFile", isa, sizeof isa)) {
        const char *mv = cpt_get(&t, isa, "miscRegFile");
        for (int i = 0; mv && *mv && i <= CPT_MISC_FRM; i++) {
            char *e;
            unsigned long long v = strtoull(mv, &e, 10);
            if (e == mv) break;
            if (i == CPT_MISC_FFLAGS) c->fflags0 = (u32)(v & 0x1F);
            if (i == CPT_MISC_FRM) c->frm0 = (u32)(v & 7);
            mv = e;
        }
    }
    /* vector configuration: only the process-start one (vtype.vill, vl 0) */
    const char *vt = cpt_get(&t, xc, "_vtype"), *vlv = cpt_get(&t, xc, "_vl");
    if ((vt && strtoull(vt, NULL, 0) != (1ULL << 63)) || (vlv && strtoull(vlv, NULL, 0) != 0)) {
        snprintf(c->err, sizeof c->err, "unsupported checkpoint (vector configuration set: vtype/vl)");
        cpt_free(&t); return c;
    }
    const char *gt = cpt_get(&t, "Globals", "curTick");
    c->tick0 = gt ? strtoull(gt, NULL, 0) : 0;
    c->pc0 = cpt_u64(&t, xc, "_pc", &ok);
    c->brk0 = cpt_u64(&t, ps, "brkPoint", &ok);
    u64 sbase = cpt_u64(&t, ps, "stackBase", &ok), smax = cpt_u64(&t, ps, "maxStackSize", &ok);
    u64 smin = cpt_u64(&t, ps, "stackMin", &ok), mend = cpt_u64(&t, ps, "mmapEnd", &ok);
    snprintf(sec, sizeof sec, "%s.vmalist", ps);
    u64 nv = cpt_u64(&t, sec, "size", &ok);
    if (!ok || sbase != STACK_BASE || smax != MAX_STACK || nv > 64) {
        snprintf(c->err, sizeof c->err, "unsupported checkpoint (stack base / max stack differ from RiscvProcess64's, "
                                        "or more than 64 VMAs)");
        cpt_free(&t); return c;
    }
    /* MemState VMA list (mem_state.hh:199-209), in order */
    c->nvma0 = (int)nv;
    for (u64 i = 0; i < nv; i++) {
        snprintf(sec, sizeof sec, "%s.vmalist.Vma%llu", ps, (unsigned long long)i);
        c->vma0[i].lo = cpt_u64(&t, sec, "addrRangeStart", &ok);
        c->vma0[i].hi = cpt_u64(&t, sec, "addrRangeEnd", &ok);
        const char *vn = cpt_get(&t, sec, "name");
        if (vn && !strcmp(vn, "stack")) { c->stack_vma_lo = c->vma0[i].lo; c->stack_vma_hi = c->vma0[i].hi; }
    }
    c->mmap_end0 = mend;
    c->stack_min0 = smin & PAGE_MASK;
    c->sp0 = c->regs0[2];
    /* page table + memory store (frames read in paddr order) */
    snprintf(sec, sizeof sec, "%s.ptable", ps);
    u64 np = cpt_u64(&t, sec, "size", &ok);
    u64 *va = (u64 *)malloc(sizeof(u64) * (np ? np : 1)), *pa = (u64 *)malloc(sizeof(u64) * (np ? np : 1));
    for (u64 i = 0; i < np; i++) {
        snprintf(sec, sizeof sec, "%s.ptable.Entry%llu", ps, (unsigned long long)i);
        va[i] = cpt_u64(&t, sec, "vaddr", &ok);
        pa[i] = cpt_u64(&t, sec, "paddr", &ok);
    }
    for (u64 i = 1; i < np; i++)
        for (u64 j = i; j > 0 && pa[j - 1] > pa[j]; j--) {
            u64 x = pa[j]; pa[j] = pa[j - 1]; pa[j - 1] = x;
            x = va[j]; va[j] = va[j - 1]; va[j - 1] = x;
        }
    snprintf(sec, sizeof sec, "%s.store0", pm);
    const char *fn = cpt_get(&t, sec, "filename");
    snprintf(path, sizeof path, "%s/%s", dir, fn ? fn : "");
    gzFile gz = fn ? gzopen(path, "rb") : NULL;
    if (!ok || !gz) { snprintf(c->err, sizeof c->err, "bad page table or memory store"); free(va); free(pa); cpt_free(&t); return c; }
    pm_free(&c->image);
    pm_init(&c->image, 64);
    u64 at = 0;
    uint8_t skip[4096];
    u64 nmem = 0;
    u64 *mp = (u64 *)malloc(sizeof(u64) * (np ? np : 1));
    for (u64 i = 0; i < np && ok; i++) {
        while (at < pa[i]) { if (gzread(gz, skip, (unsigned)PAGE) != (int)PAGE) { ok = 0; break; } at += PAGE; }
        uint8_t *pg = (uint8_t *)malloc(PAGE);
        if (!ok || at != pa[i] || gzread(gz, pg, (unsigned)PAGE) != (int)PAGE) { free(pg); ok = 0; break; }
        at += PAGE;
        pm_insert(&c->image, va[i] >> 12, pg, 1);
        if (cpt_fault_page(c, va[i])) mp[nmem++] = va[i];
    }
    gzclose(gz);
    for (u64 i = 1; i < nmem; i++)
        for (u64 j = i; j > 0 && mp[j - 1] > mp[j]; j--) { u64 x = mp[j]; mp[j] = mp[j - 1]; mp[j - 1] = x; }
    free(c->mem_pages);
    c->mem_pages = mp; c->n_mem_pages = nmem;
    if (!ok) snprintf(c->err, sizeof c->err, "memory store truncated");
    free(va); free(pa); cpt_free(&t);
    return c;
}

/* =================================================== tick-domain injection
 * (TimingSimpleCPU on the reference's SE board; rv64se.h "Tick-domain
 * injection").  One attempt = one fetch-execute of TimingSimpleCPU
 * (timing.cc:819-898): its fetch words, then either an execute that commits
 * (with its data requests, completing at completeDataAccess), or a fault
 * (ecall, a page-table fault SE fixes up) after which fetchEvent refetches. */
typedef struct {
    u64 pc, n, cyc0, next_pc;   /* pc, numInst before it, first atomic tick index, the next attempt's pc */
    int op, rd, rs1, rs2;       /* the oracle's decode of the instruction */
    uint8_t len, nfetch, kind;  /* kind: 0 commits, 1 ecall, 2 page-fault retry, 3 the run's end */
} tk_info_t;
enum { TK_COMMIT = 0, TK_ECALL = 1, TK_PGFAULT = 2, TK_END = 3 };

typedef struct tkrec {
    or_timing_op_t *ops; tk_info_t *info; u64 n, cap;
    int open;
    u64 *pv, *pp; u64 np, capp;   /* vpn -> frame, allocation order */
    char why[160];
} tkrec_t;

typedef struct tkgold {
    or_timing_op_t *ops; tk_info_t *info; or_timing_ticks_t *ticks; u64 n;
    u64 golden_ticks;
} tkgold_t;

enum { TKP_FETCH1 = 0, TKP_FETCH2 = 1, TKP_DATA = 2 };
typedef struct tkinj {
    u64 cyc;          /* atomic tick index of the attempt's tick the flip lands in */
    int phase;        /* TKP_* */
    uint32_t target; u64 mask;
} tkinj_t;

static void tk_unsupported(mach_t *m, const char *why) {
    if (m->tkr && !m->tkr->why[0]) snprintf(m->tkr->why, sizeof m->tkr->why, "%s", why);
}
static u64 tk_frame(tkrec_t *r, u64 vpn) {
    for (u64 i = 0; i < r->np; i++) if (r->pv[i] == vpn) return r->pp[i];
    return OR_NONE;
}
static void tk_page(mach_t *m, u64 vpn) {
    tkrec_t *r = m->tkr;
    if (tk_frame(r, vpn) != OR_NONE) return;
    if (r->np == r->capp) {
        r->capp = r->capp ? 2 * r->capp : 256;
        r->pv = (u64 *)realloc(r->pv, r->capp * 8); r->pp = (u64 *)realloc(r->pp, r->capp * 8);
    }
    r->pv[r->np] = vpn; r->pp[r->np] = r->np; r->np++;
}
static u64 tk_paddr(mach_t *m, u64 va) {
    u64 f = tk_frame(m->tkr, va >> 12);
    if (f == OR_NONE) { tk_unsupported(m, "an access to a page with no frame"); return 0; }
    return (f << 12) | (va & (PAGE - 1));
}
static void tk_open(mach_t *m, u64 tick_index) {
    tkrec_t *r = m->tkr;
    if (r->open) return;
    if (r->n == r->cap) {
        r->cap = r->cap ? 2 * r->cap : 4096;
        r->ops = (or_timing_op_t *)realloc(r->ops, r->cap * sizeof *r->ops);
        r->info = (tk_info_t *)realloc(r->info, r->cap * sizeof *r->info);
    }
    memset(&r->ops[r->n], 0, sizeof r->ops[0]);
    memset(&r->info[r->n], 0, sizeof r->info[0]);
    if (r->n) r->info[r->n - 1].next_pc = m->pc;
    r->info[r->n].pc = m->pc; r->info[r->n].n = m->num_inst; r->info[r->n].cyc0 = tick_index;
    r->open = 1;
}
static void tk_fetch(mach_t *m, u64 fetch_pc) {
    tkrec_t *r = m->tkr;
    or_timing_op_t *o = &r->ops[r->n];
    if (o->nfetch >= 2) { tk_unsupported(m, "more than two fetches for one instruction"); return; }
    o->fetch[o->nfetch++] = tk_paddr(m, fetch_pc);
}
static void tk_frag(mach_t *m, u64 addr, unsigned size, int cmd) {
    if (!m->tk_cpu) return;   /* syscall proxies move no CPU requests */
    tkrec_t *r = m->tkr;
    or_timing_op_t *o = &r->ops[r->n];
    if (o->nfrag >= 2) { tk_unsupported(m, "more than two data requests"); return; }
    o->addr[o->nfrag] = tk_paddr(m, addr); o->size[o->nfrag] = (uint16_t)size; o->cmd = (uint8_t)cmd;
    o->nfrag++;
}
static void tk_close(mach_t *m, int f, const dec_t *d) {
    tkrec_t *r = m->tkr;
    or_timing_op_t *o = &r->ops[r->n];
    tk_info_t *I = &r->info[r->n];
    I->op = d->op; I->rd = d->rd; I->rs1 = d->rs1; I->rs2 = d->rs2; I->len = (uint8_t)d->len;
    I->nfetch = o->nfetch;
    if (f == F_NONE + 100) {                     /* m5_exit / m5_fail ends the run after it commits */
        o->kind = OR_TOP_END; I->kind = TK_END;
    } else if (f == F_NONE) {
        o->kind = OR_TOP_EXEC; I->kind = TK_COMMIT;
        if (d->op == OP_prefetch_i || d->op == OP_prefetch_r || d->op == OP_prefetch_w)
            tk_unsupported(m, "a prefetch (a PREFETCH request) in the golden run");
        if (d->op == OP_cbo && d->imm != 4) tk_unsupported(m, "a cache-block management op in the golden run");
        if (d->op == OP_vec || d->op == OP_vset) tk_unsupported(m, "a vector op in the golden run");
    } else if (f == F_SYSCALL) {
        o->nfrag = 0;
        if (m->done) { o->kind = OR_TOP_END; I->kind = TK_END; }
        else { o->kind = OR_TOP_FAULT; I->kind = TK_ECALL; }
    } else if (f == F_PGFAULT && !m->done) {
        o->nfrag = 0; o->kind = OR_TOP_FAULT; I->kind = TK_PGFAULT;
    } else {
        tk_unsupported(m, "the golden run faults");
    }
    r->n++;
    r->open = 0;
}

/* the attempt's tick that a flip at phase lands in */
static int tk_here(const mach_t *m, u64 tick_index, int data) {
    const tkinj_t *k = m->tki;
    if (data) return k->phase == TKP_DATA && tick_index == k->cyc;
    return k->phase != TKP_DATA && tick_index == k->cyc;
}
/* before the attempt's tick: its (next) fetch request went out with the old pc */
static void tk_inject_top(mach_t *m) {
    const tkinj_t *k = m->tki;
    m->injected = 1;
    if (k->target >= 1 && k->target <= 31) {
        m->x[k->target] ^= k->mask;
    } else if (k->target == OR_T_PC) {
        m->fo = 1;
        m->fo_addr = (m->pc & ~3ULL) + m->fetch_offset;
        m->pc ^= k->mask;   /* PCState::set: npc = pc + 4 -- decode sets it again */
    } else if (k->target == OR_T_RESULT) {
        m->rarm = 1; m->rmask = k->mask;
    }
}
/* between initiateAcc and completeAcc: the completion writes rd afterwards,
 * then advancePC takes npc, which PCState::set made pc + 4 */
static void tk_inject_data(mach_t *m, const dec_t *d) {
    const tkinj_t *k = m->tki;
    m->injected = 1;
    if (k->target >= 1 && k->target <= 31) {
        if (!(m->wrote && d->rd == (int)k->target)) m->x[k->target] ^= k->mask;
    } else if (k->target == OR_T_PC) {
        m->npc = (m->pc ^ k->mask) + 4;
    } else if (k->target == OR_T_RESULT) {
        m->rarm = 1; m->rmask = k->mask;
    }
}

static int tk_is_macro(int op) {
    return (op >= OP_amoadd_w && op <= OP_amomaxu_d) || op == OP_lr_w || op == OP_lr_d || op == OP_sc_w || op == OP_sc_d;
}
/* The contract: which tick sites the numInst engine does not reproduce
 * (include/fi_engine.h FI_TK_*).  0 = reproduced. */
static int tk_contract(const tkgold_t *g, u64 j, int phase, uint32_t target, u64 mask) {
    const tk_info_t *I = &g->info[j];
    if (target == OR_T_RESULT) return 0;
    u64 gs = j;
    while (gs > 0 && (g->info[gs - 1].kind == TK_ECALL || g->info[gs - 1].kind == TK_PGFAULT)) gs--;
    if (target <= 31) {
        if (phase == TKP_DATA) return 0;
        for (u64 k = gs; k < j; k++) {
            const tk_info_t *K = &g->info[k];
            if (K->kind == TK_ECALL && target >= 10 && target <= 17) return OR_TK_NONCOUNT;
            if (K->kind == TK_PGFAULT && ((int)target == K->rs1 || (int)target == K->rs2)) return OR_TK_NONCOUNT;
        }
        return 0;
    }
    /* pc */
    if (gs != j) return OR_TK_NONCOUNT;
    const u64 pc = I->pc, npc = pc ^ mask;
    const int same_word = ((pc ^ npc) & ~3ULL) == 0;
    if (phase == TKP_DATA) return tk_is_macro(I->op) ? OR_TK_MACRO : 0;
    if (I->kind != TK_COMMIT) return (phase == TKP_FETCH1 && same_word) ? 0 : OR_TK_FAULTOP;
    const int two = I->op == OP_auipc || (I->op == OP_jal && I->rd > 0);
    if (phase == TKP_FETCH1) {
        if (same_word) return 0;
        if (I->nfetch == 2) return OR_TK_STRADDLE1;
        if ((pc & 3) != (npc & 3)) return OR_TK_ALIGN;
        return two ? OR_TK_TWO : 0;
    }
    if ((npc & 3) == 0) return OR_TK_STRADDLE2;
    return two ? OR_TK_TWO : 0;
}

static void tkgold_free(tkgold_t *g) {
    if (!g) return;
    free(g->ops); free(g->info); free(g->ticks); free(g);
}

int or_tick_setup(or_campaign_t *c, const or_timing_params_t *p) {
    if (!c->have_golden) { snprintf(c->err, sizeof c->err, "or_tick_setup: golden run required"); return -1; }
    tkgold_free(c->tk); c->tk = NULL;
    or_timing_params_t dp;
    if (!p) { or_timing_default_params(&dp); p = &dp; }
    tkrec_t r; memset(&r, 0, sizeof r);
    mach_t m; mach_init(&m, c);
    m.tkr = &r;
    for (u64 i = 0; i < c->n_alloc; i++) tk_page(&m, c->alloc_vpn[i]);   /* the image, as initState wrote it */
    run(&m, c->golden.ninst + 1);
    int rc = 0;
    if (!r.why[0] && (m.res.cls != OR_MASKED || m.num_inst != c->golden.ninst || r.n == 0 ||
                      r.ops[r.n - 1].kind != OR_TOP_END))
        snprintf(r.why, sizeof r.why, "the recorded golden run does not end with its exit");
    if (r.why[0]) {
        snprintf(c->err, sizeof c->err, "tick model: %s", r.why);
        rc = -1;
    } else {
        tkgold_t *g = (tkgold_t *)calloc(1, sizeof *g);
        g->ops = r.ops; g->info = r.info; g->n = r.n; r.ops = NULL; r.info = NULL;
        g->ticks = (or_timing_ticks_t *)calloc(g->n, sizeof *g->ticks);
        or_timing_stats_t st;
        if (or_timing_model(g->ops, g->n, p, g->ticks, &st) != 0) {
            snprintf(c->err, sizeof c->err, "tick model: a state gem5 asserts on");
            tkgold_free(g);
            rc = -1;
        } else {
            g->golden_ticks = st.ticks;
            c->tk = g;
        }
    }
    m.tkr = NULL;
    free(r.ops); free(r.info); free(r.pv); free(r.pp);
    mach_free(&m);
    return rc;
}

uint64_t or_tick_golden_ticks(or_campaign_t *c) { return c->tk ? c->tk->golden_ticks : 0; }

uint64_t or_tick_trace(or_campaign_t *c, or_timing_op_t *ops, or_timing_ticks_t *ticks, uint64_t cap) {
    if (!c->tk) return 0;
    u64 n = c->tk->n < cap ? c->tk->n : cap;
    if (ops) memcpy(ops, c->tk->ops, n * sizeof *ops);
    if (ticks) memcpy(ticks, c->tk->ticks, n * sizeof *ticks);
    return c->tk->n;
}

int or_tick_sample(or_campaign_t *c, u64 seed, u64 first, u64 n, u64 structures, u32 burst, u64 bits,
                   or_tick_site_t *out) {
    if (!c->tk) { snprintf(c->err, sizeof c->err, "or_tick_sample: or_tick_setup first"); return -1; }
    if (burst < 1 || burst > 64) burst = 1;
    structures &= ((1ULL << 32) - 2) | (1ULL << OR_T_PC) | (1ULL << OR_T_RESULT);
    int nt = __builtin_popcountll(structures);
    if (nt == 0) { snprintf(c->err, sizeof c->err, "no fault structures"); return -1; }
    for (u64 i = 0; i < n; i++) {
        u64 id = first + i;
        u64 st = seed ^ (id * 0xD6E8FEB86659FD93ULL);
        u64 r0 = splitmix(&st), r1 = splitmix(&st), r2 = splitmix(&st);
        or_tick_site_t *s = &out[i];
        s->tick = mulhi(r0, c->tk->golden_ticks);
        u64 k = mulhi(r1, (u64)nt), mm = structures;
        for (u64 j = 0; j < k; j++) mm &= mm - 1;
        s->target = (u32)__builtin_ctzll(mm);
        const u64 valid = burst == 1 ? ~0ULL : ((2ULL << (64 - burst)) - 1);
        u64 b;
        if ((bits & valid) == valid) {
            b = mulhi(r2, 65 - burst);
        } else {
            u64 bb = bits & valid;
            const u64 kk = mulhi(r2, (u64)__builtin_popcountll(bb));
            for (u64 j = 0; j < kk; j++) bb &= bb - 1;
            b = (u64)__builtin_ctzll(bb);
        }
        s->mask = (burst == 64 ? ~0ULL : ((1ULL << burst) - 1)) << b;
        s->trial = (u32)id;
    }
    return 0;
}

/* the attempt in flight at tick t (the first whose last event is at or after
 * t: a flip at t precedes every event of tick t) and the phase within it */
static void tk_locate(const tkgold_t *g, u64 t, u64 *j_out, int *phase) {
    u64 lo = 0, hi = g->n - 1;
    while (lo < hi) {
        u64 mid = (lo + hi) / 2;
        if (g->ticks[mid].done < t) lo = mid + 1; else hi = mid;
    }
    const or_timing_ticks_t *T = &g->ticks[lo];
    *j_out = lo;
    if (g->ops[lo].nfetch == 2 && t <= T->fetch_done[0]) *phase = TKP_FETCH1;
    else if (t <= T->exec) *phase = g->ops[lo].nfetch == 2 ? TKP_FETCH2 : TKP_FETCH1;
    else *phase = TKP_DATA;
}

static void tk_trial(const or_campaign_t *c, const or_tick_site_t *s, u64 cap, or_outcome_t *o, or_outcome_t *truth) {
    const tkgold_t *g = c->tk;
    u64 j; int phase;
    tk_locate(g, s->tick, &j, &phase);
    const tk_info_t *I = &g->info[j];
    tkinj_t k;
    k.phase = phase; k.target = s->target; k.mask = s->mask;
    /* the tick of the attempt the flip lands in: its first (fetch 1), its
     * second (straddle: fetch 2, and the execute that then follows) */
    k.cyc = I->cyc0 + ((phase == TKP_FETCH2 || (phase == TKP_DATA && I->nfetch == 2)) ? 1 : 0);
    const int why = tk_contract(g, j, phase, s->target, s->mask);
    or_outcome_t lit;
    memset(&lit, 0, sizeof lit);
    if (truth || !why) {
        mach_t m; mach_init(&m, c);
        m.tki = &k;
        run(&m, cap);
        lit = m.res;
        mach_free(&m);
    }
    if (truth) *truth = lit;
    if (why) {
        memset(o, 0, sizeof *o);
        o->cls = OR_ESCAPE; o->sub = OR_ESC_TIMING; o->exit_code = (uint8_t)why; o->flags = 1;
        o->detail = (u32)I->pc; o->ninst = I->n;
    } else {
        *o = lit;
    }
}

typedef struct {
    const or_campaign_t *c; const or_tick_site_t *s; u64 n, cap; or_outcome_t *out, *truth; int tid, nth;
} tkjob_t;
static void *tk_worker(void *arg) {
    tkjob_t *j = (tkjob_t *)arg;
    for (u64 i = (u64)j->tid; i < j->n; i += (u64)j->nth)
        tk_trial(j->c, &j->s[i], j->cap, &j->out[i], j->truth ? &j->truth[i] : NULL);
    return NULL;
}

int or_run_tick_trials(or_campaign_t *c, const or_tick_site_t *sites, u64 n, u64 f16, or_outcome_t *out,
                       or_outcome_t *truth, int nth) {
    if (!c->tk) { snprintf(c->err, sizeof c->err, "or_run_tick_trials: or_tick_setup first"); return -1; }
    for (u64 i = 0; i < n; i++)   /* a site lies inside the golden run: [0, golden_ticks) */
        if (sites[i].tick >= c->tk->golden_ticks) {
            snprintf(c->err, sizeof c->err, "or_run_tick_trials: site %llu at tick %llu, the run ends at %llu",
                     (unsigned long long)i, (unsigned long long)sites[i].tick,
                     (unsigned long long)c->tk->golden_ticks);
            return -1;
        }
    u64 cap = hang_cap(c, f16);
    if (nth <= 1) {
        for (u64 i = 0; i < n; i++) tk_trial(c, &sites[i], cap, &out[i], truth ? &truth[i] : NULL);
        return 0;
    }
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nth);
    tkjob_t *jobs = (tkjob_t *)malloc(sizeof(tkjob_t) * nth);
    for (int t = 0; t < nth; t++) {
        jobs[t] = (tkjob_t){c, sites, n, cap, out, truth, t, nth};
        pthread_create(&th[t], NULL, tk_worker, &jobs[t]);
    }
    for (int t = 0; t < nth; t++) pthread_join(th[t], NULL);
    free(th); free(jobs);
    return 0;
}
