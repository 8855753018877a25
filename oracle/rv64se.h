/*
 * rv64se.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement ("oracle") of gem5 v25 RISC-V AtomicSimpleCPU SE-mode
 * semantics for the fault-injection campaign path, used as the parity checker
 * for the MI355X engine in shrewd_amd/.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product never links it.
 *
 * Each function in rv64se.c cites the reference file:line it restates
 * (paths relative to the gem5/SHREWD tree).  Parity status: instruction
 * decode + integer semantics are pinned by vectors generated from gem5's own
 * ISA parser (tools/oracle/gen_isa_vectors.py -> tests/golden/); process
 * image, syscalls and crash taxonomy are restated from the cited code and
 * are "parity unpinned" against a live gem5.opt (unbuildable here: no SCons).
 */
#ifndef SHREWD_ORACLE_RV64SE_H
#define SHREWD_ORACLE_RV64SE_H

#include <stddef.h>
#include <stdint.h>

#include "timing_se.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Outcome classes and sub-codes.  Must stay identical to include/fi_engine.h. */
enum {
    OR_MASKED = 0, OR_SDC = 1, OR_CRASH = 2, OR_HANG = 3, OR_DETECTED = 4, OR_ESCAPE = 5
};
enum {
    OR_CRASH_UNKNOWN_INST = 1,  /* panic: UnknownInstFault        faults.cc:286-291 */
    OR_CRASH_ILLEGAL_INST = 2,  /* panic: IllegalInstFault        faults.cc:294-301 */
    OR_CRASH_PAGE_FAULT   = 3,  /* panic: GenericPageTableFault   sim/faults.cc:95-105 */
    OR_CRASH_SYSCALL_RANGE = 4, /* fatal: syscall out of range    syscall_desc.hh:204-214 */
    OR_CRASH_SYSCALL_UNIMPL = 5,/* fatal: unimplementedFunc       syscall_emul.cc:77-80 */
    OR_CRASH_PROXY = 6,         /* fatal: readBlob failed         port_proxy.hh:182-196 */
    OR_CRASH_FD_ASSERT = 7,     /* abort: FDArray assert          fd_array.cc:320-323 */
    OR_CRASH_SIGTRAP = 8,       /* ebreak -> kill(SIGTRAP)        faults.cc:317-322, debug.cc:64-70 */
    OR_CRASH_STACK_LIMIT = 9,   /* fatal: Maximum stack size      mem_state.cc:440 */
    OR_CRASH_AMO_LINE = 10,     /* panic: AMO across a cache line atomic.cc:569-570 */
    OR_CRASH_SC_LINE = 11,      /* abort: SC across a cache line  atomic.cc:482 assert(curr_frag_id == 0) */
    OR_CRASH_SE_PANIC = 12,     /* panic in an SE handler (null ProxyPtr, MemState::isUnmapped) */
    OR_CRASH_M5_PANIC = 13,     /* panic in an M5 pseudo-op (m5_panic, unknown initparam key) sim/pseudo_inst.* */
    OR_CRASH_VSET_SEW = 14      /* abort: vset* requesting vsew > 3, getSew's assert  arch/riscv/insts/vector.hh:55 */
};
enum {
    OR_ESC_INST = 1,            /* instruction gem5 decodes but the engine does not model */
    OR_ESC_SYSCALL = 2,         /* syscall gem5 implements but the engine does not model */
    OR_ESC_CSR = 3,             /* U-mode-accessible CSR */
    OR_ESC_HOST = 4,            /* behaviour that depends on the host (fd 0, huge buffers) */
    OR_ESC_RESOURCE = 5,        /* engine resource limit (private pages) -- device only */
    OR_ESC_UNDEF = 6,           /* gem5's own behaviour is undefined (GEM5_UNREACHABLE reached) */
    OR_ESC_TIMING = 7           /* tick-domain site the numInst engine does not reproduce (exit_code = OR_TK_*) */
};
/* OR_ESC_TIMING reasons (exit_code), the contract of include/fi_engine.h FI_TK_* */
enum {
    OR_TK_NONCOUNT = 1,   /* flip after an ecall / page-fault retry (same numInst) that the tick touches */
    OR_TK_STRADDLE1 = 2,  /* pc flip while a straddling instruction's first half is fetched: another second word */
    OR_TK_ALIGN = 3,      /* pc flip changes both the fetch word and pc % 4 */
    OR_TK_STRADDLE2 = 4,  /* pc flip to a 4-aligned pc while the decoder holds a first half */
    OR_TK_TWO = 5,        /* pc flip on auipc / jal with a link: two values change */
    OR_TK_FAULTOP = 6,    /* pc flip (another word) on an ecall / page-fault attempt */
    OR_TK_MACRO = 7,      /* pc flip while a macro-op's (AMO / LR / SC) access is outstanding */
    OR_TK_CLOCK = 8       /* the trial reads curTick (clock_gettime / rpns) */
};
enum { OR_HANG_INSTS = 1,         /* the max-insts cap (scheduleInstStop, cpu/base.cc:764-770) */
       OR_HANG_QUIESCE = 2 };      /* m5_quiesce: the only context suspends for good (thread_context.cc:167) */
/* sub-codes of MASKED / SDC: how the simulation ended (the exit event's cause) */
enum { OR_END_EXIT = 0,            /* exit / exit_group: "exiting with last active thread context" */
       OR_END_M5_EXIT = 1,         /* m5_exit: "m5_exit instruction encountered" (pseudo_inst.cc:178) */
       OR_END_M5_FAIL = 2 };       /* m5_fail: "m5_fail instruction encountered" (pseudo_inst.cc:198) */

/* structure ids for fault sites */
enum { OR_T_PC = 32, OR_T_MEM = 33, OR_T_RESULT = 34 };

typedef struct {
    uint8_t cls, sub, exit_code, flags;
    uint32_t detail;
    uint64_t ninst;
} or_outcome_t;                              /* 16 bytes == fi_outcome */

typedef struct {
    uint64_t inst;      /* numInst at whose tick-top the flip is applied */
    uint64_t mask;      /* xor mask */
    uint64_t addr;      /* memory fault: 8-byte aligned guest address */
    uint32_t target;    /* 1..31 = x reg, 32 = pc, 33 = memory word */
    uint32_t trial;     /* trial id (informational) */
} or_site_t;                                 /* 32 bytes == fi_site */

typedef struct {
    uint64_t ninst, ncycles;
    uint32_t exit_code, cls;
    uint64_t stdout_len, stderr_len;
    uint64_t fetch_bytes, data_bytes;   /* algorithmic byte counters of the golden run */
} or_golden_t;

typedef struct or_campaign or_campaign_t;

/* Build the initial process image exactly as gem5 SE would for
 * cmd=[argv0] (RiscvProcess64::argsInit, arch/riscv/process.cc:134-261). */
or_campaign_t *or_create(const uint8_t *elf, size_t elf_len, const char *argv0);
void or_destroy(or_campaign_t *c);
const char *or_error(or_campaign_t *c);

/* Campaign from a gem5 SE checkpoint directory (m5.cpt + memory store); the
 * ELF gives the executable range.  or_error() is non-empty on failure. */
or_campaign_t *or_create_checkpoint(const char *dir, const uint8_t *elf, size_t elf_len);
/* Write the golden run's state at the top of the first tick with numInst ==
 * ninst as a gem5 SE checkpoint into dir (test fixtures).  Returns 0 / -1. */
int or_write_checkpoint(or_campaign_t *c, uint64_t ninst, const char *dir);

/* Fault-free run; records golden stdout/stderr/exit code/instruction count. */
int or_golden(or_campaign_t *c, uint64_t max_inst, or_golden_t *out);
/* copies golden stdout into buf (up to cap bytes); returns length */
uint64_t or_golden_stdout(or_campaign_t *c, uint8_t *buf, uint64_t cap);
/* same for golden stderr */
uint64_t or_golden_stderr(or_campaign_t *c, uint8_t *buf, uint64_t cap);

/* Counter-based site sampler: SplitMix64 keyed by (seed, trial).  structures
 * is a bitmask over {bit r = x_r (1..31), bit 32 = pc, bit 33 = memory}; bits
 * the eligible lowest flipped bit positions (~0: all). */
int or_sample(or_campaign_t *c, uint64_t seed, uint64_t first_trial, uint64_t n,
              uint64_t structures, uint32_t burst, uint64_t bits, or_site_t *sites);

/* SHREWD selective replication by instruction class: bit k = gem5 OpClass
 * enum value k (src/cpu/FuncUnit.py).  A result fault on a replicated
 * instruction is detected (see rv64se.c:result_fault). */
void or_set_protect_opclasses(or_campaign_t *c, uint64_t mask);
/* SHREWD functional-unit contention (include/fi_engine.h, fi_issue_*): the
 * same parameter, op and counter layouts as fi_issue_params / fi_issue_op /
 * fi_issue_stats. */
typedef struct {
    uint32_t issue_width, dispatch_width, commit_width, iq_entries, rob_entries, load_latency;
    uint32_t priority_to_shadow;
    uint32_t fu_count[6];   /* IntALU, IntMultDiv, FP_ALU, FP_MultDiv, RdWrPort, IprPort */
} or_issue_params_t;
typedef struct {
    uint64_t src, dst;      /* bit r = x_r (1..31), bit 32 = FP state */
    uint8_t opclass, kind, pad[6];
} or_issue_op_t;
enum { OR_ISSUE_PLAIN = 0, OR_ISSUE_LOAD = 1, OR_ISSUE_STORE = 2, OR_ISSUE_SERIAL = 3 };
typedef struct {
    uint64_t ops, cycles, shadow_available, shadow_not_available, shadow_same_fu, shadow_not_same_fu;
    uint64_t class_available[12], class_not_available[12];
} or_issue_stats_t;
/* Replay ops[0..n) through the O3 issue model; shadow[i] = 1 if op i's shadow
 * was issued.  Returns 0, or -1 on bad parameters. */
int or_issue_model(const or_issue_op_t *ops, uint64_t n, const or_issue_params_t *p, uint8_t *shadow,
                   or_issue_stats_t *stats);
/* Turn the model on for result faults (p = NULL: off).  Runs the golden
 * program once more to record its trace.  Returns 0 or -1. */
int or_set_issue_model(or_campaign_t *c, const or_issue_params_t *p);
/* The golden run's trace as replayed ops (one per committed instruction and
 * ecall): copies up to cap, returns the count (needs or_golden first). */
uint64_t or_golden_ops(or_campaign_t *c, or_issue_op_t *out, uint64_t cap);
/* shadow per golden numInst index; returns the count (golden ninst) */
uint64_t or_shadow_map(or_campaign_t *c, uint8_t *buf, uint64_t cap, or_issue_stats_t *stats);

/* realpath of the executable, what readlinkat("/proc/self/exe") answers
 * (syscall_emul.hh:1089-1111); "" (default): that call escapes as host */
void or_set_exe_path(or_campaign_t *c, const char *path);
/* Process.input (src/sim/Process.py:44): data = the input file's bytes, read
 * by read(0) from offset 0 (syscall_emul.hh:2798-2822); NULL (default) =
 * "cin", the host's stdin (reads of fd 0 escape as host).  Returns 0 / -1. */
int or_set_stdin(or_campaign_t *c, const uint8_t *data, uint64_t len);
/* SE time and randomness: ticks per CPU cycle (clock_gettime; default 500 =
 * 2 GHz) and gem5's Random global seed (getrandom; default 5489) */
void or_set_clock(or_campaign_t *c, uint64_t period_ticks, uint64_t random_seed);

/* Run trials from scratch (no golden snapshots, no early exit): the plain
 * serial semantics the GPU engine must reproduce bit for bit. */
int or_run_trials(or_campaign_t *c, const or_site_t *sites, uint64_t n,
                  uint64_t protect_mask, uint64_t hang_factor_x16,
                  or_outcome_t *out, int n_threads);

/* ---- Tick-domain injection under TimingSimpleCPU (include/fi_engine.h):
 * the golden run again, recording every fetch / execute attempt's requests
 * (physical addresses: frames in allocation order from 0) -> timing_se.c ->
 * the tick of each attempt.  A trial's flip at tick t is applied inside the
 * attempt in flight, as the gem5 components would see it: before its fetch
 * response (the decoder then reads the word fetched before the flip), between
 * the two fetches of a straddling instruction, or while its data access is
 * outstanding (a load's completion overwrites its rd; a pc flip resets npc to
 * pc + 4).  Returns 0, or -1 with or_error() giving the reason (unsupported
 * golden run: unmaps, clock reads, failed SC, prefetch / cache-block ops,
 * vector ops). */
int or_tick_setup(or_campaign_t *c, const or_timing_params_t *p);
uint64_t or_tick_golden_ticks(or_campaign_t *c);
/* copies up to cap attempts (requests and ticks); returns the count */
uint64_t or_tick_trace(or_campaign_t *c, or_timing_op_t *ops, or_timing_ticks_t *ticks, uint64_t cap);
typedef struct {
    uint64_t tick;      /* flip applied before every event of this tick */
    uint64_t mask;
    uint32_t target;    /* 1..31, OR_T_PC, OR_T_RESULT */
    uint32_t trial;
} or_tick_site_t;
/* SplitMix64 keyed by (seed, trial), as or_sample, with tick = mulhi(r0, golden ticks) */
int or_tick_sample(or_campaign_t *c, uint64_t seed, uint64_t first, uint64_t n, uint64_t structures, uint32_t burst,
                   uint64_t bits, or_tick_site_t *out);
/* out[i] = the trial's outcome (an escape the contract names is reported as
 * OR_ESC_TIMING without running it); truth (may be NULL) = the literal outcome
 * of every trial, escapes included */
int or_run_tick_trials(or_campaign_t *c, const or_tick_site_t *sites, uint64_t n, uint64_t hang_factor_x16,
                       or_outcome_t *out, or_outcome_t *truth, int n_threads);

/* Diagnostics: run one trial and return its full stdout in buf. */
int or_run_one_capture(or_campaign_t *c, const or_site_t *site, uint64_t protect_mask,
                       uint64_t hang_factor_x16, or_outcome_t *out,
                       uint8_t *stdout_buf, uint64_t cap, uint64_t *stdout_len);

/* Single-instruction semantic probe used by the ISA-vector tests: executes
 * inst at pc with the given x[rs1]/x[rs2] values in a scratch machine whose
 * memory is one zero page at 0x1000 (loads/stores clamp there) and reports
 * the value written to rd, the next pc and the fault kind. */
typedef struct {
    uint64_t rd_value, npc;
    int32_t fault;      /* 0 none, 1 syscall, 2 breakpoint, 3 illegal, 4 unknown, 5 escape (and other
                           ends), 6 pagefault, 11 vset's vsew assert */
    int32_t rd;         /* destination register written, -1 none (32 + f for an FP destination) */
    uint32_t len;
    uint32_t op;        /* oracle-internal op id */
} or_probe_t;
int or_probe(uint32_t inst, uint64_t pc, const uint64_t regs[32], or_probe_t *out);
/* decode-only probe: returns a stable mnemonic string for inst ("unknown" for
 * gem5 Unknown, "escape:<name>" for modelled-as-escape encodings) */
const char *or_mnemonic(uint32_t inst);
/* syscall classification (0 absent,1 unimpl,2 ignore,3 escape,4 modelled) */
int or_sys_class(int num);
/* the reference's rvk.hh (oracle/_ref) present: Zkn/Zks execute; or_rvk runs
 * function fn (shrewd_amd/csrc/hip/fi_crypto.h numbering) over vectors */
int or_has_rvk(void);
void or_rvk(int fn, const uint64_t *a, const uint64_t *b, uint64_t n, uint64_t *out);
/* SoftFloat (oracle/_ref) present: F/D/Zfh arithmetic executes */
int or_has_softfloat(void);
/* the reference SoftFloat over operand vectors (op / fmt codes of
 * shrewd_amd/csrc/hip/fi_softfp.h): the pinning tests' expected values */
void or_sf_ref(int op, int fmt, int rm, const uint64_t *a, const uint64_t *b, const uint64_t *c, uint64_t n,
               uint64_t *out, uint32_t *fl);

#ifdef __cplusplus
}
#endif
#endif
