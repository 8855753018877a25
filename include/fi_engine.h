/*
 * fi_engine.h -- C ABI of the MI355X fault-injection campaign engine.
 *
 * This is the drop-in boundary for SHREWD/gem5's fault-injection campaign
 * path.  A gem5 `FaultCampaign` SimObject
 * (src/gem5ext/fault_campaign.cc) or a plain ctypes caller
 * (configs/fi_campaign.py, shrewd_amd/fi.py) drives it.  What each entry point
 * replaces in the reference:
 *
 *   fi_load_elf    Process ctor + Process::initState + RiscvProcess64::argsInit
 *                  (src/sim/process.cc:113-165,289-306;
 *                   src/arch/riscv/process.cc:71-82,98-113,134-261): builds the
 *                  initial SE process image of the workload binary.
 *   fi_golden_run  one fault-free `m5.simulate()` of the workload under
 *                  AtomicSimpleCPU (src/cpu/simple/atomic.cc:611-739), i.e. the
 *                  run a campaign compares every trial against.
 *   fi_run_trials  N independent gem5 runs, each with a BaseCPU::scheduleInstStop-
 *                  style instruction-count event (src/cpu/base.cc:764-770,
 *                  src/cpu/simple/base.cc:321-325) that flips the sampled bit(s),
 *                  followed by exit-code/stdout comparison against the golden run.
 *                  The per-trial loop is the AtomicSimpleCPU::tick loop, executed
 *                  on the GPU one trial per lane.
 *   fi_set_protect setEnableShrewd-style runtime knob (src/cpu/o3/BaseO3CPU.py:69-72,
 *                  src/cpu/o3/cpu.hh:298-302): the selective-replication mask.
 *
 * Conventions: opaque handle; caller-owned host output buffers; integer status
 * (0 = ok) plus a per-engine last-error string; one engine per host thread,
 * bound to one HIP device; never aborts the host process -- a guest "crash" is
 * a classified outcome.  There is no CPU execution path behind this ABI: if
 * the HIP device or kernels are unavailable every call fails with
 * FI_E_NODEVICE.
 */
#ifndef SHREWD_FI_ENGINE_H
#define SHREWD_FI_ENGINE_H

#ifndef __HIPCC_RTC__
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t fi_status;
#define FI_OK 0
#define FI_E_ARG -1
#define FI_E_NODEVICE -2
#define FI_E_HIP -3
#define FI_E_ELF -4
#define FI_E_STATE -5
#define FI_E_GOLDEN -6

/* Outcome classes (masked / SDC / crash / hang / detected-by-replica) plus
 * ESCAPE: behaviour gem5 has that the engine does not model -- reported, never
 * guessed. */
#define FI_MASKED 0
#define FI_SDC 1
#define FI_CRASH 2
#define FI_HANG 3
#define FI_DETECTED 4
#define FI_ESCAPE 5
#define FI_N_CLASS 6

/* FI_CRASH sub-codes: the gem5 process outcome */
#define FI_CRASH_UNKNOWN_INST 1   /* panic  UnknownInstFault      arch/riscv/faults.cc:286-291 */
#define FI_CRASH_ILLEGAL_INST 2   /* panic  IllegalInstFault      arch/riscv/faults.cc:294-301 */
#define FI_CRASH_PAGE_FAULT 3     /* panic  GenericPageTableFault sim/faults.cc:95-105 */
#define FI_CRASH_SYSCALL_RANGE 4  /* fatal  syscall out of range  sim/syscall_desc.hh:204-214 */
#define FI_CRASH_SYSCALL_UNIMPL 5 /* fatal  unimplementedFunc     sim/syscall_emul.cc:77-80 */
#define FI_CRASH_PROXY 6          /* fatal  readBlob failed       mem/port_proxy.hh:182-196 */
#define FI_CRASH_FD_ASSERT 7      /* abort  FDArray assert        sim/fd_array.cc:320-323 */
#define FI_CRASH_SIGTRAP 8        /* ebreak -> SIGTRAP            arch/riscv/faults.cc:317-322 */
#define FI_CRASH_STACK_LIMIT 9    /* fatal  max stack exceeded    sim/mem_state.cc:440 */
#define FI_CRASH_AMO_LINE 10      /* panic  AMO across a cache line cpu/simple/atomic.cc:569-570 */
#define FI_CRASH_SC_LINE 11       /* abort  SC across a cache line  cpu/simple/atomic.cc:482 assert(curr_frag_id == 0) */
#define FI_CRASH_SE_PANIC 12      /* panic  in an SE syscall handler (null ProxyPtr, MemState::isUnmapped) */
#define FI_CRASH_M5_PANIC 13      /* panic  in an M5 pseudo-op (m5_panic, unknown initparam key) sim/pseudo_inst.* */
#define FI_CRASH_VSET_SEW 14      /* abort  vset* requesting vsew > 3: getSew's assert  arch/riscv/insts/vector.hh:55 */
/* FI_HANG sub-codes */
#define FI_HANG_INSTS 1           /* the max-insts cap (hang_factor_x16 x golden numInst) */
#define FI_HANG_QUIESCE 2         /* m5_quiesce: the only context suspends for good (sim/pseudo_inst.cc:117) */
/* FI_MASKED / FI_SDC sub-codes: how the run ended (the simulate() exit cause) */
#define FI_END_EXIT 0             /* exit / exit_group: "exiting with last active thread context" */
#define FI_END_M5_EXIT 1          /* m5_exit(0): "m5_exit instruction encountered" (sim/pseudo_inst.cc:178) */
#define FI_END_M5_FAIL 2          /* m5_fail(0, code): "m5_fail instruction encountered" (:198); exit_code = code */
/* FI_ESCAPE sub-codes */
#define FI_ESC_INST 1
#define FI_ESC_SYSCALL 2
#define FI_ESC_CSR 3
#define FI_ESC_HOST 4
#define FI_ESC_RESOURCE 5   /* an engine bound: exit_code 0 = private pages (re-run with more before the
                              histogram), 1 = the VMA list / getrandom table (bounded in the oracle too) */
#define FI_ESC_UNDEF 6      /* gem5's own behaviour is undefined (GEM5_UNREACHABLE: an RVV floating-point op at SEW = 8) */
#define FI_ESC_TIMING 7     /* a tick-domain site (fi_run_tick_trials) whose TimingSimpleCPU effect is not a
                               numInst injection; exit_code = FI_TK_* (the reason), detail = the pc in flight */
/* FI_ESC_TIMING reasons.  A flip at tick t lands inside the instruction in
 * flight; most such flips equal a numInst injection (fi_run_tick_trials
 * maps them), these do not: */
#define FI_TK_NONCOUNT 1    /* after an ecall / a page-fault retry (no numInst step) that reads or writes the
                               flipped register (ecall: a0..a7; retry: rs1, rs2), or any pc flip there */
#define FI_TK_STRADDLE1 2   /* pc flip while the first half of a 32-bit instruction at pc % 4 == 2 is fetched,
                               to another word: the second fetch reads a third word */
#define FI_TK_ALIGN 3       /* pc flip that changes the fetch word and pc % 4 (the decoder re-slices the word) */
#define FI_TK_STRADDLE2 4   /* pc flip to a 4-aligned pc while the decoder holds a first half (Decoder::moreBytes
                               takes the aligned path with mid still set, arch/riscv/decoder.cc:63-116) */
#define FI_TK_TWO 5         /* pc flip while auipc / jal with a link is fetched: rd and the next pc both change */
#define FI_TK_FAULTOP 6     /* pc flip to another word on an ecall / page-fault attempt */
#define FI_TK_MACRO 7       /* pc flip while an AMO / LR / SC (a macro-op) has its access outstanding */
#define FI_TK_CLOCK 8       /* the trial reads curTick (clock_gettime, rpns): the engine keeps AtomicSimpleCPU's
                               clock */

/* Fault-site structures: 1..31 = x1..x31, 32 = pc, 33 = 8-byte memory word,
 * 34 = the result of an instruction: the value the first instruction that
 * commits at or after the inject time writes to x[rd] (a transient fault in the
 * functional unit that SHREWD's shadow execution targets) */
#define FI_T_PC 32
#define FI_T_MEM 33
#define FI_T_RESULT 34
#define FI_N_STRUCT 35

typedef struct {
    uint8_t cls, sub, exit_code, flags;  /* flags bit0: injected, bit1: memory site unmapped at t */
    uint32_t detail;                     /* low 32 bits of pc at termination / fault va / syscall #; 0 for a hang */
    uint64_t ninst;                      /* committed guest instructions (numInst) at termination */
} fi_outcome;

typedef struct {
    uint64_t inst;    /* numInst at whose tick the flip is applied */
    uint64_t mask;    /* xor mask (burst of adjacent bits) */
    uint64_t addr;    /* memory sites: 8-byte aligned guest virtual address */
    uint32_t target;  /* FI_T_* */
    uint32_t trial;   /* trial id */
} fi_site;

typedef struct {
    int32_t device;                 /* HIP device ordinal */
    uint32_t private_pages;         /* copy-on-write pages per trial (0 -> 16) */
    uint32_t hang_factor_x16;       /* hang cap = golden_ninst * f / 16 + 1000 (0 -> 32) */
    uint32_t max_trials_per_launch; /* 0 -> auto: as many as half the free device memory holds (65536 .. 2M) */
    uint32_t snapshot_interval;     /* golden snapshot every N committed insts (0 -> auto, >= 256) */
    uint32_t flags;                 /* FI_CFG_* */
    uint32_t epoch_iters;           /* first epoch's loop iterations per wave (0 -> 384; then x4, x16, unbounded) */
    uint32_t lanes_per_wave;        /* trials per 64-lane wave in the first epoch: 1, 2, 4, ..., 64 (0 -> 32) */
    uint32_t resume_lanes;          /* trials per wave in resumed epochs (0 -> default): survivors have diverged, and
                                       a wave serialises its lanes' distinct control flows, so fewer per wave */
    uint32_t epochs;                /* epochs per chunk (0 -> 2): budgets b, 4b, 16b, 16b, ..., unbounded */
} fi_config;
/* fi_config.flags: trials start from process start / run to their natural end
 * (the plain serial semantics, for A/B checks; outcomes are identical) */
#define FI_CFG_NO_SNAPSHOT_START 1u
#define FI_CFG_NO_EARLY_EXIT 2u
/* interpreter only: no load-time translation of the golden blocks (hipRTC) */
#define FI_CFG_NO_TRANSLATE 4u
/* one launch per chunk, every wave to completion (no suspend / compact / resume) */
#define FI_CFG_NO_EPOCHS 8u
/* resumed epochs pack survivors by pc run: a wave takes up to 64 consecutive
 * survivors (sorted by pc, then numInst) that stand at the same pc, instead
 * of resume_lanes survivors of any pc */
#define FI_CFG_PACK_RUNS 16u
/* resumed epochs always take resume_lanes survivors per wave (by default a
 * resumed epoch with few survivors spreads them down to one per wave, so that
 * no two diverged survivors share a wave while SIMDs idle) */
#define FI_CFG_FIXED_RESUME 32u
/* resumed epochs run on the 64-lane kernel (by default they run on the solo
 * kernel: one survivor per single-lane wave, trial state in SGPRs, low VGPR use
 * so that many waves share a SIMD) */
#define FI_CFG_NO_SOLO 64u
/* every epoch, the first included, on the solo kernel (A/B and parity checks) */
#define FI_CFG_SOLO_ALL 128u
/* diverged-lanes step loop in the 64-lane kernel: lanes at
 * different pcs each execute their own pre-decoded micro-op per step.  Off by
 * default: it trades per-trial latency for throughput, and the campaign tail
 * is latency-bound (profiles/r02d_simt_sweep.jsonl) */
#define FI_CFG_SIMT 256u
/* no first-access forwarding: a register or memory fault is
 * injected at its sampled time instead of at the golden run's next access of
 * the flipped register or bytes (A/B and parity checks; outcomes are
 * identical).  FI_CFG_NO_EARLY_EXIT implies it. */
#define FI_CFG_NO_FORWARD 512u
/* no early SDC exit: a trial whose output already differs from the golden
 * output but whose machine state equals a golden snapshot (pc, registers
 * under liveness, memory, stream positions) ends there as SDC with the golden
 * exit code and numInst -- it can only go on as the golden run does -- unless
 * this flag is set (A/B and parity checks; outcomes are identical) */
#define FI_CFG_NO_SDC_EXIT 1024u
/* no second pass for trials that ran out of copy-on-write pages: by default a
 * chunk's FI_ESC_RESOURCE trials run again with 16x the private pages (at
 * least 256) before the histogram, so that the engine's capacity does not
 * decide an outcome; one host synchronisation per chunk */
#define FI_CFG_NO_REDO 2048u
/* resumed solo epochs run every survivor on the solo kernel (by default the
 * survivors standing at an odd pc -- a pc bit-0 flip -- run on the solo-odd
 * kernel, whose translated blocks also cover the odd-pc instruction streams,
 * on a second stream beside it) (A/B and parity checks; outcomes are identical) */
#define FI_CFG_NO_ODD_KERNEL 4096u
/* Build the translated kernels even when the code-object caches (in process
 * and $SHREWD_FI_JIT_CACHE) hold them: cold-start measurements and tests of
 * the background build. */
#define FI_CFG_JIT_NO_CACHE 8192u
/* No loop proofs: neither the clean translated body's (fi_translate.cpp:
 * counted-loop hangs, run-off loops that end in a page fault or a hang,
 * fi_trial.hip loop_outcome) nor the solo interpreter's dynamic ones
 * (fi_trial.hip LoopProbe) -- every such trial runs to its cap or its
 * faulting load (A/B and parity checks; outcomes are identical: the records
 * are the same either way). */
#define FI_CFG_NO_HANG_PROOF 16384u
/* No overflow pages: by default a trial that needs more than private_pages
 * takes a block of more (up to the redo pass's 16x, at least 256, in all)
 * from a pool shared by the launch, so that it goes on at once instead of
 * ending as FI_ESC_RESOURCE and running again after the chunk (which stays
 * the fallback when the pool is spent) (A/B and parity checks; outcomes are
 * identical) */
#define FI_CFG_NO_OVERFLOW 32768u
/* The solo epoch starts its trials longest-first by the work left: the golden
 * run's remaining length, or -- for a trial inside a counted loop of the
 * golden text -- the loop's remaining passes times its length, if larger (a
 * flipped bound or pointer).  This flag drops the loop term (A/B; the order
 * never changes an outcome). */
#define FI_CFG_NO_LOOP_ORDER 65536u

typedef struct {
    uint64_t ninst, ncycles;
    uint32_t exit_code, pad;
    uint64_t stdout_len, stderr_len;
    uint64_t fetch_bytes, data_bytes;
    uint64_t snapshots, snapshot_interval; /* golden snapshots kept on the device */
    uint64_t snapshot_frames;              /* distinct 4 KiB frames behind them */
    uint64_t translated_blocks;            /* golden basic blocks compiled to straight-line code (0: interpreter only) */
    uint64_t translated_insts;
    uint64_t translate_us;                 /* translation + hipRTC build (0 if the code object was cached) */
} fi_golden_info;

typedef struct {
    uint64_t counts[FI_N_STRUCT][64][FI_N_CLASS]; /* [structure][first flipped bit][class] */
    uint64_t crash_sub[16];
    uint64_t escape_sub[8];
    uint64_t trials;
    uint64_t guest_insts;   /* sum of each trial's numInst at its end, as a serial gem5 run commits them
                               (includes the snapshot-restored prefix and a masked trial's golden suffix) */
    uint64_t fetch_bytes;   /* algorithmic bytes: instruction fetch */
    uint64_t data_bytes;    /* algorithmic bytes: loads + stores */
    uint64_t cow_pages;     /* private pages materialised (copy-on-write / zero-fill) */
    uint64_t device_insts;  /* guest instructions the device actually committed (no restored prefix, no
                               skipped suffix): the executed-instruction count behind device inst/s */
} fi_histogram;

typedef struct fi_engine fi_engine;

fi_status fi_create(const fi_config *cfg, fi_engine **out);
void fi_destroy(fi_engine *e);
const char *fi_last_error(fi_engine *e);

/* argv/envp are NULL-terminated; argv[0] is the path string gem5 was given
 * (it shapes the initial stack exactly as in RiscvProcess64::argsInit). */
fi_status fi_load_elf(fi_engine *e, const uint8_t *elf, size_t len, const char *const *argv,
                      const char *const *envp);
/* Start the campaign from a gem5 SE-mode checkpoint instead of process start
 * (Process::unserialize src/sim/process.cc:427-441,
 * m5.instantiate(ckpt_dir) src/python/m5/simulate.py:338): registers, pc,
 * memory (page table + physical memory store), brk point and stack VMA come
 * from cpt_dir/m5.cpt; the workload ELF gives the executable range for
 * pre-decode and translation.  numInst counts from the restore point (gem5
 * does not checkpoint statistics).  Restored besides: FP registers and fcsr,
 * the whole VMA list, the mmap end and curTick.  Supported: one CPU thread and
 * the process-start vector configuration; anything else is FI_E_ARG with the
 * reason in fi_last_error. */
fi_status fi_load_checkpoint(fi_engine *e, const char *cpt_dir, const uint8_t *elf, size_t len);
/* The golden run (record mode on the device), then the golden snapshots and
 * the translation of the golden basic blocks.  The translated kernels build
 * in the background (hipRTC in parallel helper processes): until they land,
 * trials run on the static kernels -- identical outcomes, bit for bit -- in
 * chunks of at most 131,072 trials, and each chunk boundary picks the build
 * up.  fi_translate_status() is "compiling" meanwhile. */
fi_status fi_golden_run(fi_engine *e, fi_golden_info *out);
/* Block until the background build has landed (or failed: see
 * fi_translate_status) and return the golden info with translated_blocks,
 * translated_insts and translate_us filled in. */
fi_status fi_wait_translation(fi_engine *e, fi_golden_info *out);
/* copies up to cap bytes of golden stdout; returns the full length in *len */
fi_status fi_golden_stdout(fi_engine *e, uint8_t *buf, uint64_t cap, uint64_t *len);
/* same for the golden run's stderr (fd 2) stream */
fi_status fi_golden_stderr(fi_engine *e, uint8_t *buf, uint64_t cap, uint64_t *len);

/* Campaign definition: SplitMix64 sites keyed by (seed, trial id); structures
 * is a bitmask (bit r = x_r, bit 32 = pc, bit 33 = memory, bit 34 = instruction
 * result); burst = adjacent
 * bits flipped (1..64). */
fi_status fi_set_campaign(fi_engine *e, uint64_t seed, uint64_t structures, uint32_t burst);
/* Eligible bit positions (SURVEY §8b `bits`): bit b set = a fault's lowest
 * flipped bit may be b (for a burst of k bits, b <= 64 - k).  Default (and
 * ~0): every position, sampled as before.  Set after fi_set_campaign. */
fi_status fi_set_bits(fi_engine *e, uint64_t bits_mask);
/* The process settings below shape the golden run as much as the trials:
 * set them after loading (or before it: they survive fi_load_elf /
 * fi_load_checkpoint) and before fi_golden_run; once a golden run exists they
 * return FI_E_STATE.
 *
 * SE time and randomness model: ticks (1 ps) per CPU cycle for clock_gettime
 * (curTick at a tick = (cycles so far - 1) x period; default 500 = 2 GHz) and
 * gem5's Random global seed for getrandom (default 5489, base/random.cc:79). */
fi_status fi_set_clock(fi_engine *e, uint64_t period_ticks, uint64_t random_seed);
/* The realpath of the workload executable, what gem5's readlinkat on
 * "/proc/self/exe" answers (realpath(Process::progName()),
 * src/sim/syscall_emul.hh:1089-1111); NULL / "" (default): that call ends the
 * trial as escape/host.  FaultCampaign sets it from `executable` (gem5's
 * Process.executable, default cmd[0]) resolved against the host working
 * directory. */
fi_status fi_set_exe_path(fi_engine *e, const char *path);
/* Process.input (src/sim/Process.py:44): data = the bytes of the input file
 * fd 0 reads (FDArray opens it O_RDONLY, src/sim/fd_array.cc:69-75; readFunc,
 * src/sim/syscall_emul.hh:2798-2822, takes min(n, left) bytes at the file
 * offset and copies n zero-padded bytes out; write/writev to fd 0 return
 * -EBADF).  Every trial starts at the golden run's offset at its start
 * snapshot; a checkpoint restart reads from offset 0, as gem5 reopens the
 * file without restoring fd 0-2 (fd_array.cc:371-380).  data = NULL (the
 * default, "cin"): fd 0 is the host's stdin and a trial that reads it ends
 * as escape/host. */
fi_status fi_set_stdin(fi_engine *e, const uint8_t *data, uint64_t len);
/* selective-replication mask over x0..x31 (bits 0..31) and pc (bit 32) */
fi_status fi_set_protect(fi_engine *e, uint64_t protect_mask);
/* SHREWD selective replication by instruction class (the reference's
 * BaseO3CPU.enableShrewd shadow issue, src/cpu/o3/inst_queue.cc:1082-1181):
 * bit k = gem5 OpClass enum value k (src/cpu/FuncUnit.py:43).  Instructions of
 * a protected class that has a shadow functional unit (FUPool::getUnit,
 * src/cpu/o3/fu_pool.cc:177-301: IntAlu, IntMult, IntDiv, FloatAdd..FloatSqrt)
 * are replicated; a result fault (FI_T_RESULT) on one is detected. */
fi_status fi_set_protect_opclasses(fi_engine *e, uint64_t opclass_mask);

/* ---- SHREWD functional-unit contention.
 *
 * In the reference a shadow copy is issued only when FUPool::getUnit(cap,
 * is_shadow=true) finds a free unit in the issue cycle
 * (src/cpu/o3/inst_queue.cc:835-1066 scheduleReadyInsts, :1082-1181
 * requestShadow; src/cpu/o3/fu_pool.cc:155-301 findFreeUnit/getUnit), either
 * before the next instruction takes its unit (BaseO3CPU.priorityToShadow) or
 * after the whole issue group (the default, "deferred").  The issue model
 * replays the golden run's committed instructions through an O3 issue stage
 * with the reference's FU pool and widths and records, per dynamic
 * instruction, whether its shadow got a unit.  With the model on, a result
 * fault (FI_T_RESULT) on a protected instruction is detected only if that
 * instruction's shadow was issued.
 *
 * What is the reference's code, restated exactly: the pool (DefaultFUPool,
 * src/cpu/o3/FUPool.py:52-66; counts, latencies and pipelining of
 * src/cpu/o3/FuncUnitConfig.py:45-198), the per-capability round-robin unit
 * queues, the shadow substitutions (IntAlu -> FloatAdd -> FloatCmp, IntMult
 * -> FloatMult, IntDiv -> FloatDiv, FloatAdd/Mult/Div/Sqrt -> IntAlu; no
 * shadow unit for memory and other classes), the unit release rules (next
 * cycle, or after op_latency for unpipelined classes; priority mode raises the
 * primary's latency to the shadow's), the age-ordered issue over ready
 * instructions with a class skipped for the rest of the cycle once it finds no
 * free unit, and issueWidth.  What is a model (no O3 pipeline runs here): the
 * schedule of ready instructions.  Cycle c: (1) units released at c are
 * freed; (2) up to commit_width oldest ops with done <= c commit; (3) issue
 * walks the IQ oldest first: an op is ready when it was dispatched before c,
 * every source register's latest older writer has done <= c, and (for a
 * serialising op) every older op has committed; done = issue + latency
 * (loads: issue + load_latency); (4) up to dispatch_width ops enter the IQ
 * and ROB in program order while both have room and no older serialising op
 * is uncommitted.  Non-memory ops leave the IQ at issue, memory ops at done.
 * Perfect branch prediction, no wrong-path work, no memory dependences. */
typedef struct {
    uint32_t issue_width;        /* BaseO3CPU.issueWidth (src/cpu/o3/BaseO3CPU.py:128): 8 */
    uint32_t dispatch_width;     /* dispatchWidth (:127): 8 */
    uint32_t commit_width;       /* commitWidth (:136): 8 */
    uint32_t iq_entries;         /* numIQEntries (:193): 64 */
    uint32_t rob_entries;        /* numROBEntries (:194): 192 */
    uint32_t load_latency;       /* model: cycles from a load's issue to its value: 2 */
    uint32_t priority_to_shadow; /* BaseO3CPU.priorityToShadow (:227): 0 */
    uint32_t fu_count[6];        /* IntALU, IntMultDiv, FP_ALU, FP_MultDiv, RdWrPort, IprPort
                                    (FuncUnitConfig.py): 6, 2, 4, 2, 4, 1 */
} fi_issue_params;

/* One dynamic instruction of the replayed trace. */
typedef struct {
    uint64_t src;      /* bit r (1..31): reads x_r; bit 32: reads the FP state */
    uint64_t dst;      /* bit r: writes x_r; bit 32: writes the FP state */
    uint8_t opclass;   /* gem5 OpClass enum value (src/cpu/FuncUnit.py:43) */
    uint8_t kind;      /* FI_ISSUE_* */
    uint8_t pad[6];
} fi_issue_op;
#define FI_ISSUE_PLAIN 0
#define FI_ISSUE_LOAD 1     /* value at issue + load_latency; holds its IQ entry until then */
#define FI_ISSUE_STORE 2    /* holds its IQ entry until done */
#define FI_ISSUE_SERIAL 3   /* ecall: issues only as the oldest op; younger ops dispatch after it commits */

/* Counters named after the reference's iqIOStats (inst_queue.cc:1082-1181). */
typedef struct {
    uint64_t ops, cycles;                  /* ops replayed; cycle at which the last one committed */
    uint64_t shadow_available, shadow_not_available;
    uint64_t shadow_same_fu, shadow_not_same_fu;
    uint64_t class_available[12];          /* per OpClass 0..11 (IntAlu..FloatSqrt at 1..11) */
    uint64_t class_not_available[12];
} fi_issue_stats;

/* Defaults listed above. */
void fi_issue_default_params(fi_issue_params *p);
/* Pure host function (no device, no engine): replay ops[0..n) and write
 * shadow[i] = 1 if op i's shadow was issued (the reference's has_shadow). */
fi_status fi_issue_model_run(const fi_issue_op *ops, uint64_t n, const fi_issue_params *p, uint8_t *shadow,
                             fi_issue_stats *stats);
/* Turn the model on for this engine's result faults (p = NULL: off, every
 * protected shadow-capable instruction is replicated, as without O3 timing).
 * Needs a golden run; computed at once from the golden trace. */
fi_status fi_set_issue_model(fi_engine *e, const fi_issue_params *p);
/* The engine's map: shadow[k] for the k-th committed golden instruction
 * (numInst index; ecalls, which numInst does not count, are left out).
 * *n = golden ninst; stats may be NULL. */
fi_status fi_shadow_map(fi_engine *e, uint8_t *shadow, uint64_t cap, uint64_t *n, fi_issue_stats *stats);

/* ---- Tick-domain injection under TimingSimpleCPU.
 *
 * The reference's own SE run script offers CPUTypes.TIMING on a NoCache board
 * (SystemXBar, width 64) with SingleChannelDDR3_1600 memory at 3 GHz
 * (tests/gem5/se_mode/hello_se/configs/simple_binary_run.py:61-64,113-126;
 * components/cachehierarchies/classic/no_cache.py;
 * components/memory/single_channel.py:45-51, dram_interfaces/ddr3.py).  Under
 * that CPU an instruction's architectural effect is the AtomicSimpleCPU one
 * (same numInst, same results) but it takes a data-dependent number of ticks:
 * TimingSimpleCPU::fetch/sendFetch/completeIfetch/completeDataAccess
 * (src/cpu/simple/timing.cc:677-1077) send one request at a time through the
 * CoherentXBar (src/mem/coherent_xbar.cc:150-507, xbar.cc:108-330) to the
 * MemCtrl (src/mem/mem_ctrl.cc) and its DRAMInterface (src/mem/
 * dram_interface.cc: banks, refresh, FR-FCFS).  The engine replays the golden
 * run's requests through a restatement of those components (an event queue
 * with gem5's same-tick LIFO order, src/sim/eventq.cc:91-158) and maps a fault
 * at tick t to the numInst injection the trial kernels already run.
 *
 * fi_timing_model_run is the model as a pure host function (no device, no
 * engine); fi_set_cpu_model(FI_CPU_TIMING) builds the golden request list
 * from the golden run and runs it; fi_run_tick_trials runs a tick-domain
 * campaign. */
typedef struct {
    uint64_t fetch[2];   /* physical address of each 4-byte instruction fetch ((pc & ~3) + fetchOffset,
                            BaseSimpleCPU::setupFetchRequest, src/cpu/simple/base.cc:304-318) */
    uint64_t addr[2];    /* physical address of each data fragment (split at a 64-byte line,
                            TimingSimpleCPU::initiateMemRead/writeMem, timing.cc:451-586) */
    uint16_t size[2];    /* fragment bytes */
    uint8_t nfetch;      /* 1, or 2 for a 32-bit instruction at pc % 4 == 2 (the decoder needs more bytes) */
    uint8_t nfrag;       /* data requests: 0 (none; also a failed SC), 1 or 2 */
    uint8_t kind;        /* FI_TOP_* */
    uint8_t cmd;         /* FI_TCMD_*: the request command of the data fragments */
    uint8_t pad[8];
} fi_timing_op;
#define FI_TOP_EXEC 0    /* executes at its completeIfetch; with data fragments it completes (commits) at the
                            completeDataAccess of the last response, else at once */
#define FI_TOP_FAULT 1   /* execute returns a fault (ecall, a page-table fault the SE fixup resolves): the next
                            fetch is the fetchEvent rescheduled at clockEdge() (timing.cc:782-797) */
#define FI_TOP_END 2     /* the exit syscall: the run ends at its execute */
#define FI_TCMD_READ 0   /* ReadReq */
#define FI_TCMD_WRITE 1  /* WriteReq */
#define FI_TCMD_SWAP 2   /* SwapReq (AMO: the memory controller's write path, a response with data) */
#define FI_TCMD_LL 3     /* LoadLockedReq (LR) */
#define FI_TCMD_SC 4     /* StoreCondReq (a successful SC) */

typedef struct {
    uint64_t fetch_send[2];   /* tick each fetch request was sent */
    uint64_t fetch_done[2];   /* tick of its completeIfetch (the CPU clock edge after the response) */
    uint64_t exec;            /* tick the instruction executes (initiateAcc for a data access) */
    uint64_t done;            /* tick it completes (completeDataAccess; == exec without data requests) */
} fi_timing_ticks;

typedef struct {
    uint64_t cpu_period;      /* CPU and crossbar clock period in ticks (1 ps): SimpleBoard clk_freq 3 GHz -> 333 */
    uint32_t xbar_frontend, xbar_forward, xbar_response, xbar_header, xbar_width, xbar_sf_lookup;
                              /* SystemXBar (src/mem/XBar.py): 3, 4, 2 cycles, header 1, NoCache width 64 B,
                                 snoop-filter lookup 1 cycle */
    uint64_t mc_frontend, mc_backend, mc_command_window;   /* MemCtrl.py: 10 ns, 10 ns, 10 ns */
    uint32_t read_buffer, write_buffer;                    /* DRAMInterface read/write_buffer_size: 32, 64 */
    uint32_t write_high_pct, write_low_pct;                /* 85, 50 */
    uint32_t min_writes_per_switch, min_reads_per_switch;  /* 16, 16 */
    uint64_t tCK, tBURST, tRCD, tCL, tRP, tRAS, tRRD, tXAW, tRFC, tWR, tWTR, tRTP, tRTW, tCS, tREFI;
                              /* DDR3_1600_8x8 (components/memory/dram_interfaces/ddr3.py) */
    uint32_t activation_limit, ranks, banks, burst_bytes, row_buffer_bytes, max_accesses_per_row;
                              /* 4, 2, 8, 64, 8 KiB (8 x 1 KiB devices), 16 */
    uint64_t mem_bytes;       /* channel capacity: 8 GiB (rows per bank) */
} fi_timing_params;

typedef struct {
    uint64_t ops, ticks;                       /* ops replayed; tick of the last op's execute (the run's end) */
    uint64_t reads, writes, write_queue_hits;  /* DRAM read / write bursts; reads the write queue serviced */
    uint64_t row_hits, activates, refreshes;
    uint64_t xbar_retries, mc_retries;         /* requests a busy crossbar layer / full controller queue refused */
} fi_timing_stats;

/* The reference board's parameters (listed above). */
void fi_timing_default_params(fi_timing_params *p);
/* Pure host function: replay ops[0..n) (the last one FI_TOP_END) through the
 * TimingSimpleCPU + SystemXBar + MemCtrl/DDR3 model; out[i] = op i's ticks. */
fi_status fi_timing_model_run(const fi_timing_op *ops, uint64_t n, const fi_timing_params *p, fi_timing_ticks *out,
                              fi_timing_stats *stats);

/* The campaign's time coordinate: FI_CPU_ATOMIC (the default: sites at a
 * numInst) or FI_CPU_TIMING (tick-domain sites, fi_run_tick_trials: the golden
 * run's requests are rebuilt and timed by fi_golden_run).  Before fi_golden_run
 * (FI_E_STATE after); p = NULL: the reference board (fi_timing_default_params). */
#define FI_CPU_ATOMIC 0
#define FI_CPU_TIMING 1
fi_status fi_set_cpu_model(fi_engine *e, int model, const fi_timing_params *p);

typedef struct {
    uint64_t golden_ticks;    /* tick of the golden run's exit (its last attempt's execute) */
    uint64_t attempts;        /* fetch-execute attempts: commits + ecalls + page-fault retries */
    fi_timing_stats stats;
    char status[160];         /* "" when tick campaigns can run, else why not (a golden run that reads curTick,
                                 unmaps memory, has a failed SC, a prefetch / cache-block / vector op; a checkpoint
                                 start; the atomic CPU model) */
} fi_tick_info;
fi_status fi_tick_golden(fi_engine *e, fi_tick_info *out);
/* The golden run's attempts as requests and their ticks (copies up to cap; *n = count). */
fi_status fi_tick_trace(fi_engine *e, fi_timing_op *ops, fi_timing_ticks *ticks, uint64_t cap, uint64_t *n);

typedef struct {
    uint64_t tick;      /* the flip happens before every event of this tick (tick < golden_ticks) */
    uint64_t mask;      /* xor mask */
    uint32_t target;    /* 1..31 = x_r, FI_T_PC, FI_T_RESULT (memory words: not in the tick domain) */
    uint32_t trial;
} fi_tick_site;
/* fi_sample_sites' SplitMix64 draw keyed by (seed, trial) with tick = mulhi(r0,
 * golden_ticks) in place of numInst (fi_set_campaign / fi_set_bits settings). */
fi_status fi_sample_tick_sites(fi_engine *e, uint64_t first_trial, uint64_t n, fi_tick_site *out);
/* The map to the kernels' numInst sites: disp[i] = 0 run sites[i]; 1 the trial
 * is the golden run (the flip does not persist: the completion of the load in
 * flight overwrites the register; a pc flip while a link-free jalr is fetched);
 * 2 escape (FI_ESC_TIMING, FI_TK_* in exit_code).  host_out (may be NULL)
 * receives the outcome of the disp 1 / 2 trials. */
fi_status fi_map_tick_sites(fi_engine *e, const fi_tick_site *ts, uint64_t n, fi_site *sites, uint8_t *disp,
                            fi_outcome *host_out);
/* A tick-domain campaign (explicit sites / sampled): map, run, classify.  The
 * histogram counts each trial under its tick site's structure and first bit.
 * Needs fi_set_protect / fi_set_protect_opclasses off. */
fi_status fi_run_tick_sites(fi_engine *e, const fi_tick_site *ts, uint64_t n, fi_outcome *out, fi_histogram *hist);
fi_status fi_run_tick_trials(fi_engine *e, uint64_t first_trial, uint64_t n, fi_outcome *out, fi_histogram *hist);

fi_status fi_sample_sites(fi_engine *e, uint64_t first_trial, uint64_t n, fi_site *out);
/* out (n entries, trial order) and hist may be NULL. hist is accumulated into (+=). */
fi_status fi_run_trials(fi_engine *e, uint64_t first_trial, uint64_t n, fi_outcome *out, fi_histogram *hist);
/* Explicit sites (parity tests, replay of a gem5-side site list). */
fi_status fi_run_sites(fi_engine *e, const fi_site *sites, uint64_t n, fi_outcome *out, fi_histogram *hist);

/* Device-resident variant for multi-GPU drivers: d_out (n fi_outcome) and
 * d_hist (one fi_histogram, accumulated) are device pointers; stream is a
 * hipStream_t (NULL = engine stream).  Asynchronous: nothing is copied back. */
fi_status fi_run_trials_device(fi_engine *e, uint64_t first_trial, uint64_t n, void *d_out, void *d_hist,
                               void *stream);
/* Synchronise the engine stream. */
fi_status fi_sync(fi_engine *e);

/* Why the translated path is off for this workload ("" when it is on). */
const char *fi_translate_status(fi_engine *e);

/* Timing of the last fi_run_* call's interpreter kernel(s), measured with
 * hipEvents on the engine stream (milliseconds). */
double fi_last_kernel_ms(fi_engine *e);
/* Accumulating per-dispatch timer of the interpreter kernel (HIP event pairs
 * recorded on the launch stream around every fi_trial_kernel dispatch: a chunk
 * is one dispatch per epoch); launches = dispatches timed. */
fi_status fi_kernel_timer_reset(fi_engine *e);
/* The effective configuration (defaults resolved). */
fi_status fi_get_config(fi_engine *e, fi_config *out);
fi_status fi_kernel_timer_read(fi_engine *e, double *total_ms, uint32_t *launches);

#ifdef __cplusplus
}
#endif
#endif
