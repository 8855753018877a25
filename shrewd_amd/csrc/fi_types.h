// fi_types.h -- structures shared by the host engine (fi_engine.cpp) and the
// CDNA4 kernels (hip/fi_kernels.hip).  Internal; the public ABI is
// include/fi_engine.h.
#pragma once
#include "fi_rtc.h"
#include "fi_engine.h"

namespace fi {

constexpr uint64_t kPage = 4096;
constexpr uint32_t kSoloLanes = 1;   // threads of a solo-kernel workgroup (one trial; fi_trial.hip kSoloOnce)
constexpr uint32_t kDmapWords = 128;  // rewritten-code map: at most 4096 granules per slot (DevCtx::dmap)
constexpr uint64_t kFwDead = ~0ULL;  // DevCtx::eff: the flipped register is dead at injection
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
constexpr uint8_t kPreLeader = 32;   // translated code may be entered here (load-time build)
constexpr uint8_t kPreOddLeader = 64;   // ... and (solo kernel) at the odd pcs that fetch this halfword
// Separates the 64-lane, solo and solo-odd translated bodies in the generated
// text (fi_translate.cpp -> fi_jit.cpp splices them at /*@TX_BODY@*/,
// /*@TX_SOLO@*/ and /*@TX_SOLO_ODD@*/).
#define FI_TX_SPLIT "\n/*@TX_SPLIT@*/\n"

// Golden snapshot: the architectural state at the top of the first tick with
// numInst == k * snap_interval, plus the page table of the whole guest address
// space at that point (process-start pages overlaid with the golden run's
// written pages).  Trials start from the snapshot at or before their inject
// time, and a trial whose state equals a later snapshot is masked (its future
// is the golden future; deterministic machine).
struct SnapState {
    uint64_t regs[32];               // x0..x31 (x0 = 0)
    uint64_t pc, ninst, ncyc, out_pos, err_pos, stack_min;
    uint32_t tab_off, tab_n;         // entries [tab_off, tab_off + tab_n) of DevCtx::snap_tab
    uint32_t live;                   // x_r whose value here the golden future reads before writing
    uint32_t trace_pos;              // record mode: golden trace events before this snapshot
    uint64_t in_pos;                 // fd 0's file offset (Process.input a file; DevCtx::stdin_data)
};
static_assert(sizeof(SnapState) == 328, "SnapState layout");
// One mapped guest page of a snapshot: vpn -> frame in the snapshot pool.
struct PageEnt {
    uint64_t vpn;
    uint32_t frame;                  // page index into DevCtx::pool
    uint32_t pad;
};

// A suspended lane (epochs): everything a resumed lane needs
// besides its site, private pages (still in place under its slot) and the
// golden data.
struct LaneSave {
    uint64_t regs[32];
    uint64_t pc, ninst, ncyc, out_pos, err_pos, stack_min, next_chk;
    int32_t watch;
    uint32_t nfail, n_priv, snap_j;
    uint32_t flags;                  // bit 0 out_bad, bits 1-2 injected, bit 3 code_dirty, bit 4 FP state,
                                     // bit 5 VM state (VmState of the slot is live)
    uint32_t dlo, dhi;               // rewritten code bytes [code_lo + dlo, code_lo + dhi) (if code_dirty)
    uint32_t pad;                    // fflags | frm << 5
    uint64_t resv, lock;             // LR/SC: load reservation and lock record (~0 = none)
};

// A counted loop of the golden text (fi_translate.cpp, the hang proofs' loops),
// for the solo order's work-left estimate: a survivor whose pc offset from
// text_lo lies in [lo, hi) has about loop_passes(x[reg] - x[treg], step) * m
// instructions left in that loop.  Only the order of the trials uses it.
struct LoopEst {
    uint32_t lo, hi;
    uint8_t reg, treg;
    int8_t step;
    uint8_t pad;
    uint32_t m;
};
constexpr uint32_t kMaxLoopEst = 64;

// A trial's SE memory-map state once it made a VM syscall (brk, mmap, munmap,
// close, set_tid_address): gem5's MemState VMA list, brk point and mmap end
// (src/sim/mem_state.hh), the fd entries 0-2 it closed and childClearTID.
// Until then the state is the process-start one (DevCtx brk0 / svma_*).
constexpr uint32_t kMaxVma = 64;    // == oracle/rv64se.c mach_t.vma (overflow: resource escape)
constexpr uint64_t kTomb = 1ULL << 63;   // priv_vpn entry: the page is unmapped for this trial
struct VmState {
    uint64_t brk, mmap_end, ctid;
    uint64_t rnd_pos;                // getrandom bytes drawn so far (index into DevCtx::rnd_tab)
    uint32_t nvma, fdc;
    uint64_t vma[kMaxVma][2];
};

// One data access of the golden run (record mode): bytes [addr, addr + len)
// read (kind 1), written (2) or read then written (3, an AMO) by the
// instruction (or syscall) at numInst == t.
struct MemEv {
    uint64_t addr;
    uint32_t t;                      // numInst | kMemEvProxy for an access of a syscall (not a CPU request)
    uint32_t len_kind;               // len (< 2^30) | kind << 30
};
constexpr uint32_t kMemEvProxy = 0x80000000u;

// First-access forwarding (fi_forward_kernel): the golden run's register
// accesses (always) and its memory accesses (when complete and the golden
// run's mappings never change: no VM syscalls), with the snapshot page tables
// to check that a memory site is mapped at its sampled time.
struct FwdCtx {
    const uint32_t *reg_off, *reg_ev;    // per register x1..x31: (2 * numInst + !ecall) << 1 | reads
    uint32_t mw_n;                       // 0: no memory forwarding
    const uint64_t *mw_addr;
    const uint32_t *mw_off;
    const uint64_t *mw_ev;
    const SnapState *snaps;
    const PageEnt *snap_tab;
    uint32_t n_snap;
    uint64_t snap_interval;
    uint64_t text_lo, text_hi;
};

// Everything one launch of the trial kernel needs.  Passed by value as the
// kernel argument (lives in the kernarg segment -> scalar loads).
constexpr int kNStats = 64;          // DevCtx::stats entries

struct DevCtx {
    // golden text, pre-decoded (pre_ok = 0 if the golden run rewrote its text)
    const PreInst *pre;
    uint64_t text_lo, text_hi;       // page-aligned executable range
    uint64_t code_lo, code_hi;       // exact byte range of the executable segments: pre-decoded entries are valid
                                     // inside it only, and a lane's store into it makes its text "dirty"
    uint32_t pre_ok;
    uint32_t text_bytes;             // text_hi - text_lo (< 4 GiB)
    uint32_t record;                 // 1 = golden run: record output (and snapshots) instead of comparing
    // snapshots: [0] is the process-start state (SE process image)
    const SnapState *snaps;
    const PageEnt *snap_tab;
    const uint8_t *pool;             // snapshot frames, 4 KiB each
    const uint8_t *zero_page;
    uint64_t snap_interval;          // I: snapshot k is at numInst == k * I
    uint32_t n_snap;
    uint32_t early_exit;             // compare with snapshots after the injection (bit 1: also with wrong output)
    uint32_t hang_proof;             // the clean translated body may prove hangs (counted loops)
    // golden reference output (or record buffers in golden mode)
    const uint8_t *gout, *gerr;
    uint64_t gout_len, gerr_len;
    uint8_t *rec_out, *rec_err;
    uint64_t rec_cap;
    uint32_t gexit, gdetail;         // golden exit code and final pc (low 32 bits)
    uint32_t gsub, gpad_;            // golden end sub-code: FI_END_EXIT / FI_END_M5_EXIT / FI_END_M5_FAIL
    uint64_t gninst;                 // golden numInst at exit
    uint32_t priv_pages;             // P
    uint32_t snap_start;             // 1 = a wave starts at the snapshot before its earliest inject time
    uint64_t hang_cap;
    uint64_t protect_mask;
    uint64_t protect_opc;            // SHREWD replication: protected gem5 OpClass values (bit mask)
    const uint64_t *eff;             // first-access forwarding: effective inject time per trial (in site order;
                                     // kFwDead = dead at injection), nullptr = the sampled times
    const uint32_t *shadow_bits;     // FU contention model: bit k = the k-th golden instruction's shadow issued
                                     // (nullptr: every shadow-capable instruction has one)
    // per-trial private (copy-on-write) pages: frames [slot][P][4096], vpns [P][n]
    uint8_t *priv_frames;
    uint64_t *priv_vpn;
    // overflow pages: a trial that needs more than P takes one block of
    // ov_pages more from a shared pool (ov_next: blocks handed out in this
    // pass; ov_of[slot]: its block, ~0 none); ov_blocks 0 = no pool
    uint8_t *ov_frames;              // [ov_blocks][ov_pages][4096]
    uint64_t *ov_vpn;                // [ov_blocks][ov_pages]
    uint32_t *ov_of;                 // [n_slots]
    uint32_t *ov_next;
    uint32_t ov_blocks, ov_pages;
    uint8_t *tx_sink;                // translated code: stores of lanes outside the running group land here
    uint64_t *fregs;                 // FP registers [32][n_slots] (written only by a lane's FP data-movement ops)
    // record mode: snapshot capture at numInst == k * rec_interval
    SnapState *rec_snaps;            // [rec_max_snaps]
    uint8_t *rec_pages;              // [rec_max_snaps][priv_pages][4096]
    uint64_t *rec_vpns;              // [rec_max_snaps][priv_pages]
    uint64_t rec_interval;
    uint32_t rec_max_snaps;
    uint32_t rec_trace_cap;          // entries of rec_trace
    uint32_t *rec_trace;             // halfword index (pc - text_lo) / 2 of every committed instruction and
                                     // ecall of the golden run, for the host's register liveness pass
    // epochs: a wave suspends its live lanes after wave_budget loop iterations
    // (0 = run to completion); a resume launch takes its lanes from resume[]
    uint32_t wave_budget;
    uint32_t n_slots;                // slots of the chunk (stride of priv_vpn)
    uint32_t lanes;                  // trials per wave (lanes >= this are idle): 8, 16, 32 or 64
    uint32_t resume_waves;           // resume: spread the survivors over this many waves when they
                                     // need fewer than `lanes` per wave (power-of-two lanes per wave,
                                     // >= 1); 0 = always `lanes` per wave
    const uint32_t *resume;          // NULL = fresh launch: lane slot = global lane index
    const uint32_t *resume_n;        // number of entries in resume[]
    const uint32_t *resume_lo;       // solo-odd launch: its entries are resume[*resume_lo .. *resume_n) (else NULL)
    unsigned long long *span;        // this dispatch's [min wave start, max wave end] (s_memrealtime, 100 MHz)
                                     // over the waves that ran a trial; NULL = not recorded
    const uint32_t *wrange;          // packed resume (FI_CFG_PACK_RUNS): wave b runs resume[wrange[2b] .. wrange[2b+1])
    const uint32_t *n_waves;         //   number of valid wrange pairs (waves b >= it exit at once)
    uint32_t *surv;                  // suspended lanes' slots are appended here
    uint32_t *surv_n;
    LaneSave *save;                  // [n_slots]
    // the work
    const fi_site *sites;            // in trial order
    const uint32_t *perm;            // launch slot -> index into sites/out (sorted by site.inst)
    fi_outcome *out;
    uint64_t n;                      // trials in this launch
    uint64_t *wave_dbg;              // per wave: {s_memtime cycles, loop iterations, translated insts, slow fetches,
                                     //            s_memrealtime at start, at end, lane 0's trial, its instructions,
                                     //            translated entries, lane 0's full page lookups}
    // SE memory map: process-start brk and "stack" VMA; per-slot VM state
    uint64_t brk0, svma_lo, svma_hi;
    VmState *vm;                     // [n_slots]
    const uint8_t *rnd_tab;          // getrandom's byte stream: mt19937_64(seed)() % 255, rnd_len bytes
    uint64_t rnd_len;
    const uint8_t *exe_path;         // realpath of the executable (readlinkat /proc/self/exe), exe_len bytes
    uint64_t exe_len;                // 0: unknown (that call escapes as host)
    uint64_t clk_period;             // ticks per CPU cycle (clock_gettime)
    uint32_t clk_esc;                // tick-domain trials (fi_run_tick_trials): a curTick read (clock_gettime,
                                     // rpns) ends the trial as FI_ESC_TIMING / FI_TK_CLOCK -- the engine's
                                     // clock is AtomicSimpleCPU's, not TimingSimpleCPU's
    uint32_t clk_esc_pad;
    uint64_t tick0;                  // curTick at the campaign start (a checkpoint's [Globals] curTick; else 0)
    const uint8_t *stdin_data;       // Process.input as a file: its bytes (NULL: "cin", reads of fd 0 escape)
    uint64_t stdin_len;
    uint64_t *in_pos;                // per slot: fd 0's file offset (used only with stdin_data)
    uint64_t clk_until;              // the golden run reads curTick (clock_gettime, rpns) at numInst < clk_until:
                                     // before that a trial equals a snapshot only with the same ncyc (0 = never)
    const uint64_t *fp0;             // a checkpoint's FP registers (NULL: none -- zero, no FP state)
    uint32_t fcsr0;                  //   and its fflags | frm << 5
    const VmState *vm0;              // a checkpoint's SE memory map (NULL: the process-start one, brk0 / svma_*)
    uint32_t *dmap;                  // per slot: rewritten-code granules of [code_lo, code_hi), dmap_words u32 each
    uint32_t dmap_words, dmap_shift; //   (granule = 2^dmap_shift bytes); NULL: the bounding range only
    uint32_t simt_min;               // diverged-lanes step loop: least lanes to enter it (0 = off)
    // memory liveness: record mode appends the golden run's data accesses to
    // rec_mem; trials look a memory fault's word up in the per-word index built
    // from them (fi_engine.cpp:build_mem_index)
    MemEv *rec_mem;
    uint32_t rec_mem_cap;
    uint32_t mem_live;               // 1 = the index below is complete: dead memory faults end at injection
    uint32_t mw_n;                   // words in the index
    const uint64_t *mw_addr;         // [mw_n] sorted 8-byte-aligned addresses the golden run accesses
    const uint32_t *mw_off;          // [mw_n + 1] each word's events in mw_ev
    const uint64_t *mw_ev;           // per word in time order: numInst << 16 | bytes read << 8 | bytes written
    unsigned long long *stats;     // [0] fetch B [1] data B [2] pages [3..5] golden ncycles/out/err
                                     // [6] loop iterations [7] lane-insts [8] slow fetches [9] min-PC [10] max iter/wave
                                     // [11] early-exit checks [12] early exits [13] snapshots captured [14] start-inst sum
                                     // [15] golden trace events [16] translated insts [17] translated entries
                                     // [18] slowest wave: iters<<32 | tx permille<<20 | entries [19] iters<<32 | slow
                                     // [20] wave-0 s_memtime delta [21] s_memrealtime delta
                                     // [22] golden run holds state outside the snapshots (FP, LR/SC, VM)
                                     // [23] instructions executed on the device
                                     // [24] lane-instructions of the diverged-lanes step loop
                                     // [25] golden data-access events [26] memory faults ended at injection
                                     // [27] register faults dead at injection [30] trials re-run with more private
                                     // pages (FI_ESC_RESOURCE, fi_engine.cpp run_chunk)
                                     // [52] record mode: 1 + numInst of the golden run's last curTick read
                                     // [62] record mode: the golden run unmapped memory (munmap, brk shrink)
                                     // [53] solo_fast_run calls [54] instructions they ran [55] hand-backs
                                     // [56] hangs proved by the clean body's counted-loop test
                                     // [57] page-fault crashes proved in run-off loops [58] loop proofs undecided
                                     // [32..39] FI_PROF phase cycles
                                     // [40 + 4k + {0,1,2,3}] fetch B, data B, pages, device insts of kernel k
                                     // (0 the 64-lane kernel, 1 solo, 2 solo-odd)
};

struct SampleCtx {
    uint64_t seed, structures, golden_ninst, first;
    uint32_t burst, n_struct;
    uint64_t bits;                   // eligible lowest-bit positions (already limited to 0..64-burst)
    const uint64_t *mem_pages;
    uint64_t n_mem_pages;
};

}  // namespace fi
