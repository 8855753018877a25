/*
 * fi_debug.h -- test hooks of libshrewd_fi.so (not part of the campaign ABI).
 */
#ifndef SHREWD_FI_DEBUG_H
#define SHREWD_FI_DEBUG_H
#include "fi_engine.h"
#ifdef __cplusplus
extern "C" {
#endif
/* Decode n raw instruction words with the device decoder (the same function
 * the interpreter's pre-decode and slow fetch path use); out receives n
 * 16-byte records {u32 raw; u8 op, rd, rs1, rs2; i32 imm; u8 len, flags; u16 aux}. */
fi_status fi_debug_decode(fi_engine *e, const uint32_t *raws, uint64_t n, void *out);
/* Counters of the last interpreter launch (layout: DevCtx::stats in
 * shrewd_amd/csrc/fi_types.h): fetch/data bytes, private pages, golden
 * cycles/output, loop iterations, lane-instructions, slow fetches, min-PC
 * reductions, snapshot comparisons and early exits, translated instructions
 * and entries, the slowest wave, wave-0 clock, per-kernel bytes; [32..39]
 * -DFI_PROF builds only.  64 entries. */
fi_status fi_debug_stats(fi_engine *e, uint64_t *out64);
/* The engine's IEEE arithmetic port (shrewd_amd/csrc/hip/fi_softfp.h) over
 * operand vectors, on the host (on_device = 0) or the device: op / fmt codes of
 * fi::sf::op; out = result bits, fl = fflags raised. */
fi_status fi_debug_softfp(int op, int fmt, int rm, const uint64_t *a, const uint64_t *b, const uint64_t *c,
                          uint64_t n, uint64_t *out, uint32_t *fl, int on_device);
/* Per wave of the last launch: {s_memtime cycles, loop iterations,
 * translated instructions, slow fetches} (4 x u64 each). */
fi_status fi_debug_waves(fi_engine *e, uint64_t *out, uint64_t n_waves);
/* Device time of each interpreter dispatch since fi_kernel_timer_reset, in
 * launch order (epochs of each chunk); *n = dispatches (at most cap written). */
fi_status fi_debug_dispatch_ms(fi_engine *e, float *ms, uint32_t cap, uint32_t *n);
/* Device busy span of each of those dispatches (ms): from the first to the
 * last s_memrealtime stamp of the waves that ran a trial -- the dispatch's own
 * work, without the time its waves waited for CU slots held by the other
 * stream's kernel (0: no trial ran).  Needs fi_kernel_timer_reset first. */
fi_status fi_debug_dispatch_span_ms(fi_engine *e, float *ms, uint32_t cap, uint32_t *n);
/* The kernel of each of those dispatches: 0 fi_trial_kernel_tx (64 lanes; the
 * static fi_trial_kernel without a load-time build), 1 the solo kernel, 2 the
 * solo-odd kernel (odd-pc survivors, on a second stream beside the solo one). */
fi_status fi_debug_dispatch_kinds(fi_engine *e, uint32_t *kinds, uint32_t cap, uint32_t *n);
/* Lanes suspended at the end of each epoch of the last chunk (16 x u32). */
fi_status fi_debug_epochs(fi_engine *e, uint32_t *out16);
/* The translator's inputs of the last fi_golden_run: the pre-decoded text
 * (16-byte records, see fi_debug_decode) and the golden trace (halfword index
 * per committed instruction or ecall, bit 31 = ecall). */
fi_status fi_debug_golden_trace(fi_engine *e, void *pre_out, uint64_t pre_cap, uint64_t *n_pre, uint32_t *trace_out,
                                uint64_t trace_cap, uint64_t *n_trace, uint64_t *text_lo);
/* Run the translator on given inputs (no device): the generated C++. */
fi_status fi_debug_translate(const void *pre, uint64_t n_pre, uint64_t text_lo, const uint32_t *trace,
                             uint64_t n_trace, char *out, uint64_t cap, uint64_t *len);
/* The translator's counted loops on given inputs (no device): the solo
 * order's work-left estimates (fi_types.h LoopEst: text span lo, hi as
 * offsets from text_lo, counter reg, compared treg, step, instructions per
 * pass m; 16 bytes each).  *n = their number, out gets up to cap of them. */
fi_status fi_debug_loop_est(const void *pre, uint64_t n_pre, uint64_t text_lo, const uint32_t *trace,
                            uint64_t n_trace, void *out, uint64_t cap, uint64_t *n);
/* The C++ generated for the golden blocks by the last fi_golden_run
 * (fi_translate.cpp); *len = its length, buf gets up to cap-1 bytes + NUL. */
fi_status fi_debug_translation(fi_engine *e, char *buf, uint64_t cap, uint64_t *len);
/* hipRTC build of the trial kernel with `body` as its translated blocks, no
 * device needed; code (cap bytes) receives the code object, *len its size,
 * err the hipRTC log on failure. */
fi_status fi_debug_jit_compile(const char *body, const char *arch, void *code, uint64_t cap, uint64_t *len,
                               char *err, uint64_t err_cap);
/* One part (1 = the 64-lane kernel, 2 solo, 3 solo-odd) of the load-time
 * build as an engine runs it, with the disk cache on (use_cache) or in
 * FI_CFG_JIT_NO_CACHE mode: ranks of one node that need the same code object
 * queue on a lock next to its cache file and one of them builds it.  No
 * device needed; *len the code object's size, *cached 1 when it was loaded. */
fi_status fi_debug_jit_build(const char *body, const char *arch, int part, int use_cache, uint64_t *len,
                             int *cached, char *err, uint64_t err_cap);

/* A run-off loop as the translated solo body reports it (SoloTxIO lp_*,
 * fi_translate.cpp): counter | compared register << 8 | (int8) step << 16,
 * instructions per iteration, loads, per load {reg | kind << 8 | size << 12 |
 * position << 16, offset, span}; the registers at the loop's first
 * instruction and `left`, the instructions to the hang cap (64-bit). */
typedef struct {
    uint64_t regs[32];
    uint64_t left;
    uint32_t lp_cnt, lp_m, lp_n;
    uint32_t lp_ld[4][3];
    uint32_t pad;
} fi_debug_loop;
typedef struct {
    int32_t verdict;      /* loop_outcome: 0 undecided, 1 hang, 2 page-fault crash after k instructions at fva */
    uint32_t body_proof;  /* the body's own proof against left capped at 2^32 - 1 (tx_hang_proof) */
    uint64_t k, fva;
} fi_debug_loop_out;
/* loop_outcome (fi_trial.hip) on device, for each record, against the
 * process-start page set of the loaded workload (after fi_golden_run) --
 * the function the solo kernel calls whenever the body claims a hang. */
fi_status fi_debug_loop_outcome(fi_engine *e, const fi_debug_loop *in, uint64_t n, fi_debug_loop_out *out);
#ifdef __cplusplus
}
#endif
#endif
