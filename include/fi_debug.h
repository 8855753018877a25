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
/* Counters of the last interpreter launch: [0] fetch bytes [1] data bytes
 * [2] private pages [3..5] golden ncycles/stdout/stderr [6] wave-loop
 * iterations [7] lane-instructions executed [8] slow-path fetches [9] min-PC
 * reductions [10] max iterations of one wave; [16..21] diagnostic builds
 * only: s_memtime cycles per loop segment. */
fi_status fi_debug_stats(fi_engine *e, uint64_t *out32);
#ifdef __cplusplus
}
#endif
#endif
