/*
 * timing_se.h -- TEST INFRASTRUCTURE ONLY (see rv64se.h).
 *
 * The oracle's own restatement of the TimingSimpleCPU + SystemXBar + MemCtrl /
 * DDR3_1600 timing of the reference's SE board (timing_se.c).  Layouts equal
 * include/fi_engine.h's fi_timing_op / fi_timing_ticks / fi_timing_params /
 * fi_timing_stats so the tests compare the two restatements on the same input.
 */
#ifndef SHREWD_ORACLE_TIMING_SE_H
#define SHREWD_ORACLE_TIMING_SE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    uint64_t fetch[2], addr[2];
    uint16_t size[2];
    uint8_t nfetch, nfrag, kind, cmd, pad[8];
} or_timing_op_t;
enum { OR_TOP_EXEC = 0, OR_TOP_FAULT = 1, OR_TOP_END = 2 };
enum { OR_TCMD_READ = 0, OR_TCMD_WRITE = 1, OR_TCMD_SWAP = 2, OR_TCMD_LL = 3, OR_TCMD_SC = 4 };

typedef struct {
    uint64_t fetch_send[2], fetch_done[2], exec, done;
} or_timing_ticks_t;

typedef struct {
    uint64_t cpu_period;
    uint32_t xbar_frontend, xbar_forward, xbar_response, xbar_header, xbar_width, xbar_sf_lookup;
    uint64_t mc_frontend, mc_backend, mc_command_window;
    uint32_t read_buffer, write_buffer, write_high_pct, write_low_pct, min_writes_per_switch, min_reads_per_switch;
    uint64_t tCK, tBURST, tRCD, tCL, tRP, tRAS, tRRD, tXAW, tRFC, tWR, tWTR, tRTP, tRTW, tCS, tREFI;
    uint32_t activation_limit, ranks, banks, burst_bytes, row_buffer_bytes, max_accesses_per_row;
    uint64_t mem_bytes;
} or_timing_params_t;

typedef struct {
    uint64_t ops, ticks, reads, writes, write_queue_hits, row_hits, activates, refreshes, xbar_retries, mc_retries;
} or_timing_stats_t;

void or_timing_default_params(or_timing_params_t *p);
/* 0, or -1 (bad input, or a state gem5 itself asserts / panics on) */
int or_timing_model(const or_timing_op_t *ops, uint64_t n, const or_timing_params_t *p, or_timing_ticks_t *out,
                    or_timing_stats_t *stats);

#ifdef __cplusplus
}
#endif
#endif
