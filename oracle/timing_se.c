/*
 * timing_se.c -- TEST INFRASTRUCTURE ONLY (see rv64se.h).
 *
 * Second, independent restatement of the gem5 timing that a TimingSimpleCPU
 * run on the reference's SE board sees (tests/gem5/se_mode/hello_se/configs/
 * simple_binary_run.py: NoCache -> SystemXBar(width=64), SingleChannelDDR3_1600,
 * 3 GHz), written directly from the reference sources as a plain event loop:
 * a flat array of pending events searched for the earliest (tick, newest
 * insertion) -- gem5 services same-tick, same-priority events last-in first-out
 * (src/sim/eventq.cc:91-158: insertBefore pushes onto the bin's stack).
 *
 * Parity status: not run against a live gem5.opt (unbuildable here, SURVEY.md
 * §8c); checked against the product model (shrewd_amd/csrc/fi_timing.cpp) and
 * against hand-derived ticks (tests/test_timing.py).
 *
 * Sources restated, function by function:
 *   TimingSimpleCPU   src/cpu/simple/timing.cc:677-1206
 *   CoherentXBar      src/mem/coherent_xbar.cc:150-507, xbar.cc:108-330,
 *                     snoop_filter.cc:66-90, XBar.py (SystemXBar)
 *   PacketQueue       src/mem/packet_queue.cc:104-205
 *   MemCtrl           src/mem/mem_ctrl.cc:188-1149, MemCtrl.py
 *   DRAMInterface     src/mem/dram_interface.cc:59-1764 (powerdown disabled,
 *                     DRAMInterface.py:71), ddr3.py DDR3_1600_8x8
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "timing_se.h"

typedef uint64_t tick_t;
#define NEVER (~(tick_t)0)
#define NO_ROW 0xFFFFFFFFu

/* ------------------------------------------------------------ event list */
enum {
    E_CPU_FETCH, E_CPU_ITICK, E_CPU_DTICK, E_CPU_DRETRY,
    E_XB_REQ_FREE, E_XB_RESP_FREE_I, E_XB_RESP_FREE_D,
    E_Q_MEM, E_Q_ICACHE, E_Q_DCACHE,
    E_MC_NEXT, E_MC_RESP,
    E_RANK /* + 5 x rank: write-done, activate, precharge, refresh, power */
};
enum { RK_WDONE, RK_ACT, RK_PRE, RK_REF, RK_PWR, RK_NEV };

typedef struct { int live; tick_t at; uint64_t order; } ev_t;

typedef struct {
    tick_t now;
    uint64_t order;
    int nev;
    ev_t *ev;
    int fail;
} evq_t;

static void ev_set(evq_t *q, int e, tick_t at) {
    if (q->ev[e].live || at < q->now) { q->fail = 1; return; }
    q->ev[e].live = 1; q->ev[e].at = at; q->ev[e].order = ++q->order;
}
static void ev_move(evq_t *q, int e, tick_t at) {   /* reschedule: a fresh insertion */
    q->ev[e].live = 0;
    ev_set(q, e, at);
}
/* earliest tick; within it the latest insertion */
static int ev_next(evq_t *q) {
    int best = -1;
    for (int e = 0; e < q->nev; e++) {
        if (!q->ev[e].live) continue;
        if (best < 0 || q->ev[e].at < q->ev[best].at ||
            (q->ev[e].at == q->ev[best].at && q->ev[e].order > q->ev[best].order)) best = e;
    }
    if (best >= 0) { q->now = q->ev[best].at; q->ev[best].live = 0; }
    return best;
}

/* -------------------------------------------------------------- packets */
typedef struct {
    uint64_t addr; uint32_t size; int cmd; int is_resp; int cpu_port; int frag;
    tick_t hdr, pay;
} req_t;

static int rq_writes(const req_t *r) { return r->cmd == OR_TCMD_WRITE || r->cmd == OR_TCMD_SWAP || r->cmd == OR_TCMD_SC; }
static int rq_reads(const req_t *r) { return r->cmd == OR_TCMD_READ || r->cmd == OR_TCMD_LL || r->cmd == OR_TCMD_SWAP; }
static int rq_data(const req_t *r) { return r->is_resp ? rq_reads(r) : rq_writes(r); }

typedef struct {   /* MemPacket */
    req_t *r; uint64_t addr; uint32_t size; int rd;
    int rank, bank; uint64_t row; tick_t ready;
} mp_t;

typedef struct { uint32_t row; tick_t rd_ok, wr_ok, pre_ok, act_ok; uint32_t accesses; } bank_t;

enum { P_IDLE, P_ACT, P_REF };
enum { RF_IDLE, RF_DRAIN, RF_PDEXIT, RF_PRE, RF_START, RF_RUN };

typedef struct {
    int pwr, pwr_next, ref;
    tick_t due;
    int outst, rd_ent, wr_ent, nactive;
    bank_t bk[32];
    tick_t act_hist[16];   /* [0] newest .. [limit-1] oldest */
} rank_t;

/* crossbar layer */
typedef struct { int st; int wait[8]; int nwait; int peer; int ev; } lay_t;
enum { L_IDLE, L_BUSY, L_RETRY };

/* packet queue (sorted by send tick) */
typedef struct { tick_t at[8]; req_t *r[8]; int n; int retry_wait; int in_order; int ev; } pq_t;

typedef struct {
    const or_timing_params_t *p;
    const or_timing_op_t *op; uint64_t nop; or_timing_ticks_t *out; or_timing_stats_t st;
    evq_t q;
    /* cpu */
    uint64_t cur; uint32_t fidx; req_t *ipend, *dpend, *itick_r, *dtick_r; req_t *frag[2]; int nout, split; int done;
    /* crossbar */
    lay_t lreq, lresp[2];
    /* queues: 0 memory controller -> xbar, 1 xbar -> icache, 2 xbar -> dcache */
    pq_t pq[3];
    /* memory controller */
    mp_t *rdq[64]; int nrd; mp_t *wrq[256]; int nwr; mp_t *resq[64]; int nres;
    int rd_retry, wr_retry; int bus_rd, bus_rd_next; tick_t nburst, nreq; uint32_t rds, wrs;
    uint64_t qrd, qwr;   /* totalRead/WriteQueueSize */
    tick_t *cmdwin; int ncmd, capcmd;
    uint32_t hi_thr, lo_thr; uint64_t rows;
    /* dram */
    rank_t rk[64]; int act_rank;
    /* allocations */
    req_t *reqs; uint64_t nreqs, capreqs; mp_t *mps; uint64_t nmps, capmps;
} sim_t;

static tick_t edge_of(const sim_t *s, uint64_t k) {
    tick_t per = s->p->cpu_period;
    return (s->q.now + per - 1) / per * per + k * per;
}
static int rk_ev(int r, int k) { return E_RANK + RK_NEV * r + k; }

static req_t *req_new(sim_t *s) {
    if (s->nreqs == s->capreqs) {   /* grow by chunks; pointers of older chunks stay valid */
        s->q.fail = 1; return NULL;
    }
    req_t *r = &s->reqs[s->nreqs++];
    memset(r, 0, sizeof *r);
    return r;
}

/* forward declarations */
static int xb_request(sim_t *s, req_t *r, int from);
static void mc_retry_to_xbar(sim_t *s);

/* ============================================================ CPU side
 * TimingSimpleCPU (timing.cc).  Each op = one fetch-execute attempt. */
static void cpu_send_fetch(sim_t *s) {   /* fetch(); sendFetch() after SE translation */
    req_t *r = req_new(s);
    if (!r) return;
    r->addr = s->op[s->cur].fetch[s->fidx]; r->size = 4; r->cmd = OR_TCMD_READ; r->cpu_port = 0;
    s->out[s->cur].fetch_send[s->fidx] = s->q.now;
    if (!xb_request(s, r, 0)) s->ipend = r;   /* IcacheRetry */
}
static void cpu_advance(sim_t *s) {
    s->cur++; s->fidx = 0;
    if (s->cur >= s->nop) s->q.fail = 1;
}
static int cpu_dsend(sim_t *s, req_t *r) {   /* handleReadPacket / handleWritePacket */
    if (xb_request(s, r, 1)) { s->dpend = NULL; return 1; }
    s->dpend = r;
    return 0;
}
static void cpu_complete_ifetch(sim_t *s) {
    const or_timing_op_t *o = &s->op[s->cur];
    s->itick_r = NULL;
    s->out[s->cur].fetch_done[s->fidx] = s->q.now;
    if (s->fidx + 1 < o->nfetch) { s->fidx++; cpu_send_fetch(s); return; }   /* stayAtPC: more bytes */
    s->out[s->cur].exec = s->q.now;
    if (o->kind == OR_TOP_END) { s->out[s->cur].done = s->q.now; s->done = 1; return; }
    if (o->kind == OR_TOP_FAULT) {   /* advanceInst(fault): reschedule(fetchEvent, clockEdge(), true) */
        s->out[s->cur].done = s->q.now;
        cpu_advance(s);
        ev_move(&s->q, E_CPU_FETCH, edge_of(s, 0));
        return;
    }
    if (!o->nfrag) { s->out[s->cur].done = s->q.now; cpu_advance(s); cpu_send_fetch(s); return; }
    s->split = o->nfrag == 2; s->nout = o->nfrag;
    for (int k = 0; k < o->nfrag; k++) {
        req_t *r = req_new(s);
        if (!r) return;
        r->addr = o->addr[k]; r->size = o->size[k]; r->cmd = o->cmd; r->cpu_port = 1; r->frag = k;
        s->frag[k] = r;
    }
    /* sendData / sendSplitData: fragment 0, then (if it went) fragment 1 */
    if (cpu_dsend(s, s->frag[0])) {
        s->frag[0] = NULL;
        if (s->split && cpu_dsend(s, s->frag[1])) s->frag[1] = NULL;
    }
}
static void cpu_icache_retry(sim_t *s) {
    if (xb_request(s, s->ipend, 0)) s->ipend = NULL;
}
static void cpu_dcache_retry(sim_t *s) {   /* DcachePort::recvReqRetry */
    req_t *r = s->dpend;
    if (!s->split) { if (xb_request(s, r, 1)) s->dpend = NULL; return; }
    if (!xb_request(s, r, 1)) return;
    s->frag[r->frag] = NULL;
    int pend = s->frag[0] ? 0 : (s->frag[1] ? 1 : -1);
    if (pend > 0) {
        s->dpend = s->frag[pend];
        if (cpu_dsend(s, s->frag[pend])) s->frag[pend] = NULL;
    } else {
        s->dpend = NULL;
    }
}
static int cpu_dresp(sim_t *s, req_t *r) {   /* DcachePort::recvTimingResp */
    if (!s->q.ev[E_CPU_DTICK].live) { s->dtick_r = r; ev_set(&s->q, E_CPU_DTICK, edge_of(s, 0)); return 1; }
    if (!s->q.ev[E_CPU_DRETRY].live) ev_set(&s->q, E_CPU_DRETRY, edge_of(s, 1));
    return 0;
}
static void cpu_iresp(sim_t *s, req_t *r) {   /* IcachePort::recvTimingResp */
    if (s->q.ev[E_CPU_ITICK].live) { s->q.fail = 1; return; }
    s->itick_r = r;
    ev_set(&s->q, E_CPU_ITICK, edge_of(s, 0));
}
static void cpu_complete_data(sim_t *s) {
    s->dtick_r = NULL;
    if (s->split) { s->nout--; if (s->nout) return; }
    s->out[s->cur].done = s->q.now;
    cpu_advance(s);
    cpu_send_fetch(s);
}

/* ======================================================== packet queues */
static void pq_arm(sim_t *s, pq_t *Q, tick_t at) {   /* schedSendEvent */
    if (Q->retry_wait || at == NEVER) return;
    if (at < s->q.now + 1) at = s->q.now + 1;
    if (!s->q.ev[Q->ev].live) ev_set(&s->q, Q->ev, at);
    else if (at < s->q.ev[Q->ev].at) ev_move(&s->q, Q->ev, at);
}
static void pq_push(sim_t *s, pq_t *Q, req_t *r, tick_t at) {   /* schedSendTiming */
    if (Q->n == 8) { s->q.fail = 1; return; }
    int k = Q->n;
    while (k > 0) {
        if ((Q->in_order && Q->r[k - 1]->addr == r->addr) || Q->at[k - 1] <= at) break;
        k--;
    }
    for (int m = Q->n; m > k; m--) { Q->at[m] = Q->at[m - 1]; Q->r[m] = Q->r[m - 1]; }
    Q->at[k] = at; Q->r[k] = r; Q->n++;
    if (k == 0) pq_arm(s, Q, at);
}
static int xb_response(sim_t *s, req_t *r);
static void pq_fire(sim_t *s, int qi) {   /* sendDeferredPacket */
    pq_t *Q = &s->pq[qi];
    tick_t at = Q->at[0]; req_t *r = Q->r[0];
    for (int m = 1; m < Q->n; m++) { Q->at[m - 1] = Q->at[m]; Q->r[m - 1] = Q->r[m]; }
    Q->n--;
    int ok;
    if (qi == 0) ok = xb_response(s, r);
    else if (qi == 1) { cpu_iresp(s, r); ok = 1; }
    else ok = cpu_dresp(s, r);
    Q->retry_wait = !ok;
    if (ok) {
        pq_arm(s, Q, Q->n ? Q->at[0] : NEVER);
    } else {
        for (int m = Q->n; m > 0; m--) { Q->at[m] = Q->at[m - 1]; Q->r[m] = Q->r[m - 1]; }
        Q->at[0] = at; Q->r[0] = r; Q->n++;
    }
}
static void pq_retry(sim_t *s, int qi) { s->pq[qi].retry_wait = 0; pq_fire(s, qi); }

/* ============================================================ crossbar */
static void lay_hold(sim_t *s, lay_t *L, tick_t until) { ev_set(&s->q, L->ev, until); }
static int lay_try(lay_t *L, int who) {
    if (L->st == L_BUSY || L->peer >= 0) { L->wait[L->nwait++] = who; return 0; }
    L->st = L_BUSY;
    return 1;
}
static void lay_retry_next(sim_t *s, lay_t *L, int is_req) {
    L->st = L_RETRY;
    int who = L->wait[0];
    for (int m = 1; m < L->nwait; m++) L->wait[m - 1] = L->wait[m];
    L->nwait--;
    if (is_req) { if (who == 0) cpu_icache_retry(s); else cpu_dcache_retry(s); }
    else pq_retry(s, 0);
    if (L->st == L_RETRY) { L->st = L_BUSY; lay_hold(s, L, edge_of(s, 0)); }
}
static void lay_free(sim_t *s, lay_t *L, int is_req) {
    L->st = L_IDLE;
    if (L->nwait && L->peer < 0) lay_retry_next(s, L, is_req);
}
static void lay_peer_ready(sim_t *s, lay_t *L, int is_req) {
    for (int m = L->nwait; m > 0; m--) L->wait[m] = L->wait[m - 1];
    L->wait[0] = L->peer; L->nwait++;
    L->peer = -1;
    if (L->st == L_IDLE) lay_retry_next(s, L, is_req);
}

static void xb_timing(sim_t *s, req_t *r, tick_t lat) {   /* calcPacketTiming */
    r->hdr += (edge_of(s, 0) - s->q.now) + lat;
    if (rq_data(r)) {
        tick_t w = (tick_t)((r->size + s->p->xbar_width - 1) / s->p->xbar_width) * s->p->cpu_period;
        if (w > r->pay) r->pay = w;
    }
}
static int mc_accept(sim_t *s, req_t *r);
static int xb_request(sim_t *s, req_t *r, int from) {   /* CoherentXBar::recvTimingReq */
    if (!lay_try(&s->lreq, from)) { s->st.xbar_retries++; return 0; }
    tick_t h0 = r->hdr;
    xb_timing(s, r, (tick_t)(s->p->xbar_frontend + s->p->xbar_forward) * s->p->cpu_period);
    tick_t busy_until = edge_of(s, s->p->xbar_header) + r->pay;
    r->hdr += (tick_t)s->p->xbar_sf_lookup * s->p->cpu_period;
    if (!mc_accept(s, r)) {
        r->hdr = h0;
        s->lreq.peer = from;
        lay_hold(s, &s->lreq, edge_of(s, 1));
        s->st.mc_retries++;
        return 0;
    }
    lay_hold(s, &s->lreq, busy_until);
    return 1;
}
static int xb_response(sim_t *s, req_t *r) {   /* CoherentXBar::recvTimingResp */
    lay_t *L = &s->lresp[r->cpu_port];
    if (!lay_try(L, 0)) { s->st.xbar_retries++; return 0; }
    xb_timing(s, r, (tick_t)s->p->xbar_response * s->p->cpu_period);
    tick_t busy_until = edge_of(s, s->p->xbar_header) + r->pay;
    tick_t lat = r->hdr;
    r->hdr = 0;
    pq_push(s, &s->pq[1 + r->cpu_port], r, s->q.now + lat);
    lay_hold(s, L, busy_until);
    return 1;
}

/* ==================================================== memory controller */
static void dram_respond(sim_t *s, int rank);
static void dram_check_refresh(sim_t *s, int rank);
static int dram_all_busy(sim_t *s);
static void dram_access(sim_t *s, mp_t *m, tick_t *cmd_at, tick_t *next_burst);

static mp_t *mp_decode(sim_t *s, req_t *r, uint64_t addr, uint32_t size, int rd) {   /* RoRaBaCoCh */
    if (s->nmps == s->capmps) { s->q.fail = 1; return NULL; }
    mp_t *m = &s->mps[s->nmps++];
    const or_timing_params_t *p = s->p;
    uint64_t a = addr / p->burst_bytes;
    a /= (p->row_buffer_bytes / p->burst_bytes);
    m->bank = (int)(a % p->banks); a /= p->banks;
    m->rank = (int)(a % p->ranks); a /= p->ranks;
    m->row = a % s->rows;
    m->r = r; m->addr = addr; m->size = size; m->rd = rd; m->ready = NEVER;
    return m;
}
static void mc_respond_to(sim_t *s, req_t *r, tick_t lat) {   /* accessAndRespond */
    r->is_resp = 1;
    tick_t when = s->q.now + lat + r->hdr + r->pay;
    r->hdr = 0; r->pay = 0;
    pq_push(s, &s->pq[0], r, when);
}
static int mc_accept(sim_t *s, req_t *r) {   /* MemCtrl::recvTimingReq */
    const or_timing_params_t *p = s->p;
    uint32_t off = (uint32_t)(r->addr & (p->burst_bytes - 1));
    uint32_t count = (off + r->size + p->burst_bytes - 1) / p->burst_bytes;
    if (count != 1) { s->q.fail = 1; return 1; }
    uint64_t balign = r->addr & ~(uint64_t)(p->burst_bytes - 1);
    if (rq_writes(r)) {
        if (s->qwr + count > p->write_buffer) { s->wr_retry = 1; return 0; }
        int merged = 0;
        for (int k = 0; k < s->nwr; k++)
            if ((s->wrq[k]->addr & ~(uint64_t)(p->burst_bytes - 1)) == balign) merged = 1;
        if (!merged) {
            mp_t *m = mp_decode(s, r, r->addr, r->size, 0);
            if (!m) return 1;
            s->rk[m->rank].wr_ent++;
            s->wrq[s->nwr++] = m;
            s->qwr++;
        }
        mc_respond_to(s, r, p->mc_frontend);
        if (!s->q.ev[E_MC_NEXT].live) ev_set(&s->q, E_MC_NEXT, s->q.now);
        return 1;
    }
    if (s->qrd + (uint64_t)s->nres + count > p->read_buffer) { s->rd_retry = 1; return 0; }
    /* serviced by the write queue: a queued write to this burst (isInWriteQueue)
       whose first range holds the whole read */
    int queued = 0;
    for (int k = 0; k < s->nwr; k++)
        if ((s->wrq[k]->addr & ~(uint64_t)(p->burst_bytes - 1)) == balign) queued = 1;
    if (queued)
        for (int k = 0; k < s->nwr; k++) {
            mp_t *w = s->wrq[k];
            if (w->addr <= r->addr && r->addr + r->size <= w->addr + w->size) {
                s->st.write_queue_hits++;
                mc_respond_to(s, r, p->mc_frontend);
                return 1;
            }
        }
    mp_t *m = mp_decode(s, r, r->addr, r->size, 1);
    if (!m) return 1;
    s->rk[m->rank].rd_ent++;
    s->rdq[s->nrd++] = m;
    s->qrd++;
    if (!s->q.ev[E_MC_NEXT].live) ev_set(&s->q, E_MC_NEXT, s->q.now);
    return 1;
}
static void mc_retry_to_xbar(sim_t *s) { lay_peer_ready(s, &s->lreq, 1); }

static void mc_respond_event(sim_t *s) {   /* processRespondEvent */
    mp_t *m = s->resq[0];
    dram_respond(s, m->rank);
    mc_respond_to(s, m->r, s->p->mc_frontend + s->p->mc_backend);
    for (int k = 1; k < s->nres; k++) s->resq[k - 1] = s->resq[k];
    s->nres--;
    if (s->nres) ev_set(&s->q, E_MC_RESP, s->resq[0]->ready);
    else dram_check_refresh(s, m->rank);
    if (s->rd_retry) { s->rd_retry = 0; mc_retry_to_xbar(s); }
}

/* command-bus slots: a multiset of window start ticks */
static void win_prune(sim_t *s) {
    int k = 0;
    for (int m = 0; m < s->ncmd; m++) if (!(s->q.now > s->cmdwin[m])) s->cmdwin[k++] = s->cmdwin[m];
    s->ncmd = k;
}
static int win_count(const sim_t *s, tick_t w) {
    int c = 0;
    for (int m = 0; m < s->ncmd; m++) c += s->cmdwin[m] == w;
    return c;
}
static tick_t win_take(sim_t *s, tick_t t) {   /* verifySingleCmd */
    tick_t W = s->p->mc_command_window, at = t, w = t - t % W;
    uint64_t maxc = s->p->mc_command_window / s->p->tCK;
    while ((uint64_t)win_count(s, w) >= maxc) { w += W; at = w; }
    if (s->ncmd == s->capcmd) { s->q.fail = 1; return at; }
    s->cmdwin[s->ncmd++] = w;
    return at;
}

/* minBankPrep + chooseNextFRFCFS over one queue; returns index or -1 */
static int mc_pick(sim_t *s, mp_t **Q, int n, tick_t extra) {
    const or_timing_params_t *p = s->p;
    if (n == 0) return -1;
    if (n == 1) return s->rk[Q[0]->rank].ref == RF_IDLE ? 0 : -1;
    tick_t min_col = s->nburst + extra;
    if (min_col < s->q.now) min_col = s->q.now;
    int pick = -1, have_mask = 0, hidden = 0, hit_hidden = 0, prepped = 0, earliest = 0;
    uint32_t mask[64];
    for (int i = 0; i < n; i++) {
        mp_t *m = Q[i];
        rank_t *R = &s->rk[m->rank];
        bank_t *B = &R->bk[m->bank];
        tick_t col_ok = m->rd ? B->rd_ok : B->wr_ok;
        if (R->ref != RF_IDLE) continue;
        if (B->row == m->row) {
            if (col_ok <= min_col) { pick = i; break; }
            if (!hit_hidden && !prepped) { pick = i; prepped = 1; }
            continue;
        }
        if (earliest) continue;
        if (!have_mask) {
            /* minBankPrep */
            int waiting[2048];
            memset(waiting, 0, sizeof(int) * p->ranks * p->banks);
            for (int k = 0; k < n; k++)
                if (s->rk[Q[k]->rank].ref == RF_IDLE) waiting[Q[k]->rank * p->banks + Q[k]->bank] = 1;
            tick_t min_act = NEVER;
            int seamless = 0;
            for (uint32_t r = 0; r < p->ranks; r++) mask[r] = 0;
            for (uint32_t r = 0; r < p->ranks; r++)
                for (uint32_t b = 0; b < p->banks; b++) {
                    if (!waiting[r * p->banks + b]) continue;
                    bank_t *X = &s->rk[r].bk[b];
                    tick_t act_at;
                    if (X->row == NO_ROW) act_at = X->act_ok > s->q.now ? X->act_ok : s->q.now;
                    else act_at = (X->pre_ok > s->q.now ? X->pre_ok : s->q.now) + p->tRP;
                    tick_t hid_max = min_col >= p->tRCD ? min_col - p->tRCD : 0;
                    if (hid_max < s->q.now) hid_max = s->q.now;
                    tick_t c = s->bus_rd ? X->rd_ok : X->wr_ok;
                    if (c < act_at + p->tRCD) c = act_at + p->tRCD;
                    int new_seam = c <= min_col;
                    if (new_seam || (!seamless && act_at <= min_act)) {
                        if (!seamless && (new_seam || act_at < min_act))
                            for (uint32_t rr = 0; rr < p->ranks; rr++) mask[rr] = 0;
                        seamless |= new_seam;
                        hidden = act_at <= hid_max;
                        mask[r] |= 1u << b;
                        min_act = act_at;
                    }
                }
            have_mask = 1;
        }
        if ((mask[m->rank] >> m->bank) & 1) {
            earliest = 1;
            hit_hidden = hidden;
            if (hidden || !prepped) pick = i;
        }
    }
    return pick;
}

static void mc_next_event(sim_t *s) {   /* processNextReqEvent */
    const or_timing_params_t *p = s->p;
    int turned = s->bus_rd != s->bus_rd_next;
    if (turned) { if (s->bus_rd) s->rds = 0; else s->wrs = 0; }
    s->bus_rd = s->bus_rd_next;
    if (dram_all_busy(s)) return;
    if (s->bus_rd) {
        int go_write = 0;
        if (s->nrd == 0) {
            if (s->nwr != 0 && (uint32_t)s->nwr > s->lo_thr) go_write = 1;
            else return;
        } else {
            tick_t gap = turned ? (p->tWTR < p->tCS ? p->tWTR : p->tCS) : 0;
            int i = mc_pick(s, s->rdq, s->nrd, gap);
            if (i < 0) return;
            mp_t *m = s->rdq[i];
            tick_t cmd_at;
            win_prune(s);
            dram_access(s, m, &cmd_at, &s->nburst);
            s->nreq = s->nburst - (p->tRP + p->tRCD);
            s->rds++;
            s->qrd--;
            if (s->nres == 0) ev_set(&s->q, E_MC_RESP, m->ready);
            s->resq[s->nres++] = m;
            /* (the interface's readQueueSize drops before the switch check; the
               entry leaves the queue after it) */
            if ((uint32_t)s->nwr > s->hi_thr && (s->rds >= p->min_reads_per_switch || s->nrd - 1 == 0)) go_write = 1;
            for (int k = i + 1; k < s->nrd; k++) s->rdq[k - 1] = s->rdq[k];
            s->nrd--;
        }
        if (go_write) s->bus_rd_next = 0;
    } else {
        tick_t gap = turned ? (p->tRTW < p->tCS ? p->tRTW : p->tCS) : 0;
        int i = mc_pick(s, s->wrq, s->nwr, gap);
        if (i < 0) return;
        mp_t *m = s->wrq[i];
        tick_t cmd_at;
        win_prune(s);
        dram_access(s, m, &cmd_at, &s->nburst);
        s->nreq = s->nburst - (p->tRP + p->tRCD);
        s->wrs++;
        s->qwr--;
        for (int k = i + 1; k < s->nwr; k++) s->wrq[k - 1] = s->wrq[k];
        s->nwr--;
        if (s->nwr == 0 || (uint32_t)s->nwr + p->min_writes_per_switch < s->lo_thr ||
            (s->nrd && s->wrs >= p->min_writes_per_switch))
            s->bus_rd_next = 1;
    }
    if (!s->q.ev[E_MC_NEXT].live) ev_set(&s->q, E_MC_NEXT, s->nreq > s->q.now ? s->nreq : s->q.now);
    if (s->wr_retry && (uint32_t)s->nwr < p->write_buffer) { s->wr_retry = 0; mc_retry_to_xbar(s); }
}

/* ================================================================= DRAM */
static void pwr_event_at(sim_t *s, int r, int state, tick_t at) {   /* schedulePowerEvent */
    if (s->q.ev[rk_ev(r, RK_PWR)].live) { s->q.fail = 1; return; }
    s->rk[r].pwr_next = state;
    ev_set(&s->q, rk_ev(r, RK_PWR), at);
}
static void bank_precharge(sim_t *s, int r, int b, tick_t at, int automatic) {
    rank_t *R = &s->rk[r];
    bank_t *B = &R->bk[b];
    const or_timing_params_t *p = s->p;
    B->row = NO_ROW;
    if (automatic) B->pre_ok = at;
    else {
        at = win_take(s, at);
        for (uint32_t k = 0; k < p->banks; k++) if (R->bk[k].pre_ok < at) R->bk[k].pre_ok = at;
    }
    tick_t fin = at + p->tRP;
    if (B->act_ok < fin) B->act_ok = fin;
    R->nactive--;
    int e = rk_ev(r, RK_PRE);
    if (!s->q.ev[e].live) { ev_set(&s->q, e, fin); R->outst++; }
    else if (s->q.ev[e].at < fin) ev_move(&s->q, e, fin);
}
static void bank_activate(sim_t *s, int r, int b, tick_t t, uint32_t row) {
    rank_t *R = &s->rk[r];
    bank_t *B = &R->bk[b];
    const or_timing_params_t *p = s->p;
    tick_t at = win_take(s, t);
    B->row = row; B->accesses = 0;
    R->nactive++;
    B->pre_ok = at + p->tRAS;
    if (B->rd_ok < at + p->tRCD) B->rd_ok = at + p->tRCD;
    if (B->wr_ok < at + p->tRCD) B->wr_ok = at + p->tRCD;
    for (uint32_t k = 0; k < p->banks; k++) if (R->bk[k].act_ok < at + p->tRRD) R->bk[k].act_ok = at + p->tRRD;
    uint32_t L = p->activation_limit;
    if (L) {
        if (R->act_hist[L - 1] && at - R->act_hist[L - 1] < p->tXAW) { s->q.fail = 1; return; }
        for (uint32_t k = L - 1; k > 0; k--) R->act_hist[k] = R->act_hist[k - 1];
        R->act_hist[0] = at;
        if (R->act_hist[L - 1] && at - R->act_hist[L - 1] < p->tXAW)
            for (uint32_t k = 0; k < p->banks; k++)
                if (R->bk[k].act_ok < R->act_hist[L - 1] + p->tXAW) R->bk[k].act_ok = R->act_hist[L - 1] + p->tXAW;
    }
    int e = rk_ev(r, RK_ACT);
    if (!s->q.ev[e].live) ev_set(&s->q, e, at);
    else if (s->q.ev[e].at > at) ev_move(&s->q, e, at);
    s->st.activates++;
}
static void dram_access(sim_t *s, mp_t *m, tick_t *cmd_at_out, tick_t *next_burst) {
    const or_timing_params_t *p = s->p;
    rank_t *R = &s->rk[m->rank];
    bank_t *B = &R->bk[m->bank];
    int hit = 1;
    if (B->row != m->row) {
        hit = 0;
        if (B->row != NO_ROW) bank_precharge(s, m->rank, m->bank, B->pre_ok > s->q.now ? B->pre_ok : s->q.now, 0);
        bank_activate(s, m->rank, m->bank, B->act_ok > s->q.now ? B->act_ok : s->q.now, (uint32_t)m->row);
    }
    tick_t at = m->rd ? B->rd_ok : B->wr_ok;
    if (at < *next_burst) at = *next_burst;
    if (at < s->q.now) at = s->q.now;
    at = win_take(s, at);
    tick_t wl = p->tCL;   /* tCWL = tCL */
    m->ready = at + (m->rd ? p->tCL : wl) + p->tBURST;
    for (uint32_t r = 0; r < p->ranks; r++)
        for (uint32_t b = 0; b < p->banks; b++) {
            tick_t to_rd, to_wr;
            if ((int)r == m->rank) {
                to_rd = m->rd ? p->tBURST : p->tBURST + p->tWTR + wl;
                to_wr = m->rd ? p->tBURST + p->tRTW : p->tBURST;
            } else {
                to_rd = to_wr = p->tBURST + p->tCS;
            }
            bank_t *X = &s->rk[r].bk[b];
            if (X->rd_ok < at + to_rd) X->rd_ok = at + to_rd;
            if (X->wr_ok < at + to_wr) X->wr_ok = at + to_wr;
        }
    s->act_rank = m->rank;
    tick_t pre = m->rd ? at + p->tRTP : m->ready + p->tWR;
    if (B->pre_ok < pre) B->pre_ok = pre;
    B->accesses++;
    int close = B->accesses == p->max_accesses_per_row;
    if (!close) {   /* open_adaptive */
        mp_t **Q = m->rd ? s->rdq : s->wrq;
        int n = m->rd ? s->nrd : s->nwr, more = 0, conflict = 0;
        for (int k = 0; k < n && !more; k++) {
            if (Q[k] == m) continue;
            int same = Q[k]->rank == m->rank && Q[k]->bank == m->bank;
            more |= same && Q[k]->row == m->row;
            conflict |= same && Q[k]->row != m->row;
        }
        close = !more && conflict;
    }
    if (close) bank_precharge(s, m->rank, m->bank, B->pre_ok > s->q.now ? B->pre_ok : s->q.now, 1);
    if (m->rd) { R->outst++; s->st.reads++; }
    else {
        int e = rk_ev(m->rank, RK_WDONE);
        if (!s->q.ev[e].live) { ev_set(&s->q, e, m->ready); R->outst++; }
        else if (s->q.ev[e].at < m->ready) ev_move(&s->q, e, m->ready);
        R->wr_ent--;
        s->st.writes++;
    }
    if (hit) s->st.row_hits++;
    *cmd_at_out = at;
    *next_burst = at + p->tBURST;
}
static int dram_all_busy(sim_t *s) {
    uint32_t busy = 0;
    for (uint32_t r = 0; r < s->p->ranks; r++) {
        rank_t *R = &s->rk[r];
        if (R->ref == RF_IDLE) continue;
        busy++;
        if (R->ref == RF_DRAIN) { R->ref = RF_PDEXIT; ev_set(&s->q, rk_ev(r, RK_REF), s->q.now); }
    }
    return busy == s->p->ranks;
}
static void dram_respond(sim_t *s, int r) { s->rk[r].rd_ent--; s->rk[r].outst--; }
static void dram_check_refresh(sim_t *s, int r) {
    if (s->rk[r].ref == RF_PRE && !s->q.ev[rk_ev(r, RK_PRE)].live) ev_set(&s->q, rk_ev(r, RK_REF), s->q.now);
}
static void rank_refresh(sim_t *s, int r) {   /* processRefreshEvent */
    rank_t *R = &s->rk[r];
    const or_timing_params_t *p = s->p;
    if (R->ref == RF_IDLE) { R->due = s->q.now; R->ref = RF_DRAIN; R->outst++; }
    if (R->ref == RF_DRAIN) {
        if (r == s->act_rank && s->q.ev[E_MC_NEXT].live) return;
        R->ref = RF_PDEXIT;
    }
    if (R->ref == RF_PDEXIT) R->ref = RF_PRE;
    if (R->ref == RF_PRE) {
        if (R->nactive) {
            tick_t at = s->q.now;
            for (uint32_t b = 0; b < p->banks; b++) if (R->bk[b].pre_ok > at) at = R->bk[b].pre_ok;
            for (uint32_t b = 0; b < p->banks; b++) {
                bank_t *B = &R->bk[b];
                if (B->row != NO_ROW) bank_precharge(s, r, (int)b, at, 1);
                else {
                    if (B->act_ok < at + p->tRP) B->act_ok = at + p->tRP;
                    if (B->pre_ok < at) B->pre_ok = at;
                }
            }
        } else if (R->pwr == P_IDLE && R->outst == 1) {
            pwr_event_at(s, r, P_REF, s->q.now);
        } else if (!s->q.ev[rk_ev(r, RK_PRE)].live && !s->q.ev[E_MC_RESP].live) {
            s->q.fail = 1;
        }
        return;
    }
    if (R->ref == RF_START) {
        tick_t fin = s->q.now + p->tRFC;
        for (uint32_t b = 0; b < p->banks; b++) R->bk[b].act_ok = fin;
        R->due += p->tREFI;
        if (R->due < fin) { s->q.fail = 1; return; }
        R->ref = RF_RUN;
        ev_set(&s->q, rk_ev(r, RK_REF), fin);
        s->st.refreshes++;
        return;
    }
    if (R->ref == RF_RUN) {
        pwr_event_at(s, r, P_IDLE, s->q.now);
        ev_set(&s->q, rk_ev(r, RK_REF), R->due - p->tRP);
    }
}
static void rank_power(sim_t *s, int r) {   /* processPowerEvent */
    rank_t *R = &s->rk[r];
    int was = R->pwr;
    R->pwr = R->pwr_next;
    if (was == P_REF) {
        R->outst--;
        R->ref = RF_IDLE;
        if (!s->q.ev[E_MC_NEXT].live) ev_set(&s->q, E_MC_NEXT, s->q.now);
    }
    if (R->pwr == P_ACT && R->ref == RF_PDEXIT) { s->q.fail = 1; return; }
    if (R->pwr == P_IDLE && (R->ref == RF_PRE || R->ref == RF_PDEXIT)) {
        if (!s->q.ev[rk_ev(r, RK_ACT)].live) {
            if (R->ref == RF_PDEXIT) { s->q.fail = 1; return; }
            R->pwr = P_REF;
        } else if (!s->q.ev[rk_ev(r, RK_PRE)].live) {
            s->q.fail = 1; return;
        }
    }
    if (R->pwr == P_REF) { ev_set(&s->q, rk_ev(r, RK_REF), s->q.now); R->ref = RF_START; }
}
static void rank_event(sim_t *s, int r, int k) {
    rank_t *R = &s->rk[r];
    if (k == RK_WDONE) R->outst--;
    else if (k == RK_ACT) { if (R->pwr != P_ACT) pwr_event_at(s, r, P_ACT, s->q.now); }
    else if (k == RK_PRE) { R->outst--; if (R->nactive == 0) pwr_event_at(s, r, P_IDLE, s->q.now); }
    else if (k == RK_REF) rank_refresh(s, r);
    else rank_power(s, r);
}

/* ================================================================ driver */
void or_timing_default_params(or_timing_params_t *p) {
    memset(p, 0, sizeof *p);
    p->cpu_period = 333;                                   /* SimpleBoard clk_freq "3GHz" */
    p->xbar_frontend = 3; p->xbar_forward = 4; p->xbar_response = 2;   /* SystemXBar */
    p->xbar_header = 1; p->xbar_width = 64; p->xbar_sf_lookup = 1;     /* NoCache: SystemXBar(width=64) */
    p->mc_frontend = 10000; p->mc_backend = 10000; p->mc_command_window = 10000;
    p->read_buffer = 32; p->write_buffer = 64; p->write_high_pct = 85; p->write_low_pct = 50;
    p->min_writes_per_switch = 16; p->min_reads_per_switch = 16;
    p->tCK = 1250; p->tBURST = 5000; p->tRCD = 13750; p->tCL = 13750; p->tRP = 13750; p->tRAS = 35000;
    p->tRRD = 6000; p->tXAW = 30000; p->tRFC = 260000; p->tWR = 15000; p->tWTR = 7500; p->tRTP = 7500;
    p->tRTW = 2500; p->tCS = 2500; p->tREFI = 7800000;
    p->activation_limit = 4; p->ranks = 2; p->banks = 8; p->burst_bytes = 64; p->row_buffer_bytes = 8192;
    p->max_accesses_per_row = 16; p->mem_bytes = 8ULL << 30;
}

int or_timing_model(const or_timing_op_t *ops, uint64_t n, const or_timing_params_t *p, or_timing_ticks_t *out,
                    or_timing_stats_t *stats) {
    if (!ops || !p || !out || !n || p->ranks > 64 || p->banks > 32 || p->activation_limit > 16 ||
        p->ranks * p->banks > 2048 || !p->cpu_period || !p->tCK || !p->mc_command_window)
        return -1;
    sim_t *s = (sim_t *)calloc(1, sizeof *s);
    if (!s) return -1;
    s->p = p; s->op = ops; s->nop = n; s->out = out;
    memset(out, 0, n * sizeof *out);
    s->q.nev = E_RANK + RK_NEV * (int)p->ranks;
    s->q.ev = (ev_t *)calloc((size_t)s->q.nev, sizeof(ev_t));
    s->capreqs = 4 * n + 16; s->reqs = (req_t *)malloc(s->capreqs * sizeof(req_t));
    s->capmps = 2 * n + 16; s->mps = (mp_t *)malloc(s->capmps * sizeof(mp_t));
    s->capcmd = 4096; s->cmdwin = (tick_t *)malloc(s->capcmd * sizeof(tick_t));
    int rc = -1;
    if (!s->q.ev || !s->reqs || !s->mps || !s->cmdwin) goto done;
    s->lreq.peer = s->lresp[0].peer = s->lresp[1].peer = -1;
    s->lreq.ev = E_XB_REQ_FREE; s->lresp[0].ev = E_XB_RESP_FREE_I; s->lresp[1].ev = E_XB_RESP_FREE_D;
    s->pq[0].ev = E_Q_MEM; s->pq[0].in_order = 1;   /* MemCtrl's response queue keeps same-address order */
    s->pq[1].ev = E_Q_ICACHE; s->pq[2].ev = E_Q_DCACHE;
    s->bus_rd = s->bus_rd_next = 1;
    s->hi_thr = (uint32_t)(p->write_buffer * p->write_high_pct / 100.0);
    s->lo_thr = (uint32_t)(p->write_buffer * p->write_low_pct / 100.0);
    {
        uint64_t cap = 1;
        while (cap < p->mem_bytes) cap <<= 1;
        s->rows = cap / ((uint64_t)p->row_buffer_bytes * p->banks * p->ranks);
    }
    for (uint32_t r = 0; r < p->ranks; r++) {
        for (uint32_t b = 0; b < p->banks; b++) s->rk[r].bk[b].row = NO_ROW;
        s->rk[r].pwr = P_IDLE; s->rk[r].ref = RF_IDLE;
    }
    for (uint64_t i = 0; i < n; i++)
        if (ops[i].nfetch < 1 || ops[i].nfetch > 2 || ops[i].nfrag > 2 || (ops[i].kind == OR_TOP_END) != (i == n - 1))
            goto done;
    /* initState: the first fetch at clockEdge(0); startup: nextBurstAt = commandOffset, refresh per rank */
    ev_set(&s->q, E_CPU_FETCH, 0);
    s->nburst = p->tRP + p->tRCD;
    for (uint32_t r = 0; r < p->ranks; r++) ev_set(&s->q, rk_ev((int)r, RK_REF), p->tREFI - p->tRP);
    while (!s->done && !s->q.fail) {
        int e = ev_next(&s->q);
        if (e < 0) break;
        switch (e) {
        case E_CPU_FETCH: cpu_send_fetch(s); break;
        case E_CPU_ITICK: cpu_complete_ifetch(s); break;
        case E_CPU_DTICK: cpu_complete_data(s); break;
        case E_CPU_DRETRY: pq_retry(s, 2); break;
        case E_XB_REQ_FREE: lay_free(s, &s->lreq, 1); break;
        case E_XB_RESP_FREE_I: lay_free(s, &s->lresp[0], 0); break;
        case E_XB_RESP_FREE_D: lay_free(s, &s->lresp[1], 0); break;
        case E_Q_MEM: pq_fire(s, 0); break;
        case E_Q_ICACHE: pq_fire(s, 1); break;
        case E_Q_DCACHE: pq_fire(s, 2); break;
        case E_MC_NEXT: mc_next_event(s); break;
        case E_MC_RESP: mc_respond_event(s); break;
        default: rank_event(s, (e - E_RANK) / RK_NEV, (e - E_RANK) % RK_NEV);
        }
    }
    if (s->done && !s->q.fail) {
        rc = 0;
        s->st.ops = n;
        s->st.ticks = out[n - 1].exec;
        if (stats) *stats = s->st;
    }
done:
    free(s->q.ev); free(s->reqs); free(s->mps); free(s->cmdwin); free(s);
    return rc;
}
