// The golden run's timing under TimingSimpleCPU on the reference run script's
// board (include/fi_engine.h, "Tick-domain injection"): one request at a time
// from the CPU through the SystemXBar to the MemCtrl and its DDR3 DRAM
// interface.  Host code, run once per golden run; a discrete-event replay of
// the golden request list with gem5's event order (same tick and priority:
// the most recently scheduled event first, src/sim/eventq.cc:91-158 -- every
// event here has Default_Pri).
//
// Reference (what each part restates):
//   CPU    src/cpu/simple/timing.cc: fetch 677-715, sendFetch 719-749,
//          advanceInst 753-815, completeIfetch 819-898, IcachePort::
//          recvTimingResp 907-926, completeDataAccess 943-1077, DcachePort::
//          recvTimingResp / recvReqRetry 1138-1206, sendData / sendSplitData /
//          handleRead/WritePacket 262-393, 503-522; SE translation is
//          synchronous (src/arch/riscv/tlb.cc:573-604).
//   XBar   src/mem/coherent_xbar.cc:150-420 (recvTimingReq), 447-507
//          (recvTimingResp); src/mem/xbar.cc:108-330 (calcPacketTiming, the
//          layer state machine); snoop filter: a CPU port's request returns no
//          snoop targets and lookup_latency cycles (src/mem/snoop_filter.cc:
//          66-90); SystemXBar latencies src/mem/XBar.py.
//   Queues src/mem/packet_queue.cc:104-205 (sorted transmit list, a send event
//          no earlier than the next tick, retry).
//   MemCtrl src/mem/mem_ctrl.cc: addToReadQueue 188-301 (write-queue
//          forwarding), addToWriteQueue 303-379 (merging, early response),
//          recvTimingReq 406-485, processRespondEvent 487-554, chooseNext
//          556-619, accessAndRespond 621-659, command-bus windows 661-703,
//          doBurstAccess 795-835, processNextReqEvent 880-1149.
//   DRAM   src/mem/dram_interface.cc: chooseNextFRFCFS 59-172, activateBank
//          174-281, prechargeBank 283-344, doBurstAccess 346-617, isBusy
//          796-832, decodePacket 834-918 (RoRaBaCoCh), respondEvent 930-975,
//          checkRefreshState 977-988, minBankPrep 1027-1116, the rank's refresh
//          and power state machines 1156-1764 with enable_dram_powerdown =
//          False (src/mem/DRAMInterface.py:71): a rank is only ever IDLE, ACT or
//          REF, and no low-power path is reachable.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <deque>
#include <map>
#include <set>
#include <stdexcept>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "fi_engine.h"

namespace {

using Tick = uint64_t;
constexpr Tick kMaxTick = ~0ULL;
constexpr uint32_t kNoRow = 0xFFFFFFFFu;

// ---- event queue: (when, newest first) -------------------------------------
enum Ev : int {
    EV_FETCH, EV_ITICK, EV_DTICK, EV_DRETRY,          // TimingSimpleCPU
    EV_XREQ_REL, EV_XRESP_REL0, EV_XRESP_REL1,        // crossbar layers (memory port; icache / dcache ports)
    EV_PQ_MC, EV_PQ_X0, EV_PQ_X1,                     // packet-queue send events (memory controller; xbar)
    EV_NEXTREQ, EV_RESPOND,                           // MemCtrl
    EV_RANK0                                          // + 5 per rank: write done, activate, precharge, refresh, power
};
enum RankEv : int { R_WRDONE, R_ACT, R_PRE, R_REF, R_PWR, R_N };

struct Queue {
    struct E { bool on = false; Tick when = 0; uint64_t seq = 0; };
    std::vector<E> ev;
    std::set<std::tuple<Tick, uint64_t, int>> q;   // (when, ~seq, id): the newest of a tick first
    uint64_t seq = 0;
    Tick now = 0;
    explicit Queue(int n) : ev(n) {}
    bool on(int id) const { return ev[id].on; }
    Tick when(int id) const { return ev[id].when; }
    void schedule(int id, Tick t) {
        if (ev[id].on || t < now) throw std::logic_error("event scheduled twice or in the past");
        ev[id] = {true, t, ++seq};
        q.insert({t, ~ev[id].seq, id});
    }
    void deschedule(int id) {
        q.erase({ev[id].when, ~ev[id].seq, id});
        ev[id].on = false;
    }
    void reschedule(int id, Tick t) {   // EventQueue::reschedule: remove, then insert anew
        if (ev[id].on) deschedule(id);
        schedule(id, t);
    }
    bool pop(int &id) {
        if (q.empty()) return false;
        auto it = q.begin();
        now = std::get<0>(*it);
        id = std::get<2>(*it);
        q.erase(it);
        ev[id].on = false;
        return true;
    }
};

// ---- packets ---------------------------------------------------------------
struct Pkt {
    uint64_t addr = 0;
    uint32_t size = 0;
    uint8_t cmd = 0;          // FI_TCMD_*
    bool resp = false;        // turned into a response
    int port = 0;             // crossbar CPU-side port: 0 icache, 1 dcache
    int frag = 0;
    Tick header = 0, payload = 0;
};
bool is_write(const Pkt &p) { return p.cmd == FI_TCMD_WRITE || p.cmd == FI_TCMD_SWAP || p.cmd == FI_TCMD_SC; }
bool is_read(const Pkt &p) { return p.cmd == FI_TCMD_READ || p.cmd == FI_TCMD_LL || p.cmd == FI_TCMD_SWAP; }
// Packet::hasData: a write request carries data, a read response does
bool has_data(const Pkt &p) { return p.resp ? is_read(p) : is_write(p); }

// one DRAM burst (MemPacket)
struct Burst {
    Pkt *pkt;
    uint64_t addr;
    uint32_t size;
    bool read;
    int rank, bank, bank_id;
    uint64_t row;
    Tick ready = kMaxTick;
};

struct Bank {
    uint32_t open_row = kNoRow;
    Tick rd_allowed = 0, wr_allowed = 0, pre_allowed = 0, act_allowed = 0;
    uint32_t row_accesses = 0;
};

enum Pwr { PWR_IDLE, PWR_REF, PWR_ACT };
enum Ref { REF_IDLE, REF_DRAIN, REF_PD_EXIT, REF_PRE, REF_START, REF_RUN };

struct Rank {
    Pwr pwr = PWR_IDLE, pwr_trans = PWR_IDLE;
    Ref ref = REF_IDLE;
    Tick ref_due = 0;
    int outstanding = 0;
    int read_entries = 0, write_entries = 0;
    int banks_active = 0;
    std::vector<Bank> banks;
    std::deque<Tick> act_ticks;   // newest first
    Tick last_burst = 0;
};

// crossbar layer (BaseXBar::Layer)
struct Layer {
    enum { IDLE, BUSY, RETRY } state = IDLE;
    std::deque<int> waiting;   // ports waiting for the layer
    int peer = -1;             // port whose packet the destination refused (waitingForPeer)
    int release_ev;
};

// packet queue (PacketQueue / QueuedResponsePort)
struct PQueue {
    std::deque<std::pair<Tick, Pkt *>> list;
    bool waiting_retry = false;
    bool force_order = false;   // never pass a queued packet to the same address (the MemCtrl's port)
    int ev;
};

class Model {
  public:
    Model(const fi_timing_params &p, const fi_timing_op *ops, uint64_t n, fi_timing_ticks *out)
        : P(p), ops_(ops), n_(n), out_(out), q_(EV_RANK0 + R_N * (int)p.ranks) {
        ranks_.resize(P.ranks);
        for (auto &r : ranks_) {
            r.banks.resize(P.banks);
            r.act_ticks.assign(P.activation_limit, 0);
        }
        xreq_.release_ev = EV_XREQ_REL;
        xresp_[0].release_ev = EV_XRESP_REL0;
        xresp_[1].release_ev = EV_XRESP_REL1;
        pq_mc_.ev = EV_PQ_MC;
        pq_mc_.force_order = true;   // MemCtrl::MemoryPort (mem_ctrl.cc:1478-1481)
        pq_x_[0].ev = EV_PQ_X0;
        pq_x_[1].ev = EV_PQ_X1;
        bursts_per_row_ = P.row_buffer_bytes / P.burst_bytes;
        uint64_t cap = 1;
        while (cap < P.mem_bytes) cap <<= 1;
        rows_per_bank_ = cap / ((uint64_t)P.row_buffer_bytes * P.banks * P.ranks);
        write_high_ = (uint32_t)(P.write_buffer * P.write_high_pct / 100.0);
        write_low_ = (uint32_t)(P.write_buffer * P.write_low_pct / 100.0);
        max_cmds_ = P.mc_command_window / P.tCK;
        tWL_ = P.tCL;   // tCWL defaults to tCL (DRAMInterface.py)
    }

    fi_timing_stats run() {
        // initState: activateContext schedules the first fetch at clockEdge(0)
        q_.schedule(EV_FETCH, 0);
        // startup(): MemCtrl (mem_ctrl.cc:109-122), then the ranks' first refresh
        // (dram_interface.cc:783-794, 1156-1166) in rank order
        next_burst_at_ = P.tRP + P.tRCD;   // commandOffset(): tRP + max(tRCD_RD, tRCD_WR)
        for (uint32_t r = 0; r < P.ranks; r++) q_.schedule(rank_ev(r, R_REF), P.tREFI - P.tRP);
        int id;
        while (!end_ && q_.pop(id)) dispatch(id);
        if (!end_) throw std::logic_error("event queue drained before the last op");
        st_.ops = n_;
        st_.ticks = out_[n_ - 1].exec;
        return st_;
    }

  private:
    const fi_timing_params P;
    const fi_timing_op *ops_;
    uint64_t n_;
    fi_timing_ticks *out_;
    Queue q_;
    fi_timing_stats st_{};
    bool end_ = false;
    std::deque<Pkt> pool_;

    Tick now() const { return q_.now; }
    int rank_ev(int r, int k) const { return EV_RANK0 + R_N * r + k; }
    // ClockedObject::clockEdge (CPU and crossbar share the board's clock domain)
    Tick edge(uint64_t cycles = 0) const {
        const Tick T = P.cpu_period;
        return (now() + T - 1) / T * T + cycles * T;
    }

    // ======================================================= TimingSimpleCPU
    uint64_t j_ = 0;             // current op
    uint32_t f_ = 0;             // its fetch index
    Pkt *itick_pkt_ = nullptr, *dtick_pkt_ = nullptr;
    Pkt *ifetch_retry_ = nullptr;  // ifetch_pkt waiting for a retry
    Pkt *dcache_pkt_ = nullptr;    // dcache_pkt waiting for a retry
    Pkt *frag_[2] = {nullptr, nullptr};   // SplitMainSenderState::fragments (not yet sent)
    int outstanding_ = 0;
    bool split_ = false;

    Pkt *new_pkt() { pool_.emplace_back(); return &pool_.back(); }

    void fetch() {   // fetch() + sendFetch(): SE translation finishes at once
        const fi_timing_op &op = ops_[j_];
        Pkt *p = new_pkt();
        p->addr = op.fetch[f_];
        p->size = 4;
        p->cmd = FI_TCMD_READ;
        p->port = 0;
        out_[j_].fetch_send[f_] = now();
        if (!xbar_req(p, 0)) ifetch_retry_ = p;   // IcacheRetry
    }
    void icache_resp(Pkt *p) {
        if (q_.on(EV_ITICK)) throw std::logic_error("two icache responses in one cycle");
        itick_pkt_ = p;
        q_.schedule(EV_ITICK, edge());
    }
    void next_op() {
        j_++;
        f_ = 0;
        if (j_ >= n_) throw std::logic_error("ran past the last op");
    }
    void complete_ifetch() {
        itick_pkt_ = nullptr;
        const fi_timing_op &op = ops_[j_];
        out_[j_].fetch_done[f_] = now();
        if (f_ + 1 < op.nfetch) {   // decoder needs more bytes: stayAtPC, advanceInst -> fetch()
            f_++;
            fetch();
            return;
        }
        out_[j_].exec = now();
        if (op.kind == FI_TOP_END) {
            out_[j_].done = now();
            end_ = true;
            return;
        }
        if (op.kind == FI_TOP_FAULT) {   // advanceInst(fault): the fetch event at clockEdge()
            out_[j_].done = now();
            next_op();
            q_.reschedule(EV_FETCH, edge());
            return;
        }
        if (op.nfrag == 0) {   // executes (or a failed SC completes inside sendData) and commits
            out_[j_].done = now();
            next_op();
            fetch();
            return;
        }
        // initiateAcc -> translation (synchronous) -> sendData / sendSplitData
        split_ = op.nfrag == 2;
        outstanding_ = op.nfrag;
        for (int k = 0; k < op.nfrag; k++) {
            Pkt *p = new_pkt();
            p->addr = op.addr[k];
            p->size = op.size[k];
            p->cmd = op.cmd;
            p->port = 1;
            p->frag = k;
            frag_[k] = p;
        }
        if (!dcache_send(frag_[0])) return;   // handleRead/WritePacket failed: DcacheRetry on fragment 0
        frag_[0] = nullptr;
        if (split_ && dcache_send(frag_[1])) frag_[1] = nullptr;
    }
    bool dcache_send(Pkt *p) {
        if (xbar_req(p, 1)) { dcache_pkt_ = nullptr; return true; }
        dcache_pkt_ = p;
        return false;
    }
    void dcache_retry() {   // DcachePort::recvReqRetry
        Pkt *p = dcache_pkt_;
        if (!split_) {
            if (xbar_req(p, 1)) dcache_pkt_ = nullptr;
            return;
        }
        if (!xbar_req(p, 1)) return;
        frag_[p->frag] = nullptr;
        const int other = frag_[0] ? 0 : frag_[1] ? 1 : -1;   // getPendingFragment
        if (other > 0) {
            dcache_pkt_ = frag_[other];
            if (dcache_send(frag_[other])) frag_[other] = nullptr;
        } else {
            dcache_pkt_ = nullptr;
        }
    }
    bool dcache_resp(Pkt *p) {   // DcachePort::recvTimingResp
        if (!q_.on(EV_DTICK)) {
            dtick_pkt_ = p;
            q_.schedule(EV_DTICK, edge());
            return true;
        }
        if (!q_.on(EV_DRETRY)) q_.schedule(EV_DRETRY, edge(1));
        return false;
    }
    void complete_data() {
        dtick_pkt_ = nullptr;
        if (split_ && --outstanding_) return;   // the other fragment is still outstanding
        out_[j_].done = now();
        next_op();
        fetch();   // completeAcc, countInst, advanceInst -> fetch()
    }
    void icache_retry() {   // IcachePort::recvReqRetry
        Pkt *p = ifetch_retry_;
        if (xbar_req(p, 0)) ifetch_retry_ = nullptr;
    }

    // ============================================================ crossbar
    Layer xreq_, xresp_[2];
    std::unordered_map<Pkt *, int> route_;

    void calc_timing(Pkt *p, Tick header_delay) {   // BaseXBar::calcPacketTiming
        p->header += (edge() - now()) + header_delay;
        if (has_data(*p))
            p->payload = std::max<Tick>(p->payload, (p->size + P.xbar_width - 1) / P.xbar_width * P.cpu_period);
    }
    bool layer_try(Layer &L, int src) {
        if (L.state == Layer::BUSY || L.peer != -1) {
            L.waiting.push_back(src);
            return false;
        }
        L.state = Layer::BUSY;
        return true;
    }
    void layer_occupy(Layer &L, Tick until) { q_.schedule(L.release_ev, until); }
    void layer_release(Layer &L, bool req_layer) {
        L.state = Layer::IDLE;
        if (!L.waiting.empty() && L.peer == -1) layer_retry_waiting(L, req_layer);
    }
    void layer_retry_waiting(Layer &L, bool req_layer) {
        L.state = Layer::RETRY;
        const int src = L.waiting.front();
        L.waiting.pop_front();
        if (req_layer) {   // sendRetryReq to a CPU port
            if (src == 0) icache_retry(); else dcache_retry();
        } else {           // sendRetryResp to the memory controller's port
            pq_retry(pq_mc_);
        }
        if (L.state == Layer::RETRY) {
            L.state = Layer::BUSY;
            layer_occupy(L, edge());
        }
    }
    void layer_recv_retry(Layer &L, bool req_layer) {   // the peer is ready again
        L.waiting.push_front(L.peer);
        L.peer = -1;
        if (L.state == Layer::IDLE) layer_retry_waiting(L, req_layer);
    }
    bool xbar_req(Pkt *p, int src) {   // CoherentXBar::recvTimingReq
        if (!layer_try(xreq_, src)) { st_.xbar_retries++; return false; }
        const Tick old_header = p->header;
        calc_timing(p, (Tick)(P.xbar_frontend + P.xbar_forward) * P.cpu_period);
        const Tick finish = edge(P.xbar_header) + p->payload;
        p->header += (Tick)P.xbar_sf_lookup * P.cpu_period;   // snoop filter: no snoopers, lookup latency
        if (!mc_recv(p)) {
            p->header = old_header;
            xreq_.peer = src;
            layer_occupy(xreq_, edge(1));   // failedTiming
            st_.mc_retries++;
            return false;
        }
        route_[p] = src;
        layer_occupy(xreq_, finish);        // succeededTiming
        return true;
    }
    bool xbar_resp(Pkt *p) {   // CoherentXBar::recvTimingResp
        const int dst = route_.at(p);
        if (!layer_try(xresp_[dst], 0)) { st_.xbar_retries++; return false; }
        calc_timing(p, (Tick)P.xbar_response * P.cpu_period);
        const Tick finish = edge(P.xbar_header) + p->payload;
        const Tick lat = p->header;
        p->header = 0;
        pq_sched(pq_x_[dst], p, now() + lat);
        route_.erase(p);
        layer_occupy(xresp_[dst], finish);
        return true;
    }

    // ========================================================= packet queues
    PQueue pq_mc_, pq_x_[2];

    void pq_sched(PQueue &Q, Pkt *p, Tick when) {   // PacketQueue::schedSendTiming
        for (auto it = Q.list.end(); it != Q.list.begin();) {
            --it;
            if ((Q.force_order && it->second->addr == p->addr) || it->first <= when) {
                Q.list.emplace(it + 1, when, p);
                return;
            }
        }
        Q.list.emplace_front(when, p);
        pq_sched_event(Q, when);
    }
    void pq_sched_event(PQueue &Q, Tick when) {
        if (Q.waiting_retry) return;
        if (when == kMaxTick) return;
        when = std::max(when, now() + 1);
        if (!q_.on(Q.ev)) q_.schedule(Q.ev, when);
        else if (when < q_.when(Q.ev)) q_.reschedule(Q.ev, when);
    }
    bool pq_deliver(PQueue &Q, Pkt *p) {
        if (&Q == &pq_mc_) return xbar_resp(p);
        if (&Q == &pq_x_[0]) { icache_resp(p); return true; }
        return dcache_resp(p);
    }
    void pq_send(PQueue &Q) {   // sendDeferredPacket
        auto front = Q.list.front();
        Q.list.pop_front();
        Q.waiting_retry = !pq_deliver(Q, front.second);
        if (!Q.waiting_retry) pq_sched_event(Q, Q.list.empty() ? kMaxTick : Q.list.front().first);
        else Q.list.push_front(front);
    }
    void pq_retry(PQueue &Q) {
        Q.waiting_retry = false;
        pq_send(Q);
    }

    // ======================================================== memory controller
    std::vector<Burst *> rdq_, wrq_;
    std::deque<Burst *> respq_;
    std::set<uint64_t> in_wrq_;              // isInWriteQueue (burst-aligned addresses)
    std::deque<Burst> bursts_;
    bool retry_rd_ = false, retry_wr_ = false;
    bool bus_read_ = true, bus_read_next_ = true;   // busState / busStateNext == READ
    Tick next_burst_at_ = 0, next_req_time_ = 0;
    uint32_t reads_this_time_ = 0, writes_this_time_ = 0;
    uint64_t total_rd_ = 0, total_wr_ = 0;   // qos counters (logRequest / logResponse)
    std::multiset<Tick> burst_ticks_;
    uint32_t bursts_per_row_ = 128, write_high_ = 0, write_low_ = 0;
    uint64_t rows_per_bank_ = 0;
    Tick max_cmds_ = 8, tWL_ = 0;

    uint64_t burst_align(uint64_t a) const { return a & ~(uint64_t)(P.burst_bytes - 1); }

    Burst *decode(Pkt *p, uint64_t addr, uint32_t size, bool read) {   // decodePacket, RoRaBaCoCh
        uint64_t a = addr / P.burst_bytes / bursts_per_row_;
        const int bank = (int)(a % P.banks);
        a /= P.banks;
        const int rank = (int)(a % P.ranks);
        a /= P.ranks;
        bursts_.push_back(Burst{p, addr, size, read, rank, bank, (int)(P.banks * rank + bank), a % rows_per_bank_});
        return &bursts_.back();
    }

    bool mc_recv(Pkt *p) {   // MemCtrl::recvTimingReq
        const uint32_t off = (uint32_t)(p->addr & (P.burst_bytes - 1));
        const uint32_t count = (off + p->size + P.burst_bytes - 1) / P.burst_bytes;
        if (is_write(*p)) {
            if (total_wr_ + count > P.write_buffer) { retry_wr_ = true; return false; }
            add_to_write_queue(p, count);
            if (!q_.on(EV_NEXTREQ)) q_.schedule(EV_NEXTREQ, now());
        } else {
            if (total_rd_ + respq_.size() + count > P.read_buffer) { retry_rd_ = true; return false; }
            if (!add_to_read_queue(p, count) && !q_.on(EV_NEXTREQ)) q_.schedule(EV_NEXTREQ, now());
        }
        return true;
    }
    bool add_to_read_queue(Pkt *p, uint32_t count) {
        if (count != 1) throw std::logic_error("a CPU request never spans two bursts");
        const uint64_t addr = p->addr;
        const uint32_t size = p->size;
        bool found = false;
        if (in_wrq_.count(burst_align(addr)))
            for (Burst *w : wrq_)
                if (w->addr <= addr && addr + size <= w->addr + w->size) { found = true; break; }
        if (found) {
            st_.write_queue_hits++;
            access_and_respond(p, P.mc_frontend);
            return true;
        }
        Burst *b = decode(p, addr, size, true);
        ranks_[b->rank].read_entries++;   // setupRank
        rdq_.push_back(b);
        total_rd_++;
        read_q_size_++;
        return false;
    }
    void add_to_write_queue(Pkt *p, uint32_t count) {
        if (count != 1) throw std::logic_error("a CPU request never spans two bursts");
        if (!in_wrq_.count(burst_align(p->addr))) {
            Burst *b = decode(p, p->addr, p->size, false);
            ranks_[b->rank].write_entries++;
            wrq_.push_back(b);
            in_wrq_.insert(burst_align(p->addr));
            total_wr_++;
            write_q_size_++;
        }
        access_and_respond(p, P.mc_frontend);   // early write response
    }
    void access_and_respond(Pkt *p, Tick static_latency) {
        p->resp = true;
        const Tick t = now() + static_latency + p->header + p->payload;
        p->header = p->payload = 0;
        pq_sched(pq_mc_, p, t);
    }
    void process_respond() {   // processRespondEvent
        Burst *b = respq_.front();
        dram_respond_event(b->rank);
        access_and_respond(b->pkt, P.mc_frontend + P.mc_backend);
        respq_.pop_front();
        if (!respq_.empty()) q_.schedule(EV_RESPOND, respq_.front()->ready);
        else check_refresh_state(b->rank);
        if (retry_rd_) {
            retry_rd_ = false;
            layer_recv_retry(xreq_, true);   // port.sendRetryReq -> the crossbar's memory-side port
        }
    }
    uint32_t read_q_size_ = 0, write_q_size_ = 0;   // the interface's readQueueSize / writeQueueSize

    bool rank_ready(const Burst *b) const { return ranks_[b->rank].ref == REF_IDLE; }   // burstReady

    // chooseNext: the single entry, or FR-FCFS
    int choose_next(std::vector<Burst *> &queue, Tick extra_col_delay) {
        if (queue.empty()) return -1;
        if (queue.size() == 1) return rank_ready(queue[0]) ? 0 : -1;
        const Tick min_col_at = std::max(next_burst_at_ + extra_col_delay, now());
        return choose_frfcfs(queue, min_col_at);
    }
    int choose_frfcfs(const std::vector<Burst *> &queue, Tick min_col_at) {
        std::vector<uint32_t> earliest(P.ranks, 0);
        bool filled = false, hidden_prep = false, found_hidden = false, found_prepped = false, found_earliest = false;
        int sel = -1;
        for (size_t i = 0; i < queue.size(); i++) {
            const Burst *b = queue[i];
            const Bank &bk = ranks_[b->rank].banks[b->bank];
            const Tick col_allowed = b->read ? bk.rd_allowed : bk.wr_allowed;
            if (!rank_ready(b)) continue;
            if (bk.open_row == b->row) {
                if (col_allowed <= min_col_at) { sel = (int)i; break; }   // seamless row hit
                if (!found_hidden && !found_prepped) { sel = (int)i; found_prepped = true; }
            } else if (!found_earliest) {
                if (!filled) {
                    std::tie(earliest, hidden_prep) = min_bank_prep(queue, min_col_at);
                    filled = true;
                }
                if ((earliest[b->rank] >> b->bank) & 1) {
                    found_earliest = true;
                    found_hidden = hidden_prep;
                    if (hidden_prep || !found_prepped) sel = (int)i;
                }
            }
        }
        return sel;
    }
    std::pair<std::vector<uint32_t>, bool> min_bank_prep(const std::vector<Burst *> &queue, Tick min_col_at) const {
        Tick min_act_at = kMaxTick;
        std::vector<uint32_t> mask(P.ranks, 0);
        bool found_seamless = false, hidden = false;
        std::vector<bool> waiting(P.ranks * P.banks, false);
        for (const Burst *b : queue)
            if (ranks_[b->rank].ref == REF_IDLE) waiting[b->bank_id] = true;
        for (uint32_t r = 0; r < P.ranks; r++)
            for (uint32_t k = 0; k < P.banks; k++) {
                if (!waiting[r * P.banks + k]) continue;
                const Bank &bk = ranks_[r].banks[k];
                const Tick act_at = bk.open_row == kNoRow ? std::max(bk.act_allowed, now())
                                                          : std::max(bk.pre_allowed, now()) + P.tRP;
                const Tick tRCD = P.tRCD;   // tRCD_RD == tRCD_WR
                const Tick hidden_act_max = std::max(min_col_at >= tRCD ? min_col_at - tRCD : 0, now());
                const Tick col_allowed = bus_read_ ? bk.rd_allowed : bk.wr_allowed;
                const Tick col_at = std::max(col_allowed, act_at + tRCD);
                const bool new_seamless = col_at <= min_col_at;
                if (new_seamless || (!found_seamless && act_at <= min_act_at)) {
                    if (!found_seamless && (new_seamless || act_at < min_act_at)) std::fill(mask.begin(), mask.end(), 0);
                    found_seamless |= new_seamless;
                    hidden = act_at <= hidden_act_max;
                    mask[r] |= 1u << k;
                    min_act_at = act_at;
                }
            }
        return {mask, hidden};
    }

    void prune_burst_ticks() {
        for (auto it = burst_ticks_.begin(); it != burst_ticks_.end();)
            if (now() > *it) it = burst_ticks_.erase(it); else ++it;
    }
    Tick verify_single_cmd(Tick cmd_tick) {   // one command slot per tCK in a command window
        Tick cmd_at = cmd_tick;
        Tick bt = cmd_tick - cmd_tick % P.mc_command_window;
        while (burst_ticks_.count(bt) >= max_cmds_) {
            bt += P.mc_command_window;
            cmd_at = bt;
        }
        burst_ticks_.insert(bt);
        return cmd_at;
    }

    void process_next_req() {   // processNextReqEvent
        const bool switched = bus_read_ != bus_read_next_;
        if (switched) {
            if (bus_read_) reads_this_time_ = 0; else writes_this_time_ = 0;
        }
        bus_read_ = bus_read_next_;
        if (dram_is_busy()) return;
        if (bus_read_) {
            bool to_writes = false;
            if (read_q_size_ == 0) {
                if (write_q_size_ != 0 && write_q_size_ > write_low_) to_writes = true;
                else return;   // nothing to do
            } else {
                const int i = choose_next(rdq_, switched ? std::min(P.tWTR, P.tCS) : 0);
                if (i < 0) return;   // no read to an available rank: a refresh restarts things
                Burst *b = rdq_[i];
                do_burst(b);
                read_q_size_--;
                total_rd_--;
                if (respq_.empty()) q_.schedule(EV_RESPOND, b->ready);
                respq_.push_back(b);
                if (write_q_size_ > write_high_ && (reads_this_time_ >= P.min_reads_per_switch || read_q_size_ == 0))
                    to_writes = true;
                rdq_.erase(rdq_.begin() + i);
            }
            if (to_writes) bus_read_next_ = false;
        } else {
            const int i = choose_next(wrq_, switched ? std::min(P.tRTW, P.tCS) : 0);
            if (i < 0) return;
            Burst *b = wrq_[i];
            do_burst(b);
            in_wrq_.erase(burst_align(b->addr));
            write_q_size_--;
            total_wr_--;
            wrq_.erase(wrq_.begin() + i);
            const bool below = write_q_size_ + P.min_writes_per_switch < write_low_;
            if (write_q_size_ == 0 || below || (read_q_size_ && writes_this_time_ >= P.min_writes_per_switch))
                bus_read_next_ = true;
        }
        if (!q_.on(EV_NEXTREQ)) q_.schedule(EV_NEXTREQ, std::max(next_req_time_, now()));
        if (retry_wr_ && write_q_size_ < P.write_buffer) {
            retry_wr_ = false;
            layer_recv_retry(xreq_, true);
        }
    }
    void do_burst(Burst *b) {   // MemCtrl::doBurstAccess
        prune_burst_ticks();
        Tick next;
        dram_burst(b, next);
        next_burst_at_ = next;
        next_req_time_ = next_burst_at_ - (P.tRP + P.tRCD);
        if (b->read) reads_this_time_++; else writes_this_time_++;
    }

    // ================================================================ DRAM
    std::vector<Rank> ranks_;
    int active_rank_ = 0;

    void dram_burst(Burst *b, Tick &next_burst) {   // DRAMInterface::doBurstAccess
        Rank &rk = ranks_[b->rank];
        Bank &bk = rk.banks[b->bank];
        bool row_hit = true;
        if (bk.open_row != b->row) {
            row_hit = false;
            if (bk.open_row != kNoRow) precharge(rk, b->rank, bk, std::max(bk.pre_allowed, now()), false);
            activate(rk, b->rank, bk, b->bank, std::max(bk.act_allowed, now()), (uint32_t)b->row);
        }
        const Tick col_allowed = b->read ? bk.rd_allowed : bk.wr_allowed;
        Tick cmd_at = std::max({col_allowed, next_burst_at_, now()});
        cmd_at = verify_single_cmd(cmd_at);
        const Tick gap = P.tBURST;   // tBURST_MIN == tBURST: no burst interleaving
        b->ready = cmd_at + (b->read ? P.tCL : tWL_) + P.tBURST;
        rk.last_burst = cmd_at;
        for (uint32_t r = 0; r < P.ranks; r++)
            for (uint32_t k = 0; k < P.banks; k++) {
                Tick to_rd, to_wr;
                if ((int)r == b->rank) {   // no bank groups
                    to_rd = b->read ? gap : P.tBURST + P.tWTR + tWL_;   // writeToReadDelay
                    to_wr = b->read ? P.tBURST + P.tRTW : gap;           // readToWriteDelay
                } else {
                    to_rd = to_wr = P.tBURST + P.tCS;                    // rankToRankDelay
                }
                Bank &o = ranks_[r].banks[k];
                o.rd_allowed = std::max(cmd_at + to_rd, o.rd_allowed);
                o.wr_allowed = std::max(cmd_at + to_wr, o.wr_allowed);
            }
        active_rank_ = b->rank;
        bk.pre_allowed = std::max(bk.pre_allowed, b->read ? cmd_at + P.tRTP : b->ready + P.tWR);
        bk.row_accesses++;
        bool auto_pre = bk.row_accesses == P.max_accesses_per_row;
        if (!auto_pre) {   // open_adaptive: close if no more hits and a bank conflict waits
            bool more_hits = false, conflict = false;
            for (const Burst *o : (b->read ? rdq_ : wrq_)) {
                if (o == b) continue;
                const bool same_bank = o->rank == b->rank && o->bank == b->bank;
                more_hits |= same_bank && o->row == b->row;
                conflict |= same_bank && o->row != b->row;
                if (more_hits) break;
            }
            auto_pre = !more_hits && conflict;
        }
        if (auto_pre) precharge(rk, b->rank, bk, std::max(now(), bk.pre_allowed), true);
        if (b->read) {
            rk.outstanding++;
            st_.reads++;
        } else {
            const int ev = rank_ev(b->rank, R_WRDONE);
            if (!q_.on(ev)) { q_.schedule(ev, b->ready); rk.outstanding++; }
            else if (q_.when(ev) < b->ready) q_.reschedule(ev, b->ready);
            rk.write_entries--;
            st_.writes++;
        }
        if (row_hit) st_.row_hits++;
        next_burst = cmd_at + gap;
    }
    void activate(Rank &rk, int r, Bank &bk, int bank, Tick act_tick, uint32_t row) {
        const Tick act_at = verify_single_cmd(act_tick);
        bk.open_row = row;
        bk.row_accesses = 0;
        rk.banks_active++;
        bk.pre_allowed = act_at + P.tRAS;
        bk.rd_allowed = std::max(act_at + P.tRCD, bk.rd_allowed);
        bk.wr_allowed = std::max(act_at + P.tRCD, bk.wr_allowed);
        for (auto &o : rk.banks) o.act_allowed = std::max(act_at + P.tRRD, o.act_allowed);
        if (!rk.act_ticks.empty()) {
            if (rk.act_ticks.back() && act_at - rk.act_ticks.back() < P.tXAW)
                throw std::logic_error("tXAW violated (gem5 panics)");
            rk.act_ticks.pop_back();
            rk.act_ticks.push_front(act_at);
            if (rk.act_ticks.back() && act_at - rk.act_ticks.back() < P.tXAW)
                for (auto &o : rk.banks) o.act_allowed = std::max(rk.act_ticks.back() + P.tXAW, o.act_allowed);
        }
        const int ev = rank_ev(r, R_ACT);
        if (!q_.on(ev)) q_.schedule(ev, act_at);
        else if (q_.when(ev) > act_at) q_.reschedule(ev, act_at);
        st_.activates++;
        (void)bank;
    }
    void precharge(Rank &rk, int r, Bank &bk, Tick pre_tick, bool auto_or_preall) {
        bk.open_row = kNoRow;
        Tick pre_at = pre_tick;
        if (auto_or_preall) {
            bk.pre_allowed = pre_at;
        } else {   // explicit PRE: a command slot; tPPD = 0
            pre_at = verify_single_cmd(pre_tick);
            for (auto &o : rk.banks) o.pre_allowed = std::max(pre_at, o.pre_allowed);
        }
        const Tick done = pre_at + P.tRP;
        bk.act_allowed = std::max(bk.act_allowed, done);
        rk.banks_active--;
        const int ev = rank_ev(r, R_PRE);
        if (!q_.on(ev)) { q_.schedule(ev, done); rk.outstanding++; }
        else if (q_.when(ev) < done) q_.reschedule(ev, done);
    }
    bool dram_is_busy() {   // isBusy: every rank refreshing (checkDrainDone on the way)
        uint32_t busy = 0;
        for (uint32_t r = 0; r < P.ranks; r++) {
            Rank &rk = ranks_[r];
            if (rk.ref != REF_IDLE) {
                busy++;
                if (rk.ref == REF_DRAIN) {   // checkDrainDone
                    rk.ref = REF_PD_EXIT;
                    q_.schedule(rank_ev(r, R_REF), now());
                }
            }
        }
        return busy == P.ranks;
    }
    void dram_respond_event(int r) {   // DRAMInterface::respondEvent (power-down off)
        Rank &rk = ranks_[r];
        rk.read_entries--;
        rk.outstanding--;
    }
    void check_refresh_state(int r) {
        Rank &rk = ranks_[r];
        if (rk.ref == REF_PRE && !q_.on(rank_ev(r, R_PRE))) q_.schedule(rank_ev(r, R_REF), now());
    }
    void schedule_power(int r, Pwr s, Tick t) {
        if (q_.on(rank_ev(r, R_PWR))) throw std::logic_error("two power events (gem5 panics)");
        ranks_[r].pwr_trans = s;
        q_.schedule(rank_ev(r, R_PWR), t);
    }
    void rank_event(int r, int k) {
        Rank &rk = ranks_[r];
        switch (k) {
        case R_WRDONE: rk.outstanding--; break;
        case R_ACT:
            if (rk.pwr != PWR_ACT) schedule_power(r, PWR_ACT, now());
            break;
        case R_PRE:
            rk.outstanding--;
            if (rk.banks_active == 0) schedule_power(r, PWR_IDLE, now());   // (power-down off)
            break;
        case R_REF: refresh_event(r); break;
        case R_PWR: power_event(r); break;
        }
    }
    void refresh_event(int r) {   // Rank::processRefreshEvent (power-down off)
        Rank &rk = ranks_[r];
        if (rk.ref == REF_IDLE) {
            rk.ref_due = now();
            rk.ref = REF_DRAIN;
            rk.outstanding++;
        }
        if (rk.ref == REF_DRAIN) {
            if (r == active_rank_ && q_.on(EV_NEXTREQ)) return;   // let the request loop hand back
            rk.ref = REF_PD_EXIT;
        }
        if (rk.ref == REF_PD_EXIT) rk.ref = REF_PRE;   // not in a low-power state
        if (rk.ref == REF_PRE) {
            if (rk.banks_active != 0) {   // precharge all
                Tick pre_at = now();
                for (auto &b : rk.banks) pre_at = std::max(b.pre_allowed, pre_at);
                const Tick act_allowed = pre_at + P.tRP;
                for (auto &b : rk.banks) {
                    if (b.open_row != kNoRow) {
                        precharge(rk, r, b, pre_at, true);
                    } else {
                        b.act_allowed = std::max(b.act_allowed, act_allowed);
                        b.pre_allowed = std::max(b.pre_allowed, pre_at);
                    }
                }
            } else if (rk.pwr == PWR_IDLE && rk.outstanding == 1) {
                schedule_power(r, PWR_REF, now());
            } else if (!q_.on(rank_ev(r, R_PRE)) && !q_.on(EV_RESPOND)) {
                throw std::logic_error("refresh waits for nothing (gem5 asserts)");
            }
            return;
        }
        if (rk.ref == REF_START) {
            const Tick done = now() + P.tRFC;
            for (auto &b : rk.banks) b.act_allowed = done;
            rk.ref_due += P.tREFI;
            if (rk.ref_due < done) throw std::logic_error("refresh delayed past its catch-up (gem5 fatal)");
            rk.ref = REF_RUN;
            q_.schedule(rank_ev(r, R_REF), done);
            st_.refreshes++;
            return;
        }
        if (rk.ref == REF_RUN) {
            schedule_power(r, PWR_IDLE, now());
            q_.schedule(rank_ev(r, R_REF), rk.ref_due - P.tRP);
        }
    }
    void power_event(int r) {   // Rank::processPowerEvent (power-down off)
        Rank &rk = ranks_[r];
        const Pwr prev = rk.pwr;
        rk.pwr = rk.pwr_trans;
        if (prev == PWR_REF) {
            rk.outstanding--;
            rk.ref = REF_IDLE;
            if (!q_.on(EV_NEXTREQ)) q_.schedule(EV_NEXTREQ, now());   // restartScheduler
        }
        if (rk.pwr == PWR_ACT && rk.ref == REF_PD_EXIT) {
            throw std::logic_error("active power-down exit without power-down (gem5 asserts)");
        } else if (rk.pwr == PWR_IDLE && (rk.ref == REF_PRE || rk.ref == REF_PD_EXIT)) {
            if (!q_.on(rank_ev(r, R_ACT))) {
                if (rk.ref == REF_PD_EXIT) throw std::logic_error("PD exit without power-down (gem5 asserts)");
                rk.pwr = PWR_REF;
            } else if (!q_.on(rank_ev(r, R_PRE))) {
                throw std::logic_error("idle with an activate but no precharge pending (gem5 asserts)");
            }
        }
        if (rk.pwr == PWR_REF) {
            q_.schedule(rank_ev(r, R_REF), now());
            rk.ref = REF_START;
        }
    }

    // ============================================================== dispatch
    void dispatch(int id) {
        switch (id) {
        case EV_FETCH: fetch(); break;
        case EV_ITICK: complete_ifetch(); break;
        case EV_DTICK: complete_data(); break;
        case EV_DRETRY: pq_retry(pq_x_[1]); break;   // sendRetryResp to the crossbar's dcache-side queue
        case EV_XREQ_REL: layer_release(xreq_, true); break;
        case EV_XRESP_REL0: layer_release(xresp_[0], false); break;
        case EV_XRESP_REL1: layer_release(xresp_[1], false); break;
        case EV_PQ_MC: pq_send(pq_mc_); break;
        case EV_PQ_X0: pq_send(pq_x_[0]); break;
        case EV_PQ_X1: pq_send(pq_x_[1]); break;
        case EV_NEXTREQ: process_next_req(); break;
        case EV_RESPOND: process_respond(); break;
        default: {
            const int k = id - EV_RANK0;
            rank_event(k / R_N, k % R_N);
        }
        }
    }
};

}  // namespace

extern "C" void fi_timing_default_params(fi_timing_params *p) {
    if (!p) return;
    *p = fi_timing_params{};
    p->cpu_period = 333;
    p->xbar_frontend = 3; p->xbar_forward = 4; p->xbar_response = 2; p->xbar_header = 1; p->xbar_width = 64;
    p->xbar_sf_lookup = 1;
    p->mc_frontend = 10000; p->mc_backend = 10000; p->mc_command_window = 10000;
    p->read_buffer = 32; p->write_buffer = 64; p->write_high_pct = 85; p->write_low_pct = 50;
    p->min_writes_per_switch = 16; p->min_reads_per_switch = 16;
    p->tCK = 1250; p->tBURST = 5000; p->tRCD = 13750; p->tCL = 13750; p->tRP = 13750; p->tRAS = 35000;
    p->tRRD = 6000; p->tXAW = 30000; p->tRFC = 260000; p->tWR = 15000; p->tWTR = 7500; p->tRTP = 7500;
    p->tRTW = 2500; p->tCS = 2500; p->tREFI = 7800000;
    p->activation_limit = 4; p->ranks = 2; p->banks = 8; p->burst_bytes = 64; p->row_buffer_bytes = 8192;
    p->max_accesses_per_row = 16;
    p->mem_bytes = 8ULL << 30;
}

extern "C" fi_status fi_timing_model_run(const fi_timing_op *ops, uint64_t n, const fi_timing_params *p,
                                         fi_timing_ticks *out, fi_timing_stats *stats) {
    if (!ops || !out || !p || n == 0) return FI_E_ARG;
    if (!p->cpu_period || !p->xbar_width || !p->mc_command_window || !p->tCK || !p->ranks || !p->banks ||
        !p->burst_bytes || p->row_buffer_bytes < p->burst_bytes || (p->burst_bytes & (p->burst_bytes - 1)) ||
        p->write_low_pct >= p->write_high_pct || !p->max_accesses_per_row || p->tREFI <= p->tRP ||
        p->tREFI <= p->tRFC || p->ranks > 64 || p->banks > 32)
        return FI_E_ARG;
    for (uint64_t i = 0; i < n; i++) {
        const fi_timing_op &o = ops[i];
        if (o.nfetch < 1 || o.nfetch > 2 || o.nfrag > 2 || o.kind > FI_TOP_END || o.cmd > FI_TCMD_SC ||
            (o.kind == FI_TOP_END) != (i == n - 1) || (o.kind != FI_TOP_EXEC && o.nfrag))
            return FI_E_ARG;
        for (int k = 0; k < o.nfrag; k++) {   // a fragment stays within one burst
            if (!o.size[k] || (o.addr[k] & (p->burst_bytes - 1)) + o.size[k] > p->burst_bytes) return FI_E_ARG;
        }
        for (int k = 0; k < o.nfetch; k++)
            if (o.fetch[k] & 3) return FI_E_ARG;
    }
    memset(out, 0, n * sizeof *out);
    try {
        Model m(*p, ops, n, out);
        const fi_timing_stats st = m.run();
        if (stats) *stats = st;
    } catch (const std::exception &) {
        return FI_E_STATE;   // a state gem5 itself asserts / panics on
    }
    return FI_OK;
}
