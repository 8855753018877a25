// SHREWD functional-unit contention: the O3 issue stage replayed over the
// golden run's committed instructions, recording per dynamic instruction
// whether its shadow copy found a functional unit (include/fi_engine.h,
// "SHREWD functional-unit contention", for what is restated and what is a
// model).  Host code, run once per golden run: O(instructions x IQ entries).
//
// Reference: src/cpu/o3/fu_pool.cc:94-150 (pool construction, per-capability
// unit queues), :155-173 (findFreeUnit), :175-301 (getUnit with the shadow
// substitutions), :303-321 (release next cycle); src/cpu/o3/inst_queue.cc:
// 830-1066 (scheduleReadyInsts: age order over op-class queues, issueWidth,
// priority / deferred shadow requests, unit release), :1082-1181
// (requestShadow); pool and latencies src/cpu/o3/FUPool.py:52-66,
// src/cpu/o3/FuncUnitConfig.py:45-198; widths src/cpu/o3/BaseO3CPU.py.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "fi_engine.h"
#include "fi_types.h"
#include "gem5_opclass_table.h"
#include "rv64_isa.h"

namespace {

// gem5 OpClass enum values used by the RV64 scalar ISA (src/cpu/FuncUnit.py:43)
enum : int {
    kNoOpClass = 0, kIntAlu = 1, kIntMult = 2, kIntDiv = 3, kFloatAdd = 4, kFloatCmp = 5, kFloatCvt = 6,
    kFloatMult = 7, kFloatMultAcc = 8, kFloatDiv = 9, kFloatMisc = 10, kFloatSqrt = 11,
    kMemRead = 52, kMemWrite = 53, kFloatMemRead = 54, kFloatMemWrite = 55, kIprAccess = 56, kNumOpClass = 77
};
// FUPool sentinels (src/cpu/o3/fu_pool.hh:148-167)
constexpr int kNoShadowFU = -7, kNoNeedFU = -3, kNoCapableFU = -2, kNoFreeFU = -1;
constexpr uint64_t kNever = ~0ULL;

struct OpDesc { int cls, lat; bool pipelined; };
struct FUDesc { int which; const OpDesc *ops; int n_ops; };
// FuncUnitConfig.py: IntALU, IntMultDiv, FP_ALU, FP_MultDiv, RdWrPort, IprPort
// (the SIMD / matrix / predicate units serve no scalar class; ReadPort and
// WritePort have count 0)
const OpDesc kIntALU[] = {{kIntAlu, 1, true}};
const OpDesc kIntMultDiv[] = {{kIntMult, 3, true}, {kIntDiv, 20, false}};
const OpDesc kFPALU[] = {{kFloatAdd, 2, true}, {kFloatCmp, 2, true}, {kFloatCvt, 2, true}};
const OpDesc kFPMultDiv[] = {{kFloatMult, 4, true}, {kFloatMultAcc, 5, true}, {kFloatMisc, 3, true},
                             {kFloatDiv, 12, false}, {kFloatSqrt, 24, false}};
const OpDesc kRdWrPort[] = {{kMemRead, 1, true}, {kMemWrite, 1, true}, {kFloatMemRead, 1, true},
                            {kFloatMemWrite, 1, true}};
const OpDesc kIprPort[] = {{kIprAccess, 3, false}};
const FUDesc kPool[6] = {{0, kIntALU, 1}, {1, kIntMultDiv, 2}, {2, kFPALU, 3},
                         {3, kFPMultDiv, 5}, {4, kRdWrPort, 4}, {5, kIprPort, 1}};

class Pool {
public:
    explicit Pool(const uint32_t count[6]) {
        std::fill(pipelined_, pipelined_ + kNumOpClass, true);
        // FUPool::FUPool: every capability gets the indices of all units able
        // to do it, in construction order; a unit queue is a round-robin
        for (const FUDesc &d : kPool) {
            const int n = (int)count[d.which];
            if (!n) continue;
            for (int j = 0; j < d.n_ops; j++) {
                const OpDesc &o = d.ops[j];
                capable_[o.cls] = true;
                for (int k = 0; k < n; k++) queue_[o.cls].units.push_back(n_units_ + k);
                max_lat_[o.cls] = std::max(max_lat_[o.cls], o.lat);
                if (!o.pipelined) pipelined_[o.cls] = false;
            }
            n_units_ += n;
        }
        release_.assign(n_units_, 0);
    }
    int lat(int cls) const { return max_lat_[cls]; }
    bool pipelined(int cls) const { return pipelined_[cls]; }
    bool capable(int cls) const { return capable_[cls]; }

    // FUPool::findFreeUnit: walk the capability's round-robin queue once
    int find_free(int cls, uint64_t now) {
        Queue &q = queue_[cls];
        if (q.units.empty()) return kNoFreeFU;   // (gem5 would index an empty queue)
        int u = q.next();
        const int start = u;
        while (release_[u] > now) {
            u = q.next();
            if (u == start) return kNoFreeFU;
        }
        return u;
    }
    // FUPool::getUnit(capability, is_shadow, approx_capability)
    int get_unit(int cls, bool shadow, int &approx, uint64_t now) {
        if (!capable_[cls]) return kNoCapableFU;
        approx = cls;
        int fu;
        if (shadow) {
            switch (cls) {
            case kIntAlu: {
                fu = find_free(cls, now);
                const int a1 = find_free(kFloatAdd, now), a2 = find_free(kFloatCmp, now);
                if (fu == kNoFreeFU) {
                    fu = a1;
                    approx = kFloatAdd;
                    if (a1 == kNoFreeFU) { approx = kFloatCmp; fu = a2; }
                }
                break;
            }
            case kIntMult: case kIntDiv: {
                const int alt = cls == kIntMult ? kFloatMult : kFloatDiv;
                fu = find_free(cls, now);
                const int a = find_free(alt, now);
                if (fu == kNoFreeFU) { approx = alt; fu = a; }
                break;
            }
            case kFloatAdd: case kFloatMult: case kFloatDiv: case kFloatSqrt: {
                fu = find_free(cls, now);
                const int a = find_free(kIntAlu, now);
                if (fu == kNoFreeFU) { approx = kIntAlu; fu = a; }
                break;
            }
            case kFloatMultAcc: case kFloatCvt: case kFloatCmp: case kFloatMisc:
                fu = find_free(cls, now);
                break;
            default:
                return kNoShadowFU;
            }
        } else {
            fu = find_free(cls, now);
        }
        if (fu == kNoFreeFU) return kNoFreeFU;
        release_[fu] = kNever;   // unitBusy until a release is scheduled
        return fu;
    }
    void release_at(int fu, uint64_t cycle) { release_[fu] = cycle; }

private:
    struct Queue {
        std::vector<int> units;
        size_t idx = 0;
        int next() {   // FUIdxQueue::getFU
            const int u = units[idx++];
            if (idx == units.size()) idx = 0;
            return u;
        }
    };
    Queue queue_[kNumOpClass];
    bool capable_[kNumOpClass] = {};
    int max_lat_[kNumOpClass] = {};
    bool pipelined_[kNumOpClass];
    std::vector<uint64_t> release_;   // a unit is busy while release_ > the current cycle
    int n_units_ = 0;
};

struct Shadow { int idx = kNoNeedFU; int cls = 0; bool has = false; };

// InstructionQueue::requestShadow
void request_shadow(Pool &pool, int idx, int cls, Shadow &s, uint64_t &lat, uint64_t now, fi_issue_stats &st) {
    if (idx == kNoFreeFU || idx == kNoCapableFU) return;
    s.cls = cls;   // shadow_op_class starts as the primary's class
    s.idx = pool.get_unit(cls, true, s.cls, now);
    if (s.idx == kNoShadowFU) return;
    if (s.idx != kNoFreeFU) {
        s.has = true;
        st.shadow_available++;
        lat = std::max<uint64_t>(lat, (uint64_t)pool.lat(s.cls));
        (cls == s.cls ? st.shadow_same_fu : st.shadow_not_same_fu)++;
    } else {
        st.shadow_not_available++;
    }
    if (cls >= kIntAlu && cls <= kFloatSqrt) (s.has ? st.class_available : st.class_not_available)[cls]++;
}

}  // namespace

extern "C" void fi_issue_default_params(fi_issue_params *p) {
    if (!p) return;
    *p = fi_issue_params{};
    p->issue_width = 8; p->dispatch_width = 8; p->commit_width = 8;
    p->iq_entries = 64; p->rob_entries = 192; p->load_latency = 2; p->priority_to_shadow = 0;
    const uint32_t c[6] = {6, 2, 4, 2, 4, 1};
    memcpy(p->fu_count, c, sizeof c);
}

extern "C" fi_status fi_issue_model_run(const fi_issue_op *ops, uint64_t n, const fi_issue_params *p,
                                        uint8_t *shadow, fi_issue_stats *stats_out) {
    if ((n && (!ops || !shadow)) || !p) return FI_E_ARG;
    if (!p->issue_width || !p->dispatch_width || !p->commit_width || !p->iq_entries || !p->rob_entries ||
        !p->load_latency)
        return FI_E_ARG;
    for (uint64_t i = 0; i < n; i++)
        if (ops[i].opclass >= kNumOpClass || ops[i].kind > FI_ISSUE_SERIAL) return FI_E_ARG;
    fi_issue_stats st{};
    st.ops = n;
    Pool pool(p->fu_count);

    std::vector<uint64_t> done(n, kNever);     // cycle the op's value is available (kNever: not issued)
    std::vector<uint64_t> disp(n, 0);
    // producers: the latest older writer of each source register, fixed at dispatch
    std::vector<uint32_t> prod_off(n + 1, 0);
    std::vector<uint64_t> prod;
    int64_t last_writer[64];
    std::fill(last_writer, last_writer + 64, -1);
    std::vector<uint64_t> iq;                  // op ids in age order (issued memory ops stay until done)
    iq.reserve(p->iq_entries);
    uint64_t head = 0, tail = 0;               // ROB: committed ops [0, head), dispatched [0, tail)
    int64_t serial_pending = -1;               // an uncommitted serialising op blocks dispatch
    struct Issued { uint64_t op; int idx; int cls; uint64_t lat; };
    std::vector<Issued> group;
    bool blocked[kNumOpClass];

    uint64_t c = 0;
    while (head < n) {
        // (2) commit, in order
        for (uint32_t k = 0; k < p->commit_width && head < tail && done[head] <= c; k++) head++;
        if (serial_pending >= 0 && (uint64_t)serial_pending < head) serial_pending = -1;
        if (head == n) break;
        // memory ops leave the IQ when done
        iq.erase(std::remove_if(iq.begin(), iq.end(), [&](uint64_t i) { return done[i] <= c; }), iq.end());
        // (3) issue
        std::fill(blocked, blocked + kNumOpClass, false);
        group.clear();
        uint32_t issued = 0;
        for (size_t q = 0; q < iq.size() && issued < p->issue_width; q++) {
            const uint64_t i = iq[q];
            if (done[i] != kNever || disp[i] >= c) continue;
            const int cls = ops[i].opclass;
            if (blocked[cls]) continue;
            bool ready = ops[i].kind != FI_ISSUE_SERIAL || head == i;
            for (uint32_t k = prod_off[i]; ready && k < prod_off[i + 1]; k++) ready = done[prod[k]] <= c;
            if (!ready) continue;
            int idx = kNoNeedFU;
            uint64_t lat = 1;
            if (cls != kNoOpClass) {
                int approx = cls;
                idx = pool.get_unit(cls, false, approx, c);
                if (idx > kNoFreeFU) lat = (uint64_t)pool.lat(cls);
            }
            Shadow s;
            if (p->priority_to_shadow) request_shadow(pool, idx, cls, s, lat, c, st);
            if (!(idx > kNoFreeFU || idx == kNoNeedFU || idx == kNoCapableFU)) {
                blocked[cls] = true;   // FU busy: this op-class queue waits for the next cycle
                continue;
            }
            if (lat == 1) {
                if (idx >= 0) {
                    pool.release_at(idx, c + 1);
                    if (s.has) pool.release_at(s.idx, c + 1);
                }
            } else {
                pool.release_at(idx, pool.pipelined(cls) ? c + 1 : c + lat);
                if (s.has) pool.release_at(s.idx, pool.pipelined(s.cls) ? c + 1 : c + lat);
            }
            if (!p->priority_to_shadow) group.push_back({i, idx, cls, lat});
            shadow[i] = s.has ? 1 : 0;
            const uint8_t kind = ops[i].kind;
            done[i] = c + (kind == FI_ISSUE_LOAD ? (uint64_t)p->load_latency : lat);
            issued++;
            if (kind != FI_ISSUE_LOAD && kind != FI_ISSUE_STORE) { iq.erase(iq.begin() + (ptrdiff_t)q); q--; }
        }
        // deferred shadows: after the issue group, in issue order
        for (const Issued &g : group) {
            Shadow s;
            uint64_t lat = g.lat;
            request_shadow(pool, g.idx, g.cls, s, lat, c, st);
            if (!s.has) { shadow[g.op] = 0; continue; }
            shadow[g.op] = 1;
            if (lat == 1) { if (s.idx >= 0) pool.release_at(s.idx, c + 1); }
            else pool.release_at(s.idx, pool.pipelined(s.cls) ? c + 1 : c + lat);
        }
        // (4) dispatch, in program order
        for (uint32_t k = 0; k < p->dispatch_width && tail < n && serial_pending < 0 &&
                             iq.size() < p->iq_entries && tail - head < p->rob_entries; k++) {
            const uint64_t i = tail++;
            disp[i] = c;
            uint64_t src = ops[i].src & ~1ULL;
            while (src) {
                const int r = __builtin_ctzll(src);
                src &= src - 1;
                if (last_writer[r] >= 0) prod.push_back((uint64_t)last_writer[r]);
            }
            prod_off[i + 1] = (uint32_t)prod.size();
            uint64_t dst = ops[i].dst & ~1ULL;
            while (dst) {
                const int r = __builtin_ctzll(dst);
                dst &= dst - 1;
                last_writer[r] = (int64_t)i;
            }
            iq.push_back(i);
            if (ops[i].kind == FI_ISSUE_SERIAL) serial_pending = (int64_t)i;
        }
        c++;
    }
    st.cycles = c;
    if (stats_out) *stats_out = st;
    return FI_OK;
}

namespace fi {

// gem5 OpClass of an executed op (the table fi_trial.hip:op_class uses)
static int host_op_class(int op) {
    switch (op) {
#define FI_OPC(n, c) case OP_##n: return c;
        FI_GEM5_OPCLASS(FI_OPC)
#undef FI_OPC
    default: return 0;
    }
}

// The replayed trace of a golden run: one op per trace event (committed
// instruction or ecall, fi_engine.cpp golden pass 2).  Integer operands are
// the pre-decoded ones (kPreRs1/kPreRs2/kPreRd, x0 dropped); an ecall reads
// a0..a7 and writes a0 and serialises.  FP register dataflow is not tracked:
// every FP arithmetic op reads and writes one "FP state" register (bit 32), an
// FP load writes it and an FP store reads it, so FP ops form one chain.
// Kinds: MemRead / FloatMemRead (and the AMOs, whose class is their load's) are
// loads, MemWrite / FloatMemWrite stores.  Restated in oracle/rv64se.c:issue_op.
std::vector<fi_issue_op> issue_ops_from_trace(const std::vector<PreInst> &pre, const std::vector<uint32_t> &trace) {
    std::vector<fi_issue_op> ops(trace.size());
    for (size_t i = 0; i < trace.size(); i++) {
        fi_issue_op &o = ops[i];
        o = fi_issue_op{};
        const uint32_t h = trace[i] & 0x7FFFFFFFu;
        if (h >= pre.size()) continue;   // (callers only pass complete traces)
        const PreInst &p = pre[h];
        const int cls = host_op_class(p.op);
        o.opclass = (uint8_t)cls;
        if (trace[i] & 0x80000000u) {
            o.src = 0x3FC00ULL;   // x10..x17
            o.dst = 1ULL << 10;
            o.kind = FI_ISSUE_SERIAL;
            continue;
        }
        if ((p.flags & kPreRs1) && p.rs1) o.src |= 1ULL << p.rs1;
        if ((p.flags & kPreRs2) && p.rs2) o.src |= 1ULL << p.rs2;
        if ((p.flags & kPreRd) && p.rd) o.dst |= 1ULL << p.rd;
        if (cls >= kFloatAdd && cls <= kFloatSqrt) { o.src |= 1ULL << 32; o.dst |= 1ULL << 32; }
        if (cls == kFloatMemRead) o.dst |= 1ULL << 32;
        if (cls == kFloatMemWrite) o.src |= 1ULL << 32;
        o.kind = (cls == kMemRead || cls == kFloatMemRead) ? FI_ISSUE_LOAD
               : (cls == kMemWrite || cls == kFloatMemWrite) ? FI_ISSUE_STORE : FI_ISSUE_PLAIN;
    }
    return ops;
}

}  // namespace fi
