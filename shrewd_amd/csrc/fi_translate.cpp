// fi_translate.cpp -- load-time translation of the golden run's basic blocks
// into straight-line HIP code.
//
// The interpreter (hip/fi_trial.hip) pays a scalar dispatch tree, ballots and
// a dozen branches per guest instruction (~20 cycles per scalar branch on
// gfx950, tools/microbench).  Here each block of the golden text that the
// golden run executed becomes a run of C statements on 31 locals X1..X31 --
// the guest registers, in VGPRs with static indices -- with one ballot-driven
// uniform branch at its end.  The generated code is compiled into the trial
// kernel with hipRTC (fi_jit.cpp) and entered at block leaders; whatever it
// does not cover (ecall, CSR, escapes, illegal encodings, TLB misses,
// copy-on-write, misaligned accesses, divergence, events, untranslated pcs)
// leaves to the interpreter before the instruction, with every counter
// (numInst, cycles, fetch and data bytes) exact.
//
// Semantics follow the interpreter's general path op for op, i.e. the
// generated StaticInst::execute bodies of src/arch/riscv/isa/decoder.isa.
#include <cstdlib>
#include <cctype>
#include <cstdarg>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <map>
#include <set>
#include <unordered_map>
#include <string>
#include <vector>

#include "fi_types.h"
#include "rv64_isa.h"

namespace fi {

namespace {

struct Gen {
    const std::vector<PreInst> &pre;
    uint64_t text_lo;
    const std::set<uint32_t> &leaders;
    const std::set<uint32_t> &executed;
    std::string out;

    void put(const char *fmt, ...) __attribute__((format(printf, 2, 3))) {
        char buf[1024];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        out += buf;
    }
    static std::string R(uint32_t r) { return r ? "X" + std::to_string(r) : std::string("0ULL"); }
    uint64_t pc_of(uint32_t h) const { return text_lo + 2ULL * h; }
};

std::string sfmt(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
std::string sfmt(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    return std::string(buf);
}

enum Cls { C_STOP, C_ALU, C_NOP, C_LOAD, C_STORE, C_BR, C_JAL, C_JALR };

// Classify an instruction and, for ALU ops, produce its value expression in
// terms of A (rs1), B (rs2), IMM and PC.  Every case mirrors the general path
// of fi_trial_kernel; the encodings that raise IllegalInst there are C_STOP.
Cls classify(const PreInst &p, std::string &expr, uint32_t &size, int &sext, const char *&cond) {
    const int64_t imm = p.imm;
    size = 0; sext = 0; cond = nullptr;
    switch (p.op) {
    case OP_c_addi4spn: if (imm == 0) return C_STOP; expr = "A + IMM"; return C_ALU;
    case OP_c_lwsp: if (p.rd == 0) return C_STOP; size = 4; sext = 32; return C_LOAD;
    case OP_c_lw: case OP_lw: size = 4; sext = 32; return C_LOAD;
    case OP_c_ldsp: if (p.rd == 0) return C_STOP; size = 8; return C_LOAD;
    case OP_c_ld: case OP_ld: size = 8; return C_LOAD;
    case OP_c_lbu: case OP_lbu: size = 1; return C_LOAD;
    case OP_c_lhu: case OP_lhu: size = 2; return C_LOAD;
    case OP_c_lh: case OP_lh: size = 2; sext = 16; return C_LOAD;
    case OP_lb: size = 1; sext = 8; return C_LOAD;
    case OP_lwu: size = 4; return C_LOAD;
    case OP_c_sb: case OP_sb: size = 1; return C_STORE;
    case OP_c_sh: case OP_sh: size = 2; return C_STORE;
    case OP_c_sw: case OP_sw: case OP_c_swsp: size = 4; return C_STORE;
    case OP_c_sd: case OP_sd: case OP_c_sdsp: size = 8; return C_STORE;
    case OP_c_addi: case OP_addi: expr = "A + IMM"; return C_ALU;
    case OP_c_addiw: if (p.rd == 0) return C_STOP; expr = "sx32(A + IMM)"; return C_ALU;
    case OP_addiw: expr = "sx32(A + IMM)"; return C_ALU;
    case OP_c_li: case OP_lui: expr = "IMM"; return C_ALU;
    case OP_c_addi16sp: if (imm == 0) return C_STOP; expr = "A + IMM"; return C_ALU;
    case OP_c_lui: if (imm == 0) return C_STOP; expr = "IMM"; return C_ALU;
    case OP_c_srli: case OP_srli: expr = "A >> IMM"; return C_ALU;
    case OP_c_srai: case OP_srai: expr = "(uint64_t)((int64_t)A >> IMM)"; return C_ALU;
    case OP_c_andi: case OP_andi: expr = "A & IMM"; return C_ALU;
    case OP_c_sub: case OP_sub: expr = "A - B"; return C_ALU;
    case OP_c_xor: case OP_xor_: expr = "A ^ B"; return C_ALU;
    case OP_c_or: case OP_or_: expr = "A | B"; return C_ALU;
    case OP_c_and: case OP_and_: expr = "A & B"; return C_ALU;
    case OP_c_subw: case OP_subw: expr = "sx32((uint32_t)A - (uint32_t)B)"; return C_ALU;
    case OP_c_addw: case OP_addw: expr = "sx32((uint32_t)A + (uint32_t)B)"; return C_ALU;
    case OP_c_mul: case OP_mul: expr = "A * B"; return C_ALU;
    case OP_c_zext_b: expr = "A & 0xFFULL"; return C_ALU;
    case OP_c_sext_b: case OP_sext_b: expr = "(uint64_t)sext64(A & 0xFF, 8)"; return C_ALU;
    case OP_c_zext_h: expr = "A & 0xFFFFULL"; return C_ALU;
    case OP_c_sext_h: case OP_sext_h: expr = "(uint64_t)sext64(A & 0xFFFF, 16)"; return C_ALU;
    case OP_c_zext_w: expr = "A & 0xFFFFFFFFULL"; return C_ALU;
    case OP_c_not: expr = "~A"; return C_ALU;
    case OP_c_j: return C_JAL;
    case OP_c_beqz: cond = "A == 0"; return C_BR;
    case OP_c_bnez: cond = "A != 0"; return C_BR;
    case OP_c_slli: case OP_slli: expr = "A << IMM"; return C_ALU;
    case OP_c_jr: if (p.rs1 == 0) return C_STOP; return C_JALR;
    case OP_c_mv: expr = "B"; return C_ALU;
    case OP_c_jalr: return C_JALR;
    case OP_c_add: case OP_add: expr = "A + B"; return C_ALU;
    case OP_fence: case OP_fence_i: case OP_prefetch_i: case OP_prefetch_r: case OP_prefetch_w: return C_NOP;
    case OP_bseti: expr = "A | (1ULL << (IMM & 63))"; return C_ALU;
    case OP_bclri: expr = "A & ~(1ULL << (IMM & 63))"; return C_ALU;
    case OP_binvi: expr = "A ^ (1ULL << (IMM & 63))"; return C_ALU;
    case OP_clz: expr = "(A ? (uint64_t)__builtin_clzll(A) : 64ULL)"; return C_ALU;
    case OP_ctz: expr = "(A ? (uint64_t)__builtin_ctzll(A) : 64ULL)"; return C_ALU;
    case OP_cpop: expr = "(uint64_t)__builtin_popcountll(A)"; return C_ALU;
    case OP_slti: expr = "((int64_t)A < (int64_t)IMM ? 1ULL : 0ULL)"; return C_ALU;
    case OP_sltiu: expr = "(A < IMM ? 1ULL : 0ULL)"; return C_ALU;
    case OP_xori: expr = "A ^ IMM"; return C_ALU;
    case OP_orc_b: expr = "orc_b(A)"; return C_ALU;
    case OP_bexti: expr = "(A >> (IMM & 63)) & 1"; return C_ALU;
    case OP_rori: expr = "(A >> IMM) | (A << ((64 - IMM) & 63))"; return C_ALU;
    case OP_rev8: expr = "__builtin_bswap64(A)"; return C_ALU;
    case OP_ori_hint: case OP_ori: expr = "A | IMM"; return C_ALU;
    case OP_auipc: expr = "PC + IMM"; return C_ALU;
    case OP_slliw: expr = "sx32((uint32_t)A << IMM)"; return C_ALU;
    case OP_slli_uw: expr = "(A & 0xFFFFFFFFULL) << IMM"; return C_ALU;
    case OP_clzw: expr = "((uint32_t)A ? (uint64_t)__builtin_clz((uint32_t)A) : 32ULL)"; return C_ALU;
    case OP_ctzw: expr = "((uint32_t)A ? (uint64_t)__builtin_ctz((uint32_t)A) : 32ULL)"; return C_ALU;
    case OP_cpopw: expr = "(uint64_t)__builtin_popcount((uint32_t)A)"; return C_ALU;
    case OP_srliw: expr = "sx32((uint32_t)A >> IMM)"; return C_ALU;
    case OP_sraiw: expr = "(uint64_t)(int64_t)((int32_t)(uint32_t)A >> IMM)"; return C_ALU;
    case OP_roriw: expr = "sx32(((uint32_t)A >> IMM) | ((uint32_t)A << ((32 - IMM) & 31)))"; return C_ALU;
    case OP_sll: expr = "A << (B & 63)"; return C_ALU;
    case OP_mulh: expr = "(uint64_t)__mul64hi((int64_t)A, (int64_t)B)"; return C_ALU;
    case OP_clmul: expr = "clmul(A, B)"; return C_ALU;
    case OP_bset: expr = "A | (1ULL << (B & 63))"; return C_ALU;
    case OP_bclr: expr = "A & ~(1ULL << (B & 63))"; return C_ALU;
    case OP_rol: expr = "((A << (B & 63)) | (A >> ((64 - (B & 63)) & 63)))"; return C_ALU;
    case OP_binv: expr = "A ^ (1ULL << (B & 63))"; return C_ALU;
    case OP_slt: expr = "((int64_t)A < (int64_t)B ? 1ULL : 0ULL)"; return C_ALU;
    case OP_mulhsu: expr = "(__umul64hi(A, B) - (((int64_t)A < 0) ? B : 0ULL))"; return C_ALU;
    case OP_clmulr: expr = "clmulr(A, B)"; return C_ALU;
    case OP_sh1add: expr = "(A << 1) + B"; return C_ALU;
    case OP_sltu: expr = "(A < B ? 1ULL : 0ULL)"; return C_ALU;
    case OP_mulhu: expr = "__umul64hi(A, B)"; return C_ALU;
    case OP_clmulh: expr = "clmulh(A, B)"; return C_ALU;
    case OP_div_: expr = "div64(A, B)"; return C_ALU;
    case OP_pack: expr = "(B << 32) | (A & 0xFFFFFFFFULL)"; return C_ALU;
    case OP_min_: expr = "((int64_t)A < (int64_t)B ? A : B)"; return C_ALU;
    case OP_sh2add: expr = "(A << 2) + B"; return C_ALU;
    case OP_xnor: expr = "~(A ^ B)"; return C_ALU;
    case OP_srl: expr = "A >> (B & 63)"; return C_ALU;
    case OP_divu: expr = "(B == 0 ? ~0ULL : A / B)"; return C_ALU;
    case OP_czero_eqz: expr = "(B == 0 ? 0ULL : A)"; return C_ALU;
    case OP_sra: expr = "(uint64_t)((int64_t)A >> (B & 63))"; return C_ALU;
    case OP_minu: expr = "(A < B ? A : B)"; return C_ALU;
    case OP_bext: expr = "(A >> (B & 63)) & 1"; return C_ALU;
    case OP_ror: expr = "((A >> (B & 63)) | (A << ((64 - (B & 63)) & 63)))"; return C_ALU;
    case OP_rem: expr = "rem64(A, B)"; return C_ALU;
    case OP_max_: expr = "((int64_t)A > (int64_t)B ? A : B)"; return C_ALU;
    case OP_sh3add: expr = "(A << 3) + B"; return C_ALU;
    case OP_orn: expr = "A | ~B"; return C_ALU;
    case OP_remu: expr = "(B == 0 ? A : A % B)"; return C_ALU;
    case OP_packh: expr = "((B & 0xFF) << 8) | (A & 0xFF)"; return C_ALU;
    case OP_maxu: expr = "(A > B ? A : B)"; return C_ALU;
    case OP_czero_nez: expr = "(B != 0 ? 0ULL : A)"; return C_ALU;
    case OP_andn: expr = "A & ~B"; return C_ALU;
    case OP_mulw: expr = "sx32((uint32_t)A * (uint32_t)B)"; return C_ALU;
    case OP_add_uw: expr = "(A & 0xFFFFFFFFULL) + B"; return C_ALU;
    case OP_sllw: expr = "sx32((uint32_t)A << (B & 31))"; return C_ALU;
    case OP_rolw: expr = "rolw(A, B)"; return C_ALU;
    case OP_sh1add_uw: expr = "((A & 0xFFFFFFFFULL) << 1) + B"; return C_ALU;
    case OP_divw: expr = "divw(A, B)"; return C_ALU;
    case OP_packw: expr = "sx32(((B & 0xFFFF) << 16) | (A & 0xFFFF))"; return C_ALU;
    case OP_sh2add_uw: expr = "((A & 0xFFFFFFFFULL) << 2) + B"; return C_ALU;
    case OP_srlw: expr = "sx32((uint32_t)A >> (B & 31))"; return C_ALU;
    case OP_divuw: expr = "((uint32_t)B == 0 ? ~0ULL : sx32((uint32_t)A / (uint32_t)B))"; return C_ALU;
    case OP_sraw: expr = "(uint64_t)(int64_t)((int32_t)(uint32_t)A >> (B & 31))"; return C_ALU;
    case OP_rorw: expr = "rorw(A, B)"; return C_ALU;
    case OP_remw: expr = "remw(A, B)"; return C_ALU;
    case OP_sh3add_uw: expr = "((A & 0xFFFFFFFFULL) << 3) + B"; return C_ALU;
    case OP_remuw: expr = "((uint32_t)B == 0 ? sx32(A) : sx32((uint32_t)A % (uint32_t)B))"; return C_ALU;
    case OP_beq: cond = "A == B"; return C_BR;
    case OP_bne: cond = "A != B"; return C_BR;
    case OP_blt: cond = "(int64_t)A < (int64_t)B"; return C_BR;
    case OP_bge: cond = "(int64_t)A >= (int64_t)B"; return C_BR;
    case OP_bltu: cond = "A < B"; return C_BR;
    case OP_bgeu: cond = "A >= B"; return C_BR;
    case OP_jalr: return C_JALR;
    case OP_jal: return C_JAL;
    default: return C_STOP;   // ecall, ebreak, CSR, escapes, unknown
    }
}

// Substitute A, B, IMM, PC in an expression template (whole tokens only).
std::string subst(const std::string &t, const std::string &a, const std::string &b, const std::string &imm,
                  const std::string &pc) {
    std::string r;
    for (size_t i = 0; i < t.size();) {
        auto tok = [&](const char *w) {
            const size_t n = strlen(w);
            if (t.compare(i, n, w) != 0) return false;
            const bool lb = i == 0 || !(isalnum((unsigned char)t[i - 1]) || t[i - 1] == '_');
            const bool rb = i + n >= t.size() || !(isalnum((unsigned char)t[i + n]) || t[i + n] == '_');
            return lb && rb;
        };
        if (tok("IMM")) { r += imm; i += 3; }
        else if (tok("PC")) { r += pc; i += 2; }
        else if (tok("A")) { r += a; i += 1; }
        else if (tok("B")) { r += b; i += 1; }
        else r += t[i++];
    }
    return r;
}

const char *gtype(uint32_t size) {
    return size == 1 ? "u8" : size == 2 ? "u16" : size == 4 ? "u32" : "u64";
}

const char *ltype(uint32_t size) {
    return size == 1 ? "uint8_t" : size == 2 ? "uint16_t" : size == 4 ? "uint32_t" : "uint64_t";
}

}  // namespace

namespace {

// Reducible entries.  Every cycle of blocks must have a single
// entry (its header), or the compiler's irreducible-flow fix routes every
// transition through a guard chain -- and then all loops run slowly.  The
// headers are found the classic way: strongly connected components, one
// header each (its lowest-address entry block), recursively inside each
// component with the back edges to its header removed.  Every block stays an
// entry point of the translated code, but the dispatch switch jumps only to
// top-level blocks and headers: a block inside cycles is reached through the
// outermost cycle's header, each header's prologue routing the wanted block
// (etgt) one nesting level further.  Loop back edges are direct gotos; an edge
// that enters a cycle from the side goes through the dispatch switch.
struct Structurer {
    const std::map<uint32_t, std::vector<uint32_t>> &succ;   // block -> successor blocks (direct candidates)
    std::set<uint32_t> entries;                            // top-level entries: reached from dispatch directly
    std::set<std::pair<uint32_t, uint32_t>> exits;         // side entries into a cycle: routed through dispatch
    std::map<uint32_t, std::vector<uint32_t>> chain;       // block -> headers of the cycles around it, outermost first
    std::set<uint32_t> headers;

    void run(const std::vector<uint32_t> &nodes, bool top, std::set<std::pair<uint32_t, uint32_t>> removed) {
        const std::set<uint32_t> in(nodes.begin(), nodes.end());
        // Tarjan's SCC over the induced subgraph (iterative)
        std::map<uint32_t, int> idx, low;
        std::set<uint32_t> onst;
        std::vector<uint32_t> st;
        std::vector<std::vector<uint32_t>> sccs;
        int counter = 0;
        auto edges = [&](uint32_t v) {
            std::vector<uint32_t> r;
            auto it = succ.find(v);
            if (it == succ.end()) return r;
            for (uint32_t w : it->second)
                if (in.count(w) && !removed.count({v, w})) r.push_back(w);
            return r;
        };
        for (uint32_t root : nodes) {
            if (idx.count(root)) continue;
            std::vector<std::pair<uint32_t, size_t>> stack{{root, 0}};
            idx[root] = low[root] = counter++;
            st.push_back(root);
            onst.insert(root);
            while (!stack.empty()) {
                auto &[v, i] = stack.back();
                const std::vector<uint32_t> es = edges(v);
                if (i < es.size()) {
                    const uint32_t w = es[i++];
                    if (!idx.count(w)) {
                        idx[w] = low[w] = counter++;
                        st.push_back(w);
                        onst.insert(w);
                        stack.push_back({w, 0});
                    } else if (onst.count(w)) {
                        low[v] = std::min(low[v], idx[w]);
                    }
                    continue;
                }
                if (low[v] == idx[v]) {
                    std::vector<uint32_t> comp;
                    uint32_t w;
                    do {
                        w = st.back();
                        st.pop_back();
                        onst.erase(w);
                        comp.push_back(w);
                    } while (w != v);
                    sccs.push_back(comp);
                }
                const uint32_t done = v;
                stack.pop_back();
                if (!stack.empty()) low[stack.back().first] = std::min(low[stack.back().first], low[done]);
            }
        }
        for (auto &comp : sccs) {
            std::sort(comp.begin(), comp.end());
            const std::set<uint32_t> cs(comp.begin(), comp.end());
            bool cyclic = comp.size() > 1;
            if (!cyclic)
                for (uint32_t w : edges(comp[0]))
                    if (w == comp[0]) cyclic = true;
            if (!cyclic) {
                if (top) entries.insert(comp[0]);
                continue;
            }
            uint32_t header = comp[0];
            bool have = false;
            for (uint32_t v : nodes) {   // lowest-address block entered from outside the component
                if (cs.count(v)) continue;
                for (uint32_t w : edges(v))
                    if (cs.count(w) && (!have || w < header)) { header = w; have = true; }
            }
            for (uint32_t v : nodes) {
                if (cs.count(v)) continue;
                for (uint32_t w : edges(v))
                    if (cs.count(w) && w != header) exits.insert({v, w});
            }
            if (top) entries.insert(header);
            headers.insert(header);
            for (uint32_t v : comp) chain[v].push_back(header);
            auto inner = removed;
            for (uint32_t v : comp) inner.insert({v, header});
            run(comp, false, inner);
        }
    }
};

struct Block {
    uint32_t h0;
    std::vector<uint32_t> insts;
    bool term;
    uint64_t opc = 0;             // odd-pc block (solo body only): its first pc
    std::vector<uint64_t> opcs;   // ... and the pc of each instruction (insts: their keys)
};

}  // namespace

// Leaders: the first executed instruction, every instruction the golden run
// reached other than by falling through, the successor of every executed
// control transfer or ecall, the extra pcs, and the same for the code
// statically reachable from the executed code.  trace = halfword index per
// golden event (bit 31: ecall).
//
// Four bodies are generated (joined by the marker FI_TX_SPLIT): the 64-lane
// one (blocks B_*, guest registers X1..X31 in VGPRs, register writes as
// selects on the running group, divergence parked and merged by the min-PC
// rule), the solo one for the one-trial-per-wave kernel (blocks S_*, every
// value uniform, no groups), the solo-odd one (the solo blocks again as Q_*
// plus the odd-pc streams as QO_*; empty when there are none) and the clean
// solo one: the solo blocks for a trial that rewrote no code and watches no
// register -- no rewritten-byte or watch checks, and a store into the code
// range leaves before it (the interpreter marks the bytes; the trial then
// takes the full solo body).
std::string translate_blocks(const std::vector<PreInst> &pre, uint64_t text_lo, const std::vector<uint32_t> &trace,
                             const std::vector<uint64_t> &extra_pcs, std::vector<uint32_t> &leaders_out,
                             uint32_t &n_insts, bool odd_streams, std::vector<LoopEst> *loops_out) {
    std::set<uint32_t> executed, leaders;
    auto valid = [&](uint32_t h) { return h < pre.size() && (pre[h].flags & kPreValid); };
    // only code the golden run executed more than once is translated: straight-
    // line code run once gains nothing from it, and a long run of it makes one
    // huge block that takes the load-time compiler minutes
    std::unordered_map<uint32_t, uint32_t> runs;
    for (size_t i = 0; i < trace.size(); i++) {
        const uint32_t h = trace[i] & 0x7FFFFFFFu;
        if (valid(h)) runs[h]++;
    }
    for (size_t i = 0; i < trace.size(); i++) {
        const uint32_t h = trace[i] & 0x7FFFFFFFu;
        if (!valid(h) || runs[h] < 2) continue;
        executed.insert(h);
        const bool is_ecall = trace[i] & 0x80000000u;
        if (i == 0) leaders.insert(h);
        if (i + 1 < trace.size()) {
            const uint32_t nh = trace[i + 1] & 0x7FFFFFFFu;
            if (is_ecall || nh != h + pre[h].len / 2u) leaders.insert(nh);
        }
    }
    for (auto it = leaders.begin(); it != leaders.end();) {   // (a transition into code run once)
        if (!executed.count(*it)) it = leaders.erase(it);
        else ++it;
    }
    for (uint32_t h : executed) {   // successors of control transfers
        std::string e;
        uint32_t sz;
        int sx;
        const char *cond;
        const Cls k = classify(pre[h], e, sz, sx, cond);
        if ((k == C_BR || k == C_JAL || k == C_JALR) && executed.count(h + pre[h].len / 2u))
            leaders.insert(h + pre[h].len / 2u);
    }
    const std::set<uint32_t> golden_exec = executed;
    // static closure: code the golden run never executed but that its direct
    // control flow reaches (the other side of a branch, a call's return site,
    // the code after an ecall) -- faulty trials go there, and translated code
    // runs it ~4x faster than the pre-decoded interpreter
    {
        std::vector<uint32_t> work(executed.begin(), executed.end());
        auto push = [&](int64_t h, bool lead) {
            if (h < 0 || !valid((uint32_t)h)) return;
            if (lead) leaders.insert((uint32_t)h);
            if (executed.insert((uint32_t)h).second) work.push_back((uint32_t)h);
        };
        while (!work.empty()) {
            const uint32_t h = work.back();
            work.pop_back();
            std::string e;
            uint32_t sz;
            int sx;
            const char *cond;
            const Cls k = classify(pre[h], e, sz, sx, cond);
            const int64_t ft = (int64_t)h + pre[h].len / 2;
            const int64_t tg = (int64_t)h + pre[h].imm / 2;
            switch (k) {
            case C_BR: push(ft, true); push(tg, true); break;
            case C_JAL: push(tg, true); push(ft, true); break;
            case C_JALR: case C_STOP: push(ft, true); break;
            default: push(ft, false); break;
            }
        }
    }
    for (uint64_t pc : extra_pcs) {
        if (pc < text_lo || ((pc - text_lo) & 1)) continue;
        const uint64_t h = (pc - text_lo) / 2;
        if (h < pre.size() && executed.count((uint32_t)h)) leaders.insert((uint32_t)h);
    }
    // drop leaders whose first instruction is not translatable (no block)
    for (auto it = leaders.begin(); it != leaders.end();) {
        std::string e;
        uint32_t sz;
        int sx;
        const char *cond;
        if (!valid(*it) || classify(pre[*it], e, sz, sx, cond) == C_STOP) it = leaders.erase(it);
        else ++it;
    }

    // ---- odd-pc streams (solo body only).  A pc bit-0 flip leaves the pc odd;
    // an odd pc fetches its word's pc | 2 halfword (key (pc & ~3) | 2) and
    // steps by the instruction length, so the stream stays odd until a jalr.
    // The entries are the golden pcs | 1 (both odd pcs of a word, which share
    // one pre-decoded entry and its flag), closed under the stream's direct
    // control flow.  Blocks run from an odd leader (a branch or jal target, the
    // pc after a control transfer, a pc no other odd instruction falls into)
    // to a control transfer or the next leader; they are entered and left
    // through the dispatch (no direct edges: the even blocks' cycle structure
    // stays as the structurer made it).  Both odd pcs of a word lead together:
    // they share the key's kPreOddLeader flag, at which the interpreter hands
    // over.
    // The odd blocks take a crc32 pc bit-0 tail trial from ~600 to ~128 ns
    // per instruction and a qsort one from ~676 to ~275 ns, but they are ~2.7x
    // the solo body's even code on crc32, and in the solo kernel itself (SGPR
    // spills 1.7k -> 8.3k) they slowed the whole solo epoch by ~10 %
    // (profiles/r02p_odd_ab.txt).  So they go into a third body (solo-odd: the
    // even blocks again plus the odd ones, labels Q*) that only the survivors
    // standing at an odd pc run (fi_trial_kernel_tx_solo_odd, fi_engine.cpp).
    std::set<uint64_t> odd;
    if (odd_streams) {
        const size_t cap = 2 * golden_exec.size() + 1024;
        std::vector<uint64_t> work;
        for (uint32_t h : golden_exec) work.push_back(text_lo + 2ULL * h + 1);
        while (!work.empty() && odd.size() < cap) {
            const uint64_t pc = work.back();
            work.pop_back();
            if (pc < text_lo || odd.count(pc)) continue;
            const uint64_t hk = (((pc & ~3ULL) | 2) - text_lo) / 2;
            if (hk >= pre.size() || !valid((uint32_t)hk)) continue;
            std::string e;
            uint32_t sz;
            int sx;
            const char *cond;
            const Cls k = classify(pre[hk], e, sz, sx, cond);
            if (k == C_STOP) continue;
            odd.insert(pc);
            work.push_back(pc ^ 2);
            const uint64_t ft = pc + pre[hk].len, tg = pc + (int64_t)pre[hk].imm;
            if (k == C_BR) { work.push_back(ft); work.push_back(tg); }
            else if (k == C_JAL) work.push_back(tg);
            else if (k != C_JALR) work.push_back(ft);
        }
    }

    // ---- the blocks: from a leader until a control transfer (inclusive), an
    // untranslatable or unexecuted instruction, or the next leader
    std::vector<Block> blocks;
    std::map<uint32_t, std::vector<uint32_t>> succ;
    auto hof = [&](uint64_t pc, uint32_t &h) {
        const uint64_t off = pc - text_lo;
        if (pc < text_lo || (off & 1) || off / 2 >= pre.size() || !leaders.count((uint32_t)(off / 2))) return false;
        h = (uint32_t)(off / 2);
        return true;
    };
    for (uint32_t h0 : leaders) {
        Block b{h0, {}, false};
        uint32_t h = h0;
        for (;;) {
            if (!valid(h) || !executed.count(h)) break;
            if (h != h0 && leaders.count(h)) break;
            std::string e;
            uint32_t sz;
            int sx;
            const char *cond;
            const Cls k = classify(pre[h], e, sz, sx, cond);
            if (k == C_STOP) break;
            b.insts.push_back(h);
            if (k == C_BR || k == C_JAL || k == C_JALR) { b.term = true; break; }
            h += pre[h].len / 2u;
        }
        auto &sv = succ[h0];
        const uint64_t pc_last = b.insts.empty() ? text_lo + 2ULL * h0 : text_lo + 2ULL * b.insts.back();
        const PreInst &pl = pre[b.insts.empty() ? h0 : b.insts.back()];
        uint32_t t;
        if (b.term) {
            std::string e;
            uint32_t sz;
            int sx;
            const char *cond;
            const Cls k = classify(pl, e, sz, sx, cond);
            if (k == C_BR || k == C_JAL) {
                if (hof(pc_last + (int64_t)pl.imm, t)) sv.push_back(t);
            }
            if (k == C_BR && hof(pc_last + pl.len, t)) sv.push_back(t);
        } else if (!b.insts.empty() && hof(pc_last + pl.len, t)) {
            sv.push_back(t);
        }
        blocks.push_back(b);
    }
    Structurer S{succ, {}, {}};
    S.run(std::vector<uint32_t>(leaders.begin(), leaders.end()), true, {});
    auto okey = [&](uint64_t pc) { return (uint32_t)((((pc & ~3ULL) | 2) - text_lo) / 2); };
    auto ocls = [&](uint64_t pc) {
        std::string e;
        uint32_t sz;
        int sx;
        const char *cond;
        return classify(pre[okey(pc)], e, sz, sx, cond);
    };
    std::set<uint64_t> olead, ofall;   // odd leaders; odd pcs some odd non-transfer falls into
    for (uint64_t pc : odd) {
        const Cls k = ocls(pc);
        const uint64_t ft = pc + pre[okey(pc)].len;
        if (k == C_BR || k == C_JAL) {
            const uint64_t tg = pc + (int64_t)pre[okey(pc)].imm;
            if (odd.count(tg)) olead.insert(tg);
        }
        if (k == C_BR || k == C_JAL || k == C_JALR) { if (odd.count(ft)) olead.insert(ft); }
        else ofall.insert(ft);
    }
    for (uint64_t pc : odd)
        if (!ofall.count(pc)) olead.insert(pc);
    for (uint64_t pc : std::vector<uint64_t>(olead.begin(), olead.end()))
        if (odd.count(pc ^ 2)) olead.insert(pc ^ 2);
    for (uint64_t pc0 : olead) {
        Block b{okey(pc0), {}, false};
        b.opc = pc0;
        for (uint64_t pc = pc0; odd.count(pc) && (pc == pc0 || !olead.count(pc));) {
            b.insts.push_back(okey(pc));
            b.opcs.push_back(pc);
            const Cls k = ocls(pc);
            if (k == C_BR || k == C_JAL || k == C_JALR) { b.term = true; break; }
            pc += pre[okey(pc)].len;
        }
        blocks.push_back(b);
    }
    bool cur_odd = false;   // generating an odd-pc block: every edge goes through the dispatch
    bool oddon = false;     // generating the solo-odd body (even and odd blocks, labels Q*)
    std::string SB = "S_", SD = "S_dispatch", SOB = "SO_";

    enum Edge { E_DIRECT, E_DISPATCH, E_OUT };
    auto edge = [&](uint32_t from, uint64_t pc) {
        uint32_t t;
        if (!hof(pc, t)) return E_OUT;
        return S.exits.count({from, t}) ? E_DISPATCH : E_DIRECT;
    };

    Gen g{pre, text_lo, leaders, executed, {}};
    Gen so{pre, text_lo, leaders, executed, {}};
    Gen sq{pre, text_lo, leaders, executed, {}};
    Gen sc{pre, text_lo, leaders, executed, {}};   // the clean solo body (mode 0 only)
    // clean body: memory sites in cycles keep the last page they translated
    // (CV_i / CP_i: vpn and TLB entry; the TLB does not change inside the
    // blocks, so a hit equals tlb_find) -- at most kSiteCaches of them
    constexpr uint32_t kSiteCaches = 8;
    uint32_t n_sites = 0;
    n_insts = 0;
    auto hex = [](uint64_t v) {
        char b[32];
        snprintf(b, sizeof b, "0x%llxULL", (unsigned long long)v);
        return std::string(b);
    };
    // wave: where to go from block `from` to pc (lanes of the running group)
    auto wgo = [&](uint32_t from, uint64_t pc) {
        const Edge k = edge(from, pc);
        uint32_t t = 0;
        hof(pc, t);
        if (k == E_DIRECT) return "goto B_" + std::to_string(t) + ";";
        return "{ spc = " + hex(pc) + (k == E_DISPATCH ? "; goto tx_dispatch; }" : "; goto tx_out; }");
    };
    // clean body (profiles/r04an-r04ap): a load site caches only a mapped page
    // (the probe's checks move to the miss), a store site only a private page
    // outside the code range, the budget counts down (one compare per check
    // point), and the site caches' miss / leave tests and the budget tests are
    // hinted cold (SCOLD) so that a block's hot path falls through.  (Losing
    // variants removed in round 5: loads from private pages hinted cold, within
    // noise; proofs re-tested on direct loop entries, -9 %, profiles/r04at.)
    const char *cold = "SCOLD";
    auto sgo = [&](uint32_t from, uint64_t pc) {
        // solo-odd body: an odd target with a block is a direct edge (the
        // odd blocks are entered at their first pc only); an even one goes
        // through the dispatch
        if (oddon && (pc & 1))
            return olead.count(pc) ? "goto " + SOB + std::to_string((uint32_t)((pc - text_lo) >> 1)) + ";"
                                   : "{ spc = " + hex(pc) + "; goto S_out; }";
        if (oddon && cur_odd) return "{ spc = " + hex(pc) + "; goto " + SD + "; }";
        const Edge k = edge(from, pc);
        uint32_t t = 0;
        hof(pc, t);
        if (k == E_DIRECT) return "goto " + SB + std::to_string(t) + ";";
        return "{ spc = " + hex(pc) + (k == E_DISPATCH ? "; goto " + SD + "; }" : "; goto S_out; }");
    };
    // ---- counted-loop hang proofs (clean body).  A cycle of blocks with no
    // nested cycle, no memory access and no indirect jump, left only by one
    // branch on a register Xk against zero (it stays in the cycle while Xk !=
    // 0) right after the cycle's only write of Xk, Xk = Xk + c with c = +-1 in
    // the same block: from any block boundary in the cycle the branch is
    // passed n more times, Xk + n c = 0 (mod 2^64; n = 2^64 for Xk = 0), and
    // between two passes the trial commits at least m instructions (the
    // shortest way around the cycle).  It cannot terminate, fault or call
    // inside, so it commits at least (n - 1) m instructions before it leaves
    // -- once that reaches the hang cap the trial is a hang, and nothing it
    // would do until then can change its outcome: it cannot meet a golden
    // snapshot either (the golden run would then run that loop past the cap
    // too).  The clean body's dispatch tests it (TXHANG) whenever it enters
    // such a cycle, i.e. once per call.
    //
    // Run-off loops (one block that branches to itself): the same counter
    // test, the exit also against a register the block does not write (bne
    // a0, a1), steps of +-1, 2, 4, 8, and plain loads whose address is either
    // the counter plus a constant or a register the block does not write plus
    // a bounded offset (andi / slli / shNadd chains: a table lookup), and
    // stores at the counter plus a constant (round 6: the data they write
    // never steers the loop).  Such a loop that cannot leave before the cap
    // either faults on a counter access's first page that is not mapped (a
    // crash at an exact instruction) or reaches the cap; the kernel decides
    // which from the lane's page set (loop_outcome, fi_trial.hip; a store walk
    // that would reach the code range stays undecided), so the body only
    // passes the accesses on.
    // kind 0 counter load, 1 bounded load, 2 counter store, 3 / 4 load / store
    // at another induction register (span = its step per iteration, int32)
    struct ProofLoad { uint32_t reg, kind, size, pos; int64_t off; uint64_t span; };
    struct HangProof { uint32_t reg, treg; int step; uint32_t m; std::vector<ProofLoad> loads; bool rel = false; };
    std::map<uint32_t, HangProof> hang_proof;
    // abstract value of a register inside a run-off block: TOP unknown; CNT the
    // counter's value at the iteration's start + lo; BND base register (0: none)
    // plus an offset in [lo, hi]
    struct AVal { int k; uint32_t base; int64_t lo, hi; };
    enum { AV_TOP, AV_CNT, AV_BND, AV_IND };   // AV_IND: another induction register base, + lo
    const int64_t kAvLim = (int64_t)1 << 40;
    auto av_ok = [&](AVal v) { return v.k == AV_BND && v.lo > -kAvLim && v.hi < kAvLim && v.lo <= v.hi ? v : AVal{AV_TOP, 0, 0, 0}; };
    auto av_add = [&](AVal a, AVal b) -> AVal {
        if (a.k != AV_BND || b.k != AV_BND || (a.base && b.base)) return AVal{AV_TOP, 0, 0, 0};
        return av_ok(AVal{AV_BND, a.base | b.base, a.lo + b.lo, a.hi + b.hi});
    };
    auto av_shl = [&](AVal a, int64_t k) -> AVal {
        if (a.k != AV_BND || a.base || a.lo < 0 || k < 0 || k > 20) return AVal{AV_TOP, 0, 0, 0};
        return av_ok(AVal{AV_BND, 0, a.lo << k, a.hi << k});
    };
    auto av_const = [&](int64_t lo, int64_t hi) { return av_ok(AVal{AV_BND, 0, lo, hi}); };
    for (uint32_t H : S.headers) {
        std::vector<uint32_t> cyc;
        bool nested = false;
        for (const auto &kv : S.chain) {
            const auto pos = std::find(kv.second.begin(), kv.second.end(), H);
            if (pos == kv.second.end()) continue;
            if (pos + 1 != kv.second.end()) nested = true;
            cyc.push_back(kv.first);
        }
        if (nested || cyc.empty()) continue;
        const std::set<uint32_t> in(cyc.begin(), cyc.end());
        std::map<uint32_t, const Block *> bl;
        for (const Block &b : blocks)
            if (b.opc == 0 && in.count(b.h0)) bl[b.h0] = &b;
        if (bl.size() != in.size()) continue;
        bool ok = true;
        uint32_t writes[32] = {0};
        std::map<uint32_t, std::vector<uint32_t>> nx;   // edges inside the cycle
        uint32_t n_exit = 0, eblk = 0;
        bool exit_on_taken = false;
        for (const auto &kv : bl) {
            const Block &b = *kv.second;
            if (b.insts.empty()) { ok = false; break; }
            auto to = [&](uint64_t pc, bool taken) {
                uint32_t t;
                if (hof(pc, t) && in.count(t) && !S.exits.count({b.h0, t})) nx[b.h0].push_back(t);
                else { n_exit++; eblk = b.h0; exit_on_taken = taken; }
            };
            for (size_t i = 0; i < b.insts.size() && ok; i++) {
                std::string e;
                uint32_t sz;
                int sx;
                const char *cond;
                const PreInst &p = pre[b.insts[i]];
                const uint64_t pc = text_lo + 2ULL * b.insts[i];
                const Cls k = classify(p, e, sz, sx, cond);
                if (k == C_JALR || k == C_STOP || ((k == C_LOAD || k == C_STORE) && in.size() != 1)) ok = false;
                if ((k == C_ALU || k == C_JAL || k == C_LOAD) && p.rd) writes[p.rd]++;
                if (k == C_BR) { to(pc + (int64_t)p.imm, true); to(pc + p.len, false); }
                if (k == C_JAL) to(pc + (int64_t)p.imm, true);
            }
            if (ok && !b.term) to(text_lo + 2ULL * b.insts.back() + pre[b.insts.back()].len, false);
        }
        if (!ok || n_exit != 1) continue;
        const Block &E = *bl[eblk];
        const PreInst &br = pre[E.insts.back()];
        uint32_t reg = 0, treg = 0;    // counter, and the register it is compared with (0: zero)
        bool exit_when_zero = false;   // the exit edge is taken when Xk == X[treg]
        if (br.op == OP_c_beqz || br.op == OP_c_bnez) {
            reg = br.rs1;
            exit_when_zero = (br.op == OP_c_beqz) == exit_on_taken;
        } else if ((br.op == OP_beq || br.op == OP_bne) && (br.rs1 == 0) != (br.rs2 == 0)) {
            reg = br.rs1 ? br.rs1 : br.rs2;
            exit_when_zero = (br.op == OP_beq) == exit_on_taken;
        } else if ((br.op == OP_beq || br.op == OP_bne) && br.rs1 && br.rs2 && br.rs1 != br.rs2) {
            if (writes[br.rs1] == 1 && writes[br.rs2] == 0) { reg = br.rs1; treg = br.rs2; }
            else if (writes[br.rs2] == 1 && writes[br.rs1] == 0) { reg = br.rs2; treg = br.rs1; }
            exit_when_zero = (br.op == OP_beq) == exit_on_taken;
        }
        if (!reg || !exit_when_zero || writes[reg] != 1) continue;
        int step = 0;
        for (size_t i = 0; i + 1 < E.insts.size(); i++) {
            const PreInst &p = pre[E.insts[i]];
            const int a = p.imm < 0 ? -p.imm : p.imm;
            if ((p.op == OP_addi || p.op == OP_c_addi) && p.rd == reg && p.rs1 == reg && (a == 1 || a == 2 || a == 4 || a == 8))
                step = p.imm;
        }
        if (!step) continue;
        // run-off block: the loads' addresses
        std::vector<ProofLoad> loads;
        if (in.size() == 1) {
            AVal av[32];
            for (uint32_t r = 0; r < 32; r++) av[r] = writes[r] ? AVal{AV_TOP, 0, 0, 0} : AVal{AV_BND, r, 0, 0};
            // other induction registers: written once per iteration, by
            // addi r, r, c -- an access at r walks memory with its own step
            // (kinds 3 / 4: the step travels in the span field)
            int ind_step[32] = {0};
            for (size_t i = 0; i < E.insts.size(); i++) {
                const PreInst &p = pre[E.insts[i]];
                if ((p.op == OP_addi || p.op == OP_c_addi) && p.rd && p.rd == p.rs1 && p.rd != reg && writes[p.rd] == 1 &&
                    p.imm != 0 && p.imm >= -2048 && p.imm <= 2048) {
                    ind_step[p.rd] = p.imm;
                    av[p.rd] = AVal{AV_IND, p.rd, 0, 0};
                }
            }
            av[reg] = AVal{AV_CNT, 0, 0, 0};
            for (size_t i = 0; i < E.insts.size() && ok; i++) {
                std::string e;
                uint32_t sz;
                int sx;
                const char *cond;
                const PreInst &p = pre[E.insts[i]];
                const Cls k = classify(p, e, sz, sx, cond);
                const AVal A = av[p.rs1], B = av[p.rs2];
                const int64_t imm = p.imm;
                if (k == C_LOAD) {
                    if (A.k == AV_CNT) loads.push_back({reg, 0u, sz, (uint32_t)i, A.lo + imm, 0u});
                    else if (A.k == AV_IND)
                        loads.push_back({A.base, 3u, sz, (uint32_t)i, A.lo + imm, (uint64_t)(uint32_t)ind_step[A.base]});
                    else if (A.k == AV_BND) loads.push_back({A.base, 1u, sz, (uint32_t)i, A.lo + imm, (uint64_t)(A.hi - A.lo)});
                    else ok = false;
                    if (p.rd) av[p.rd] = AVal{AV_TOP, 0, 0, 0};
                    continue;
                }
                // a store at the counter plus a constant walks memory like a
                // counter load (kind 2: loop_outcome also keeps it out of the
                // code range); its data never steers the loop, whose exit
                // depends on the counter alone.  Any other store: no proof.
                if (k == C_STORE) {
                    if (A.k == AV_CNT) loads.push_back({reg, 2u, sz, (uint32_t)i, A.lo + imm, 0u});
                    else if (A.k == AV_IND)
                        loads.push_back({A.base, 4u, sz, (uint32_t)i, A.lo + imm, (uint64_t)(uint32_t)ind_step[A.base]});
                    else ok = false;
                    continue;
                }
                if (!p.rd || (k != C_ALU && k != C_JAL)) continue;
                AVal v{AV_TOP, 0, 0, 0};
                if (k == C_ALU) switch (p.op) {
                case OP_addi: case OP_c_addi: case OP_c_addi4spn: case OP_c_addi16sp:
                    if (A.k == AV_CNT) v = AVal{AV_CNT, 0, A.lo + imm, A.lo + imm};
                    else if (A.k == AV_IND && p.rd == A.base) v = AVal{AV_IND, A.base, A.lo + imm, A.lo + imm};
                    else v = av_add(A, av_const(imm, imm));
                    break;
                case OP_add: case OP_c_add: v = av_add(A, B); break;
                case OP_c_mv: v = B; break;
                case OP_andi: case OP_c_andi: if (imm >= 0) v = av_const(0, imm); break;
                case OP_c_zext_b: v = av_const(0, 0xFF); break;
                case OP_c_zext_h: v = av_const(0, 0xFFFF); break;
                case OP_slli: case OP_c_slli: v = av_shl(A, imm); break;
                case OP_srli: case OP_c_srli: if (imm >= 44 && imm < 64) v = av_const(0, (int64_t)((1ULL << (64 - imm)) - 1)); break;
                case OP_sh1add: v = av_add(av_shl(A, 1), B); break;
                case OP_sh2add: v = av_add(av_shl(A, 2), B); break;
                case OP_sh3add: v = av_add(av_shl(A, 3), B); break;
                case OP_c_li: case OP_lui: v = av_const(imm, imm); break;
                default: break;
                }
                av[p.rd] = v;
            }
            for (const ProofLoad &l : loads)
                if (l.off <= -((int64_t)1 << 31) || l.off >= ((int64_t)1 << 31) || (l.kind < 3 && l.span >= (1u << 20)))
                    ok = false;
            if (!ok || loads.size() > 4) continue;
        }
        // m: the fewest instructions from E's successor in the cycle around to E's end
        std::map<uint32_t, uint32_t> dist;
        std::set<std::pair<uint32_t, uint32_t>> q;
        for (uint32_t t : nx[eblk]) {
            const uint32_t d = (uint32_t)bl[t]->insts.size();
            if (!dist.count(t) || d < dist[t]) { dist[t] = d; q.insert({d, t}); }
        }
        uint32_t m = 0;
        while (!q.empty()) {
            const auto [d, v] = *q.begin();
            q.erase(q.begin());
            if (d != dist[v]) continue;
            if (v == eblk) { m = d; break; }
            for (uint32_t t : nx[v]) {
                const uint32_t nd = d + (uint32_t)bl[t]->insts.size();
                if (!dist.count(t) || nd < dist[t]) { dist[t] = nd; q.insert({nd, t}); }
            }
        }
        if (!m) continue;
        for (uint32_t h : cyc) { hang_proof[h] = {reg, treg, step, m, loads}; }
        if (loops_out && loops_out->size() < kMaxLoopEst) {   // the loop's text span (offsets from text_lo)
            uint32_t lo = ~0u, hi = 0;
            for (const auto &kv : bl) {
                const Block &b = *kv.second;
                lo = std::min(lo, 2u * b.h0);
                hi = std::max(hi, 2u * b.insts.back() + pre[b.insts.back()].len);
            }
            loops_out->push_back(LoopEst{lo, hi, (uint8_t)reg, (uint8_t)treg, (int8_t)step, 0, m});
        }
    }

    // ---- region proofs (round 6): an outer counted loop that calls a leaf
    // function and reads / writes bounded tables.  Block E ends with
    // `bltu rc, rl, H` back to a header H (the loop runs while rc < rl,
    // unsigned), E holds the region's only write of rc, `addi rc, rc, c`
    // (0 < c <= 8), and rl is written nowhere in the region.  The region is
    // every block reachable from H by direct edges, a call (`jal ra, f`) into
    // f's blocks, and f's `ret` back to the call's return site, without
    // passing E's fall-through (the exit).  Every block of it must be
    // translated code (no ecall, CSR, indirect jump other than that ret, no
    // nested call, ra written only by the calls) and every load / store
    // address a register the region never writes plus a bounded offset (a
    // table).  Then nothing in the region can leave it but E's exit test,
    // nothing in it can fault once the tables' pages are in the lane's set
    // and the stores miss the code range (loop_outcome, kinds 1 / 5), and rc
    // grows by at most c per pass -- E runs once per pass --, so from any
    // point of the region the loop passes E at least k = ceil((rl - rc) / c)
    // more times, at least m instructions apart (m: the shortest pass, callee
    // included): it commits (k - 1) m instructions before it can leave.  Data
    // (the hash, the tables' contents, the callee's inner loops) never matter:
    // a pass that spins inside the region only makes the trial longer.  The
    // test runs at the dispatch entries of the loop's own blocks (not the
    // callee's, which other call sites share), including the return site that
    // every `ret` enters through the dispatch.
    {
        std::map<uint32_t, const Block *> blk;
        for (const Block &b : blocks)
            if (b.opc == 0 && !b.insts.empty()) blk[b.h0] = &b;
        for (const Block &E : blocks) {
            if (E.opc != 0 || E.insts.empty() || !E.term) continue;
            const PreInst &br = pre[E.insts.back()];
            if (br.op != OP_bltu || !br.rs1 || !br.rs2 || br.rs1 == br.rs2) continue;
            const uint64_t epc = g.pc_of(E.insts.back()), hpc = epc + (int64_t)br.imm;
            uint32_t H;
            if (!hof(hpc, H) || !blk.count(H) || hpc > epc) continue;
            const uint32_t rc = br.rs1, rl = br.rs2;
            int c = 0;
            for (size_t i = 0; i + 1 < E.insts.size(); i++) {
                const PreInst &p = pre[E.insts[i]];
                if ((p.op == OP_addi || p.op == OP_c_addi) && p.rd == rc && p.rs1 == rc && p.imm > 0 && p.imm <= 8) c = p.imm;
            }
            if (!c || hang_proof.count(H)) continue;
            // the region: blocks by direct edges, calls and their returns
            std::set<uint32_t> own, callee, ret_sites;
            std::vector<std::pair<uint32_t, bool>> work{{H, false}};
            std::map<uint32_t, std::vector<uint32_t>> nxt;   // region edges (for the shortest pass)
            bool ok = true;
            std::set<std::pair<uint32_t, bool>> seen;
            while (!work.empty() && ok) {
                const auto [h, in_f] = work.back();
                work.pop_back();
                if (!seen.insert({h, in_f}).second) continue;
                if (seen.size() > 256) { ok = false; break; }
                auto bi = blk.find(h);
                if (bi == blk.end()) { ok = false; break; }
                const Block &b = *bi->second;
                (in_f ? callee : own).insert(h);
                auto go = [&](uint64_t pc, bool f) {
                    uint32_t t;
                    if (!hof(pc, t) || !blk.count(t)) { ok = false; return; }
                    nxt[h].push_back(t);
                    work.push_back({t, f});
                };
                for (size_t i = 0; i < b.insts.size() && ok; i++) {
                    std::string e;
                    uint32_t sz;
                    int sx;
                    const char *cond;
                    const PreInst &p = pre[b.insts[i]];
                    const uint64_t pc = g.pc_of(b.insts[i]);
                    const Cls k = classify(p, e, sz, sx, cond);
                    if (k == C_STOP) ok = false;
                    else if (k == C_BR) {
                        if (&b == &E && i + 1 == b.insts.size()) { go(hpc, false); continue; }   // the exit: not followed
                        go(pc + (int64_t)p.imm, in_f);
                        go(pc + p.len, in_f);
                    } else if (k == C_JAL) {
                        if (p.rd == 0) go(pc + (int64_t)p.imm, in_f);
                        else if (p.rd == 1 && !in_f) {   // a call: the callee, and the return site after it
                            uint32_t rs;
                            if (!hof(pc + p.len, rs) || !blk.count(rs)) { ok = false; continue; }
                            ret_sites.insert(rs);
                            go(pc + (int64_t)p.imm, true);
                            work.push_back({rs, false});   // (no edge: a pass goes through the callee)
                        }
                        else ok = false;   // another link register, or a nested call
                    } else if (k == C_JALR) {
                        // only a callee's `ret` (jalr x0, 0(ra) or c.jr ra), back to the
                        // return sites (c.jalr links ra: no)
                        if (!(in_f && p.op != OP_c_jalr && p.rd == 0 && p.rs1 == 1 && p.imm == 0)) ok = false;
                    }
                }
                if (ok && !b.term) go(g.pc_of(b.insts.back()) + pre[b.insts.back()].len, in_f);
            }
            if (!ok || own.empty() || !own.count(E.h0)) continue;
            for (uint32_t r : ret_sites) {   // each ret continues at the return sites
                for (uint32_t f : callee) {
                    const Block &fb = *blk[f];
                    const PreInst &lp = pre[fb.insts.back()];
                    std::string e;
                    uint32_t sz;
                    int sx;
                    const char *cond;
                    if (classify(lp, e, sz, sx, cond) == C_JALR) nxt[f].push_back(r);
                }
            }
            // writes, accesses: every block of the region (own and callee)
            std::set<uint32_t> all(own);
            all.insert(callee.begin(), callee.end());
            uint32_t writes[32] = {0};
            for (uint32_t h : all) {
                const Block &b = *blk[h];
                for (uint32_t hh : b.insts) {
                    std::string e;
                    uint32_t sz;
                    int sx;
                    const char *cond;
                    const PreInst &p = pre[hh];
                    const Cls k = classify(p, e, sz, sx, cond);
                    if ((k == C_ALU || k == C_LOAD || k == C_JAL) && p.rd) writes[p.rd]++;
                }
            }
            if (writes[rc] != 1 || writes[rl] != 0) continue;
            {   // ra: written only by the calls (one jal per call site)
                uint32_t jals = 0;
                for (uint32_t h : own) {
                    const Block &b = *blk[h];
                    const PreInst &lp = pre[b.insts.back()];
                    if (lp.op == OP_jal && lp.rd == 1) jals++;
                }
                if (writes[1] != jals) continue;
            }
            // the accesses: a register the region never writes + a bounded offset
            std::vector<ProofLoad> acc;
            for (uint32_t h : all) {
                const Block &b = *blk[h];
                AVal av[32];
                for (uint32_t r = 0; r < 32; r++) av[r] = writes[r] ? AVal{AV_TOP, 0, 0, 0} : AVal{AV_BND, r, 0, 0};
                for (size_t i = 0; i < b.insts.size() && ok; i++) {
                    std::string e;
                    uint32_t sz;
                    int sx;
                    const char *cond;
                    const PreInst &p = pre[b.insts[i]];
                    const Cls k = classify(p, e, sz, sx, cond);
                    const AVal A = av[p.rs1], B = av[p.rs2];
                    const int64_t imm = p.imm;
                    if (k == C_LOAD || k == C_STORE) {
                        if (A.k != AV_BND || !A.base || A.hi - A.lo >= (1 << 20) || A.lo + imm <= -((int64_t)1 << 31) ||
                            A.lo + imm >= ((int64_t)1 << 31)) { ok = false; break; }
                        const ProofLoad l{A.base, k == C_STORE ? 5u : 1u, sz, 0u, A.lo + imm, (uint64_t)(A.hi - A.lo)};
                        bool dup = false;
                        for (ProofLoad &q : acc)
                            if (q.reg == l.reg && q.kind == l.kind && q.off == l.off && q.span == l.span) {
                                q.size = std::max(q.size, l.size);
                                dup = true;
                            }
                        if (!dup) acc.push_back(l);
                        if (k == C_LOAD && p.rd) av[p.rd] = AVal{AV_TOP, 0, 0, 0};
                        continue;
                    }
                    if (!p.rd || (k != C_ALU && k != C_JAL)) continue;
                    AVal v{AV_TOP, 0, 0, 0};
                    if (k == C_ALU) switch (p.op) {
                    case OP_addi: case OP_c_addi: case OP_c_addi4spn: case OP_c_addi16sp: v = av_add(A, av_const(imm, imm)); break;
                    case OP_add: case OP_c_add: v = av_add(A, B); break;
                    case OP_c_mv: v = B; break;
                    case OP_andi: case OP_c_andi: if (imm >= 0) v = av_const(0, imm); break;
                    case OP_c_zext_b: v = av_const(0, 0xFF); break;
                    case OP_c_zext_h: v = av_const(0, 0xFFFF); break;
                    case OP_slli: case OP_c_slli: v = av_shl(A, imm); break;
                    case OP_srli: case OP_c_srli: if (imm >= 44 && imm < 64) v = av_const(0, (int64_t)((1ULL << (64 - imm)) - 1)); break;
                    case OP_sh1add: v = av_add(av_shl(A, 1), B); break;
                    case OP_sh2add: v = av_add(av_shl(A, 2), B); break;
                    case OP_sh3add: v = av_add(av_shl(A, 3), B); break;
                    case OP_c_li: case OP_lui: v = av_const(imm, imm); break;
                    default: break;
                    }
                    av[p.rd] = v;
                }
                if (!ok) break;
            }
            if (!ok || acc.empty() || acc.size() > 4) continue;
            // m: the shortest pass, H around to E's end (callee included)
            std::map<uint32_t, uint32_t> dist;
            std::set<std::pair<uint32_t, uint32_t>> q;
            dist[H] = (uint32_t)blk[H]->insts.size();
            q.insert({dist[H], H});
            uint32_t m = 0;
            while (!q.empty()) {
                const auto [d, v] = *q.begin();
                q.erase(q.begin());
                if (d != dist[v]) continue;
                if (v == E.h0) { m = d; break; }
                for (uint32_t t : nxt[v]) {
                    if (t == H) continue;
                    const uint32_t nd = d + (uint32_t)blk[t]->insts.size();
                    if (!dist.count(t) || nd < dist[t]) { dist[t] = nd; q.insert({nd, t}); }
                }
            }
            if (!m) continue;
            HangProof P{rc, rl, c, m, acc, true};
            for (uint32_t h : own)
                if (!hang_proof.count(h)) hang_proof[h] = P;
        }
    }

    // ---- clean body budget tests.  Only a check point tests the budget: a
    // top-level block or a cycle header (the dispatch and the back edges enter
    // those), or a block routed to through its headers (the routing tests it).
    // The test covers the longest run of direct edges through blocks that are
    // not check points (the blocks inside a cycle below its header), so a loop
    // iteration tests once.  (A test that fails leaves with the budget not
    // spent; the kernel then interprets up to its event, fi_trial.hip.)
    std::map<uint32_t, uint32_t> run_len;   // instructions from a block to the next check point
    std::set<uint32_t> forced_cp;
    auto is_cp = [&](uint32_t h) { return forced_cp.count(h) || !(S.chain.count(h) && !S.headers.count(h)); };
    {
        std::map<uint32_t, const Block *> blk;
        for (const Block &b : blocks)
            if (b.opc == 0) blk[b.h0] = &b;
        auto direct_succ = [&](const Block &b) {
            std::vector<uint32_t> r;
            auto add = [&](uint64_t pc) {
                uint32_t t;
                if (hof(pc, t) && !S.exits.count({b.h0, t})) r.push_back(t);
            };
            for (uint32_t h : b.insts) {
                std::string e;
                uint32_t sz;
                int sx;
                const char *cond;
                const PreInst &p = pre[h];
                const uint64_t pc = text_lo + 2ULL * h;
                const Cls k = classify(p, e, sz, sx, cond);
                if (k == C_BR) { add(pc + (int64_t)p.imm); add(pc + p.len); }
                if (k == C_JAL) add(pc + (int64_t)p.imm);
            }
            if (!b.term && !b.insts.empty()) add(text_lo + 2ULL * b.insts.back() + pre[b.insts.back()].len);
            return r;
        };
        std::set<uint32_t> on_path;
        std::function<uint32_t(uint32_t)> longest = [&](uint32_t h) -> uint32_t {
            auto it = run_len.find(h);
            if (it != run_len.end()) return it->second;
            auto bi = blk.find(h);
            if (bi == blk.end()) return 0;
            on_path.insert(h);
            uint32_t best = 0;
            for (uint32_t t : direct_succ(*bi->second)) {
                if (is_cp(t)) continue;
                if (on_path.count(t)) { forced_cp.insert(t); continue; }   // (defensive: a cycle of non-headers)
                best = std::max(best, longest(t));
            }
            on_path.erase(h);
            return run_len[h] = (uint32_t)bi->second->insts.size() + best;
        };
        for (const Block &b : blocks)
            if (b.opc == 0) longest(b.h0);
        if (!forced_cp.empty()) {   // recompute with those as check points
            run_len.clear();
            for (const Block &b : blocks)
                if (b.opc == 0) longest(b.h0);
        }
    }

    g.put("tx_dispatch: {\n  const uint64_t off_ = spc - 0x%llxULL;\n", (unsigned long long)text_lo);
    g.put("  if ((off_ >> 32) != 0 || (off_ & 1)) goto tx_out;\n  switch ((uint32_t)off_ >> 1) {\n");
    for (uint32_t h : leaders) {
        auto it = S.chain.find(h);
        if (it == S.chain.end() || (it->second.size() == 1 && it->second[0] == h)) g.put("  case %u: goto B_%u;\n", h, h);
        else g.put("  case %u: etgt = %uu; goto B_%u;\n", h, h, it->second[0]);
    }
    g.put("  default: goto tx_out;\n  }\n}\n");
    // the clean body's loop-proof test on entering block h ("" if none)
    auto proof_test = [&](uint32_t h) {
        auto hp = hang_proof.find(h);
        if (hp == hang_proof.end()) return std::string();
        const HangProof &P = hp->second;
        const std::string x = P.treg ? sfmt("X%u - X%u", P.reg, P.treg) : sfmt("X%u", P.reg);
        const uint32_t lp = P.reg | P.treg << 8 | (uint32_t)(uint8_t)(int8_t)P.step << 16 | (P.rel ? 1u << 24 : 0u);
        std::string r = P.rel ? sfmt("if (TXHANGU(X%u, X%u, %d, %uu)) { spc = %s; hang = 1u; TXLOOP(%uu, %uu, %uu); ", P.reg,
                                     P.treg, P.step, P.m, hex(g.pc_of(h)).c_str(), lp, P.m, (uint32_t)P.loads.size())
                              : sfmt("if (TXHANG(%s, %d, %uu)) { spc = %s; hang = 1u; TXLOOP(%uu, %uu, %uu); ", x.c_str(),
                                     P.step, P.m, hex(g.pc_of(h)).c_str(), lp, P.m, (uint32_t)P.loads.size());
        for (size_t j = 0; j < P.loads.size(); j++) {
            const ProofLoad &l = P.loads[j];
            r += sfmt("TXLD(%u, %uu, %d, %uu); ", (uint32_t)j, l.reg | l.kind << 8 | l.size << 12 | l.pos << 16,
                      (int)l.off, (uint32_t)l.span);
        }
        return r + "goto S_out; } ";
    };
    // solo dispatch (plain or with the odd-pc entries)
    auto sdispatch = [&](Gen &sx, bool clean) {
        sx.put("%s: {\n  const uint64_t off_ = spc - 0x%llxULL;\n", SD.c_str(), (unsigned long long)text_lo);
        if (!oddon) {
            sx.put("  if ((off_ >> 32) != 0 || (off_ & 1)) goto S_out;\n  switch ((uint32_t)off_ >> 1) {\n");
        } else {
            sx.put("  if ((off_ >> 32) != 0) goto S_out;\n  if (off_ & 1) switch ((uint32_t)off_ >> 1) {\n");
            for (uint64_t pc : olead) {
                const uint32_t i = (uint32_t)((pc - text_lo) >> 1);
                sx.put("  case %u: goto %s%u;\n", i, SOB.c_str(), i);
            }
            sx.put("  default: goto S_out;\n  }\n  switch ((uint32_t)off_ >> 1) {\n");
        }
        for (uint32_t h : leaders) {
            auto it = S.chain.find(h);
            sx.put("  case %u: ", h);
            if (clean) sx.out += proof_test(h);
            if (it == S.chain.end() || (it->second.size() == 1 && it->second[0] == h))
                sx.put("goto %s%u;\n", SB.c_str(), h);
            else
                sx.put("etgt = %uu; eon = 1; goto %s%u;\n", h, SB.c_str(), it->second[0]);
        }
        sx.put("  default: goto S_out;\n  }\n}\n");
    };

    // mode 0: the 64-lane body and the plain solo body (even blocks); mode 1:
    // the solo-odd body (even and odd blocks; its wave text is dropped)
    for (int mode = 0; mode < 2; mode++) {
    oddon = mode == 1;
    if (oddon && odd.empty()) break;
    SB = oddon ? "Q_" : "S_"; SD = oddon ? "Q_dispatch" : "S_dispatch"; SOB = oddon ? "QO_" : "SO_";
    Gen &so_ = oddon ? sq : so;
    std::string g_mode;
    if (oddon) g_mode.swap(g.out);
    sdispatch(so_, false);
    if (!oddon) sdispatch(sc, true);
    // text that the full and the clean solo bodies share (mode 0)
    auto sboth = [&](const std::string &t) { so_.out += t; if (!oddon) sc.out += t; };
    for (const Block &b : blocks) {
        if (!oddon && b.opc != 0) continue;
        const uint32_t h0 = b.h0;
        const std::vector<uint32_t> &insts = b.insts;
        const uint32_t n = (uint32_t)insts.size();
        if (!oddon || b.opc != 0) n_insts += n;
        cur_odd = b.opc != 0;
        std::string g_keep;   // an odd-pc block has no wave form: its wave text is dropped
        if (cur_odd) g_keep.swap(g.out);
        const uint64_t pc0 = cur_odd ? b.opc : g.pc_of(h0);
        const std::string P0 = hex(pc0);
        uint32_t rw = 0;   // registers the block reads or writes (watch check)
        for (uint32_t hh : insts) {
            const PreInst &p = pre[hh];
            if ((p.flags & kPreRs1) && p.rs1) rw |= 1u << p.rs1;
            if ((p.flags & kPreRs2) && p.rs2) rw |= 1u << p.rs2;
            if ((p.flags & kPreRd) && p.rd) rw |= 1u << p.rd;
        }
        uint64_t blo = pc0 & ~3ULL, bhi = g.pc_of(insts.empty() ? h0 : insts.back()) + 6;
        if (cur_odd) {   // the bytes the keys cover
            blo = ~0ULL; bhi = 0;
            for (uint32_t hh : insts) {
                blo = std::min<uint64_t>(blo, g.pc_of(hh) & ~3ULL);
                bhi = std::max<uint64_t>(bhi, g.pc_of(hh) + 7);
            }
        }
        g.put("B_%u: { // pc 0x%llx, %u insts\n", h0, (unsigned long long)pc0, n);
        if (cur_odd)
            so_.put("%s%u: { // pc 0x%llx (odd)\n", SOB.c_str(), (uint32_t)((pc0 - text_lo) >> 1),
                    (unsigned long long)pc0);
        else
            sboth(sfmt("%s%u: { // pc 0x%llx, %u insts\n", SB.c_str(), h0, (unsigned long long)pc0, n));
        if (!cur_odd && S.headers.count(h0)) {   // a cycle header routes an entry into its cycle one level on (etgt)
            std::string rw_, rs_, rc_;
            for (uint32_t x : leaders) {
                auto it = S.chain.find(x);
                if (it == S.chain.end() || x == h0) continue;
                const auto &ch = it->second;
                const auto pos = std::find(ch.begin(), ch.end(), h0);
                if (pos == ch.end()) continue;
                const uint32_t next = (pos + 1 != ch.end()) ? *(pos + 1) : x;
                // a nested header routes further, and clears etgt when it is the target
                const std::string clr = S.headers.count(next) ? "" : "etgt = 0xFFFFFFFFu; ";
                const std::string sclr = S.headers.count(next) ? "" : "eon = 0; ";
                rw_ += "case " + std::to_string(x) + ": " + clr + "goto B_" + std::to_string(next) + "; ";
                rs_ += "case " + std::to_string(x) + ": " + sclr + "goto " + SB + std::to_string(next) + "; ";
                // clean body: a routed block that is no check point tests the budget here
                const std::string chk = (!oddon && next == x && !is_cp(x))
                    ? sfmt("if (SOVER(%uu)) { spc = %s; bst = 1u; goto S_out; } ", run_len[x], hex(g.pc_of(x)).c_str())
                    : std::string();
                rc_ += "case " + std::to_string(x) + ": " + sclr + chk + "goto " + SB + std::to_string(next) + "; ";
            }
            const char *fmt = "  if (etgt != 0xFFFFFFFFu) { if (etgt == %uu) etgt = 0xFFFFFFFFu; "
                              "else switch (etgt) { %sdefault: break; } }\n";
            // solo: a separate pending flag (eon), opaque at every header --
            // otherwise the compiler threads each back edge through a switch
            // on etgt, a compare tree per loop iteration
            const char *sfm = "  ETGT_OPAQUE(); if (__builtin_expect(eon != 0, 0)) { if (etgt == %uu) eon = 0; "
                              "else switch (etgt) { %sdefault: break; } }\n";
            g.put(fmt, h0, rw_.c_str());
            so_.put(sfm, h0, rs_.c_str());
            if (!oddon) sc.put(sfm, h0, rc_.c_str());
        }
        // ---- wave block prologue: merge a parked group waiting here, leave or
        // switch groups when lanes outside run first, then one combined check
        // (budget, watched registers, rewritten bytes)
        g.put("  if (!ult64(%s, wmin)) {\n    if (%s == pmin && ult64(pmin, owm)) TXMERGE(%s);\n"
              "    else { spc = %s; goto tx_sched; }\n  }\n", P0.c_str(), P0.c_str(), P0.c_str(), P0.c_str());
        g.put("  if (((wst + %uu > ubud) & ((wst + %uu > wbud) | (TXB(mine && rem - lst < %uu) != 0)))", n, n, n);
        if (rw) g.put(" |\n      (wwatch & (TXB(mine && (lwm & 0x%xu) != 0) != 0))", rw);
        g.put(" |\n      (wdirty & (TXB(mine && ldlo < %s && ldhi > %s) != 0))) { spc = %s; goto tx_out; }\n",
              hex(bhi).c_str(), hex(blo).c_str(), P0.c_str());
        // ---- solo block prologue: one uniform check
        so_.put("  if ((st + %uu > bud)", n);
        if (rw) so_.put(" | ((lwm & 0x%xu) != 0)", rw);
        so_.put(" | SDIRTY(%uu, %uu)) { spc = %s; goto S_out; }\n", (uint32_t)(blo - text_lo),
                (uint32_t)(bhi - text_lo), P0.c_str());
        if (!oddon && is_cp(h0)) sc.put("  if (SOVER(%uu)) { spc = %s; bst = 1u; goto S_out; }\n", run_len[h0], P0.c_str());
        uint32_t k_st = 0, k_xt = 0, k_fb = 0, k_db = 0;   // committed so far in this block
        auto commit = [&](uint32_t st, uint32_t xt, uint32_t fb, uint32_t db) {
            // per-lane counters of the running lanes (zero terms omitted), wave iterations
            if (!st) return std::string();
            std::string r = "{ const uint32_t mm_ = mine ? 0xFFFFFFFFu : 0u; lst += " + std::to_string(st) + "u & mm_; ";
            if (xt) r += "lxt += " + std::to_string(xt) + "u & mm_; ";
            if (fb) r += "lfb += " + std::to_string(fb) + "u & mm_; ";
            if (db) r += "ldb += " + std::to_string(db) + "u & mm_; ";
            return r + "wst = uni32(wst + " + std::to_string(st) + "u); } ";
        };
        auto scommit = [&](uint32_t st, uint32_t xt, uint32_t fb, uint32_t db) {
            if (!st) return std::string();
            std::string r = "SADD(" + std::to_string(st) + "u); ";
            if (xt) r += "xt += " + std::to_string(xt) + "u; ";
            if (fb) r += "fb += " + std::to_string(fb) + "u; ";
            if (db) r += "db += " + std::to_string(db) + "u; ";
            return r;
        };
        for (uint32_t i = 0; i < n; i++) {
            const PreInst &p = pre[insts[i]];
            const uint64_t pc = cur_odd ? b.opcs[i] : g.pc_of(insts[i]);
            const uint64_t ft = pc + p.len;
            std::string e;
            uint32_t sz;
            int sx;
            const char *cond;
            const Cls k = classify(p, e, sz, sx, cond);
            const std::string A = Gen::R(p.rs1), B = Gen::R(p.rs2);
            char immb[48];
            snprintf(immb, sizeof immb, "((uint64_t)(int64_t)%dLL)", p.imm);
            const std::string pcb = hex(pc), ftb = hex(ft);
            const uint32_t xt = (p.flags & kPreStraddle) ? 1 : 0;
            const std::string leave_here = "{ " + commit(k_st, k_xt, k_fb, k_db) + "spc = " + pcb + "; goto tx_out; }";
            const std::string sleave_here = "{ " + scommit(k_st, k_xt, k_fb, k_db) + "spc = " + pcb + "; goto S_out; }";
            switch (k) {
            case C_ALU: {
                const std::string v = subst(e, A, B, immb, pcb);
                if (p.rd) {
                    g.put("  TXSET(%u, %s);\n", p.rd, v.c_str());
                    sboth(sfmt("  SX(%u, %s);\n", p.rd, v.c_str()));
                }
                break;
            }
            case C_NOP:
                break;
            case C_LOAD:
                g.put("  { uint8_t *p_; const bool ok_ = tx_probe(m, %s + %s, %uu, false, p_, tx);\n", A.c_str(), immb, sz);
                g.put("    if (TXB(mine && !ok_)) %s\n", leave_here.c_str());
                // (solo: pages the trial has not copied through the scalar cache)
                {
                    const std::string pl = sfmt("  { uint8_t *p_; bool pv_; if (SCOND(!tx_probe_ld(m, %s + %s, %uu, p_, pv_))) %s\n",
                                                A.c_str(), immb, sz, sleave_here.c_str());
                    so_.out += pl;
                    if (!oddon) {
                        if (S.chain.count(h0) && n_sites < kSiteCaches) {
                            const uint32_t i = n_sites++;
                            sc.put("  { uint8_t *p_; bool pv_; const uint64_t ea_ = %s + %s, vp_ = ea_ >> 12;\n"
                                   "    if (%s(vp_ != CV%u)) { const uint64_t e_ = tlb_find(m, vp_); if (SCOND(!e_)) %s "
                                   "SC_SET(%u, vp_, e_); }\n", A.c_str(), immb, cold, i, sleave_here.c_str(), i);
                            if (sz > 1)
                                sc.put("    if (%s(((uint32_t)ea_ & 4095u) > %uu)) %s\n", cold, 4096u - sz, sleave_here.c_str());
                            sc.put("    p_ = SC_PTR(%u, ea_); pv_ = SC_PRIV(%u);\n", i, i);
                        } else {
                            sc.out += pl;
                        }
                    }
                }
                if (p.rd) {
                    g.put("    p_ = ok_ ? p_ : const_cast<uint8_t *>(zp);\n");
                    sboth(sfmt("    uint64_t v_; if (SPRIV(pv_)) v_ = *(const g_%s *)p_; else v_ = tx_sload(p_, %uu);\n",
                               gtype(sz), sz));
                    if (sx) {
                        g.put("    TXSET(%u, (int64_t)(int%d_t)*(const g_%s *)p_); }\n", p.rd, sx, gtype(sz));
                        sboth(sfmt("    X%u = (uint64_t)(int64_t)(int%d_t)v_; }\n", p.rd, sx));
                    } else {
                        g.put("    TXSET(%u, *(const g_%s *)p_); }\n", p.rd, gtype(sz));
                        sboth(sfmt("    X%u = v_; }\n", p.rd));
                    }
                } else {
                    g.put("  }\n");
                    sboth("  }\n");
                }
                break;
            case C_STORE:
                g.put("  { uint8_t *p_; const bool ok_ = tx_probe(m, %s + %s, %uu, true, p_, tx);\n", A.c_str(), immb, sz);
                g.put("    if (TXB(mine && !ok_)) %s\n", leave_here.c_str());
                g.put("    p_ = (mine && ok_) ? p_ : sink; *(g_%s *)p_ = (%s)%s; }\n", gtype(sz), ltype(sz), B.c_str());
                // solo: a store into the code range is performed too; it marks the
                // bytes rewritten and leaves after itself if they lie ahead in this block
                // (a code-range store that leaves the bytes as they were rewrites nothing)
                so_.put("  { uint8_t *p_; const uint64_t ea_ = %s + %s; const uint32_t cs_ = tx_probe_st(m, ea_, %uu, "
                       "p_, tx); if (SCOND(!cs_)) %s\n", A.c_str(), immb, sz, sleave_here.c_str());
                so_.put("    const bool chg_ = SCOND(cs_ & 2u) && SUNI((uint64_t)*(g_%s *)p_) != (uint64_t)(%s)%s;\n", gtype(sz),
                        ltype(sz), B.c_str());
                so_.put("    *(g_%s *)p_ = (%s)%s;\n", gtype(sz), ltype(sz), B.c_str());
                so_.put("    if (SCOND(chg_)) { TXCODE(ea_, %uu); if (SCOND(ea_ < %s && ea_ + %uu > %s)) { %sspc = %s; "
                       "goto S_out; } } }\n", sz, hex(bhi).c_str(), sz, ftb.c_str(),
                       scommit(k_st + 1, k_xt + xt, k_fb + p.len, k_db + sz).c_str(), ftb.c_str());
                // clean: a store into the code range (or any the probe refuses) leaves before itself
                if (!oddon) {
                    if (S.chain.count(h0) && n_sites < kSiteCaches) {
                        const uint32_t i = n_sites++;
                        // (a page meeting the code range is never cached: every store probes it)
                        sc.put("  { uint8_t *p_; const uint64_t ea_ = %s + %s, vp_ = ea_ >> 12;\n"
                               "    if (SCOND(vp_ == CV%u)) {\n", A.c_str(), immb, i);
                        if (sz > 1)
                            sc.put("      if (SCOND(((uint32_t)ea_ & 4095u) > %uu)) %s\n", 4096u - sz, sleave_here.c_str());
                        sc.put("      p_ = SC_PTR(%u, ea_);\n"
                               "    } else {\n      const uint64_t e_ = tlb_find(m, vp_);\n"
                               "      if (SCOND(!tx_probe_st_e(e_, ea_, %uu, p_, tx))) %s\n"
                               "      if (SCOND((vp_ << 12) >= tx.chi || ((vp_ + 1) << 12) <= tx.clo)) SC_SET(%u, vp_, e_);\n"
                               "    }\n    *(g_%s *)p_ = (%s)%s; }\n", i, sz, sleave_here.c_str(), i, gtype(sz), ltype(sz),
                               B.c_str());
                    } else {
                        sc.put("  { uint8_t *p_; if (SCOND(!tx_probe(m, %s + %s, %uu, true, p_, tx))) %s\n"
                               "    *(g_%s *)p_ = (%s)%s; }\n", A.c_str(), immb, sz, sleave_here.c_str(), gtype(sz),
                               ltype(sz), B.c_str());
                    }
                }
                break;
            case C_BR: {
                const std::string c = subst(cond, A, B, immb, pcb);
                const uint64_t tgt = pc + (int64_t)p.imm;
                g.put("  { const bool c_ = %s; const uint64_t tk_ = uni64(TXB(mine && c_));\n", c.c_str());
                g.put("    %s\n", commit(k_st + 1, k_xt + xt, k_fb + p.len, k_db).c_str());
                g.put("    if (tk_ == gmr) %s\n", wgo(h0, tgt).c_str());
                g.put("    if (tk_ == 0) %s\n", wgo(h0, ft).c_str());
                // divergent: the lanes bound for the higher pc park, the others run on
                if (tgt > ft) {
                    g.put("    lp = (mine && c_) ? %s : lp; pend = uni64(pend | tk_); mine = mine && !c_;"
                          " gmr = uni64(gmr & ~tk_);\n", hex(tgt).c_str());
                    g.put("    pmin = uni64(ult64(%s, pmin) ? %s : pmin);"
                          " wmin = uni64(ult64(pmin, owm) ? pmin : owm);\n", hex(tgt).c_str(), hex(tgt).c_str());
                    g.put("    %s }\n", wgo(h0, ft).c_str());
                } else {
                    g.put("    lp = (mine && !c_) ? %s : lp; pend = uni64(pend | (gmr & ~tk_)); mine = mine && c_;"
                          " gmr = uni64(tk_);\n", ftb.c_str());
                    g.put("    pmin = uni64(ult64(%s, pmin) ? %s : pmin); wmin = uni64(ult64(pmin, owm) ? pmin : owm);\n",
                          ftb.c_str(), ftb.c_str());
                    g.put("    %s }\n", wgo(h0, tgt).c_str());
                }
                sboth(sfmt("  %s\n  if (SCOND(%s)) %s\n  %s\n", scommit(k_st + 1, k_xt + xt, k_fb + p.len, k_db).c_str(),
                         c.c_str(), sgo(h0, tgt).c_str(), sgo(h0, ft).c_str()));
                break;
            }
            case C_JAL: {
                const uint64_t tgt = pc + (int64_t)p.imm;
                if (p.rd) {
                    g.put("  TXSET(%u, %s);\n", p.rd, ftb.c_str());
                    sboth(sfmt("  SX(%u, %s);\n", p.rd, ftb.c_str()));
                }
                g.put("  %s %s\n", commit(k_st + 1, k_xt + xt, k_fb + p.len, k_db).c_str(), wgo(h0, tgt).c_str());
                sboth(sfmt("  %s %s\n", scommit(k_st + 1, k_xt + xt, k_fb + p.len, k_db).c_str(), sgo(h0, tgt).c_str()));
                break;
            }
            case C_JALR: {
                const int64_t im = (p.op == OP_jalr) ? p.imm : 0;
                const uint32_t rd = (p.op == OP_c_jalr) ? 1 : (p.op == OP_c_jr ? 0 : p.rd);
                g.put("  { const uint64_t t_ = (%s + (uint64_t)(int64_t)%lldLL) & ~1ULL;\n", A.c_str(), (long long)im);
                if (rd) g.put("    TXSET(%u, %s);\n", rd, ftb.c_str());
                g.put("    %s\n", commit(k_st + 1, k_xt + xt, k_fb + p.len, k_db).c_str());
                g.put("    const uint64_t t0_ = rdl64<kNL>(t_, __ffsll((unsigned long long)gmr) - 1);\n");
                g.put("    if (TXB(mine && t_ != t0_)) { dpc = t_; jdiv = mine; goto tx_out; }\n");
                g.put("    spc = uni64(t0_); goto tx_dispatch; }\n");
                sboth(sfmt("  { const uint64_t t_ = (%s + (uint64_t)(int64_t)%lldLL) & ~1ULL;\n", A.c_str(), (long long)im));
                if (rd) sboth(sfmt("    SX(%u, %s);\n", rd, ftb.c_str()));
                sboth(sfmt("    %s spc = SUNI(t_); goto %s; }\n", scommit(k_st + 1, k_xt + xt, k_fb + p.len, k_db).c_str(),
                         SD.c_str()));
                break;
            }
            default:
                break;
            }
            k_st += 1; k_xt += xt; k_fb += p.len; k_db += (k == C_LOAD || k == C_STORE) ? sz : 0;
        }
        if (!b.term) {   // fell into the next leader, or stops before an instruction it does not cover
            const uint64_t nxt = cur_odd ? (n ? b.opcs[n - 1] + pre[insts[n - 1]].len : pc0)
                                         : n ? g.pc_of(insts[n - 1]) + pre[insts[n - 1]].len : pc0;
            g.put("  %s %s\n", commit(k_st, k_xt, k_fb, k_db).c_str(), wgo(h0, nxt).c_str());
            sboth(sfmt("  %s %s\n", scommit(k_st, k_xt, k_fb, k_db).c_str(), sgo(h0, nxt).c_str()));
        }
        g.put("}\n");
        sboth("}\n");
        if (cur_odd) g.out.swap(g_keep);
    }
    if (oddon) g.out.swap(g_mode);
    }
    cur_odd = false;
    leaders_out.assign(leaders.begin(), leaders.end());
    // odd-pc entries: bit 31 + the pre-decoded index of their key (kPreOddLeader)
    for (uint64_t pc : olead) leaders_out.push_back(0x80000000u | okey(pc));
    // the clean body's entry: its site caches start empty (declared without an
    // initializer: the dispatch label below them is also a jump target)
    std::string sc_head;
    // the budget counts down (solo_tx_clean_run: SADD / SOVER / SDONE); cold hints
    sc_head += "#undef SADD\n#undef SOVER\n#undef SDONE\n#define SADD(n_) (brem -= (n_))\n"
               "#define SOVER(n_) __builtin_expect(brem < (n_), 0)\n#define SDONE() (bud - brem)\n"
               "#define SCOLD(x) __builtin_expect(!!(x), 0)\n";
    for (uint32_t i = 0; i < kSiteCaches; i++) sc_head += sfmt("  uint64_t CV%u, CP%u; uint32_t CQ%u;\n", i, i, i);
    sc_head += "S_entry:\n";
    for (uint32_t i = 0; i < kSiteCaches; i++) sc_head += sfmt("  CV%u = ~0ULL; CP%u = 0; CQ%u = 0;\n", i, i, i);
    sc_head += "  goto S_dispatch;\n";
    // the bodies' temporaries live at function scope (fi_trial.hip declares
    // them, TX_TEMPS): a goto out of a block that declares a variable leaves
    // through clang's lifetime cleanup switch -- a flag set, compared and
    // branched on at every exit test (crc32's clean loop: 38 -> 23 scalar
    // instructions per iteration, and loaded values stay in VGPRs)
    auto hoist = [](std::string t) {
        for (const auto &[from, to] : std::vector<std::pair<std::string, std::string>>{
                 {"uint8_t *p_; ", ""}, {"bool pv_; ", ""}, {"uint64_t v_; ", ""},
                 {", vp_ = ea_ >> 12;", "; vp_ = ea_ >> 12;"}, {"const uint64_t ea_ = ", "ea_ = "},
                 {"const uint64_t e_ = ", "e_ = "}, {"const uint64_t t_ = ", "t_ = "},
                 {"const uint64_t t0_ = ", "t0_ = "}, {"const uint64_t off_ = ", "off_ = "},
                 {"const uint32_t cs_ = ", "cs_ = "}, {"const bool chg_ = ", "chg_ = "},
                 {"const bool ok_ = ", "ok_ = "}, {"const bool c_ = ", "c_ = "},
                 {"const uint64_t tk_ = ", "tk_ = "}, {"const uint32_t mm_ = ", "mm_ = "}}) {
            for (size_t at = t.find(from); at != std::string::npos; at = t.find(from, at + to.size()))
                t.replace(at, from.size(), to);
        }
        return t;
    };
    // (the clean body only: hoisting the 64-lane body's doubles its spills
    // (intmix 183 -> 985 VGPRs), the full solo body's costs crc32 +3 % and
    // saves qsort 7 %: profiles/r06h_ab_hoist_scope_*.jsonl)
    return g.out + FI_TX_SPLIT + so.out + FI_TX_SPLIT + sq.out + FI_TX_SPLIT + sc_head + hoist(sc.out);
}

}  // namespace fi
