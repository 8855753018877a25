// Reader of gem5 SE-mode checkpoints (m5.cpt + physical memory store), the
// campaign start of SURVEY.md §8f2.  What gem5 writes, restated from the
// reference:
//   m5.cpt            INI: one [section] per SimObject path, key=value lines
//                     (src/sim/serialize.cc, paramOut / arrayParamOut:
//                     src/sim/serialize.hh:385-400, arrays space-separated,
//                     bytes as numbers: serialize_handlers.hh:130-140)
//   thread context    [<cpu>.xc.0] (BaseCPU::serialize, src/cpu/base.cc:739):
//                     regs.integer = 33 x 8 bytes (x0..x31 + the ureg temp,
//                     src/arch/riscv/regs/int.hh:62-80; serialize(tc),
//                     src/cpu/thread_context.cc:194-218), regs.floating_point,
//                     _pc (PCStateBase::serialize, src/arch/generic/pcstate.hh:143)
//   process           [<process>] MemState::serialize (src/sim/mem_state.hh:
//                     189-210): brkPoint, stackBase, stackSize, maxStackSize,
//                     stackMin, nextThreadStackBase, mmapEnd; [<process>.vmalist]
//                     size + [.VmaN] name/addrRangeStart/addrRangeEnd;
//                     [<process>.ptable] size + [.EntryN] vaddr/paddr/flags
//                     (EmulationPageTable::serialize, src/mem/page_table.cc:186-201)
//   memory            [<system>.physmem] nbr_of_stores + [.storeN] filename,
//                     range_size; the file is the store's bytes, gzip-compressed
//                     (PhysicalMemory::serializeStore, src/mem/physical.cc:363-405)
//   ISA               [<cpu>.isa] miscRegFile (fflags, frm); the PC state's
//                     _vtype/_vl (riscv/pcstate.hh:146-156); [Globals] curTick
//   fd table          [<process>.fdarray.EntryN] is deliberately NOT read for
//                     fds 0-2: FDArray::unserialize skips them
//                     (src/sim/fd_array.cc:378-381), and restoreFileOffsets
//                     (:126-282), the only code that would seek fd 0 to the
//                     checkpointed _fileOffset, has no caller in the reference
//                     tree.  A restored process's fd 0 is the one its
//                     FDArray constructor opened from Process.input
//                     (:50-75), at offset 0 -- what fi_load_checkpoint sets.
// Host code; the product reads what SE trials need: pages, integer and FP
// registers, fcsr, pc, brk point, the VMA list, mmap end and curTick.  Parity with a checkpoint written by a real
// gem5 is unpinned (no gem5 build here); the format is pinned by the
// oracle's writer (oracle/rv64se.c:or_write_checkpoint) and by round trips
// against runs from process start (tests/test_checkpoint.py).
#include <zlib.h>

#include "fi_checkpoint.h"

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

namespace fi {

namespace {

constexpr int kMiscFflags = 120, kMiscFrm = 121;   // MiscRegIndex: MISCREG_FFLAGS, MISCREG_FRM

using Ini = std::map<std::string, std::map<std::string, std::string>>;

bool read_ini(const std::string &path, Ini &ini) {
    std::ifstream f(path);
    if (!f) return false;
    std::string sec, line;
    while (std::getline(f, line)) {
        while (!line.empty() && (line.back() == '\r' || line.back() == '\n')) line.pop_back();
        if (line.empty() || line[0] == '#' || line[0] == ';') continue;
        if (line[0] == '[') {
            const size_t e = line.find(']');
            sec = line.substr(1, e == std::string::npos ? std::string::npos : e - 1);
            ini[sec];
            continue;
        }
        const size_t eq = line.find('=');
        if (eq != std::string::npos) ini[sec][line.substr(0, eq)] = line.substr(eq + 1);
    }
    return true;
}

bool get_u64(const std::map<std::string, std::string> &s, const char *k, uint64_t &v) {
    auto it = s.find(k);
    if (it == s.end()) return false;
    v = strtoull(it->second.c_str(), nullptr, 0);
    return true;
}

std::vector<uint8_t> byte_array(const std::string &v) {
    std::vector<uint8_t> out;
    std::istringstream is(v);
    unsigned x;
    while (is >> x) out.push_back((uint8_t)x);
    return out;
}

const std::string *find_section_with(const Ini &ini, const char *key) {
    for (auto &kv : ini)
        if (kv.second.count(key)) return &kv.first;
    return nullptr;
}

}  // namespace

std::string read_gem5_checkpoint(const std::string &dir, CptImage &img) {
    Ini ini;
    if (!read_ini(dir + "/m5.cpt", ini)) return "cannot read " + dir + "/m5.cpt";
    // thread context 0 of the (single) CPU
    const std::string *xc = find_section_with(ini, "regs.integer");
    if (!xc) return "no thread context (regs.integer) in m5.cpt";
    const auto &X = ini.at(*xc);
    const std::vector<uint8_t> ir = byte_array(X.at("regs.integer"));
    if (ir.size() < 32 * 8) return "regs.integer holds fewer than 32 registers";
    for (int r = 0; r < 32; r++) {
        uint64_t v = 0;
        for (int b = 0; b < 8; b++) v |= (uint64_t)ir[r * 8 + b] << (8 * b);
        img.regs[r] = r ? v : 0;
    }
    if (X.count("regs.floating_point")) {
        const std::vector<uint8_t> fr = byte_array(X.at("regs.floating_point"));
        for (size_t i = 0; i < fr.size() && i < 32 * 8; i++) img.fregs[i / 8] |= (uint64_t)fr[i] << (8 * (i % 8));
    }
    // fflags and frm: the ISA's misc registers (ISA::serialize, src/arch/riscv/
    // isa.cc:977-983, miscRegFile in MiscRegIndex order, regs/misc.hh;
    // indices pinned by tests/golden/riscv_miscreg.json)
    if (const std::string *is = find_section_with(ini, "miscRegFile")) {
        std::istringstream in(ini.at(*is).at("miscRegFile"));
        unsigned long long v;
        for (int i = 0; i <= kMiscFrm && (in >> v); i++) {
            if (i == kMiscFflags) img.fflags = (uint32_t)(v & 0x1F);
            if (i == kMiscFrm) img.frm = (uint32_t)(v & 7);
        }
    }
    for (uint64_t f : img.fregs) img.fp_state |= f != 0;
    img.fp_state |= img.fflags != 0 || img.frm != 0;
    // the vector configuration lives in the PC state (riscv/pcstate.hh:146-156):
    // only the process-start one (vtype.vill, vl = 0) is modelled
    uint64_t vt = 1ULL << 63, vlen = 0;
    get_u64(X, "_vtype", vt);
    get_u64(X, "_vl", vlen);
    if (vt != (1ULL << 63) || vlen != 0) return "vector configuration set (vtype/vl): not supported";
    if (!get_u64(X, "_pc", img.pc)) return "no _pc in " + *xc;
    auto gl = ini.find("Globals");
    if (gl != ini.end()) get_u64(gl->second, "curTick", img.tick0);
    // the process: MemState, VMA list, page table
    const std::string *ps = find_section_with(ini, "brkPoint");
    if (!ps) return "no process (brkPoint) in m5.cpt";
    const auto &P = ini.at(*ps);
    if (!get_u64(P, "brkPoint", img.brk) || !get_u64(P, "stackBase", img.stack_base) ||
        !get_u64(P, "stackSize", img.stack_size) || !get_u64(P, "maxStackSize", img.max_stack) ||
        !get_u64(P, "stackMin", img.stack_min) || !get_u64(P, "mmapEnd", img.mmap_end))
        return "incomplete MemState in " + *ps;
    uint64_t nv = 0;
    auto vl = ini.find(*ps + ".vmalist");
    if (vl != ini.end()) get_u64(vl->second, "size", nv);
    for (uint64_t i = 0; i < nv; i++) {
        auto v = ini.find(*ps + ".vmalist.Vma" + std::to_string(i));
        if (v == ini.end()) return "missing VMA " + std::to_string(i);
        uint64_t lo = 0, hi = 0;
        get_u64(v->second, "addrRangeStart", lo);
        get_u64(v->second, "addrRangeEnd", hi);
        img.vmas.emplace_back(lo, hi);
        img.vma_names.push_back(v->second.count("name") ? v->second.at("name") : "");
    }
    uint64_t np = 0;
    auto pt = ini.find(*ps + ".ptable");
    if (pt == ini.end() || !get_u64(pt->second, "size", np)) return "no page table in " + *ps;
    std::vector<std::pair<uint64_t, uint64_t>> map;   // (paddr, vpn)
    for (uint64_t i = 0; i < np; i++) {
        auto en = ini.find(*ps + ".ptable.Entry" + std::to_string(i));
        if (en == ini.end()) return "missing page-table entry " + std::to_string(i);
        uint64_t va = 0, pa = 0;
        if (!get_u64(en->second, "vaddr", va) || !get_u64(en->second, "paddr", pa)) return "bad page-table entry";
        if ((va | pa) & 4095) return "page-table entry not page aligned";
        map.emplace_back(pa, va >> 12);
    }
    // physical memory: one store, gzip-compressed, its bytes from address 0
    const std::string *pm = find_section_with(ini, "nbr_of_stores");
    if (!pm) return "no physical memory (nbr_of_stores) in m5.cpt";
    auto st = ini.find(*pm + ".store0");
    if (st == ini.end() || !st->second.count("filename")) return "no store0 in " + *pm;
    uint64_t range = 0;
    get_u64(st->second, "range_size", range);
    gzFile gz = gzopen((dir + "/" + st->second.at("filename")).c_str(), "rb");
    if (!gz) return "cannot open " + st->second.at("filename");
    std::sort(map.begin(), map.end());
    uint64_t at = 0;
    std::vector<uint8_t> skip(1 << 16);
    std::string err;
    for (auto &m : map) {
        if (m.first + 4096 > range) { err = "page-table entry beyond the memory store"; break; }
        while (at < m.first) {   // stream forward to the frame
            const unsigned n = (unsigned)std::min<uint64_t>(skip.size(), m.first - at);
            if (gzread(gz, skip.data(), n) != (int)n) { err = "memory store truncated"; break; }
            at += n;
        }
        if (!err.empty()) break;
        std::vector<uint8_t> pg(4096);
        if (at == m.first) {
            if (gzread(gz, pg.data(), 4096) != 4096) { err = "memory store truncated"; break; }
            at += 4096;
        } else {   // two virtual pages on one frame
            err = "frame mapped twice (shared frames are not supported)";
            break;
        }
        img.pages[m.second] = std::move(pg);
    }
    gzclose(gz);
    return err;
}

}  // namespace fi
