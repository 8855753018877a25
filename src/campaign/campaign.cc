// campaign.cc -- see campaign.hh.
#include "campaign.hh"

#include <chrono>
#include <climits>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <thread>

namespace shrewd {

namespace {

const char *kClass[FI_N_CLASS] = {"masked", "sdc", "crash", "hang", "detected", "escape"};
// sub-code names (include/fi_engine.h FI_CRASH_* / FI_ESC_*; the same as
// shrewd_amd/fi.py CRASH_NAMES / ESCAPE_NAMES)
const char *kCrash[] = {"", "panic_unknown_inst", "panic_illegal_inst", "panic_page_fault", "fatal_syscall_range",
                        "fatal_syscall_unimpl", "fatal_proxy", "abort_fd_assert", "sigtrap", "fatal_stack_limit",
                        "panic_amo_line", "abort_sc_line", "panic_se_handler", "panic_m5op",
                        "abort_vset_sew"};
const char *kEscape[] = {"", "inst", "syscall", "csr", "host", "resource", "undefined", "timing"};
constexpr int kNCrash = sizeof(kCrash) / sizeof(kCrash[0]);
constexpr int kNEscape = sizeof(kEscape) / sizeof(kEscape[0]);
static_assert(kNCrash == FI_CRASH_VSET_SEW + 1 && kNEscape == FI_ESC_TIMING + 1, "sub-code names");

void check(fi_engine *e, fi_status s, const char *what) {
    if (s != FI_OK) {
        std::string msg = std::string(what) + ": " + fi_last_error(e);
        throw std::runtime_error(msg);
    }
}

std::vector<uint8_t> read_file(const std::string &path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open workload " + path);
    return std::vector<uint8_t>(std::istreambuf_iterator<char>(f), {});
}

void hist_add(fi_histogram &a, const fi_histogram &b) {
    const uint64_t *src = reinterpret_cast<const uint64_t *>(&b);
    uint64_t *dst = reinterpret_cast<uint64_t *>(&a);
    for (size_t i = 0; i < sizeof(fi_histogram) / 8; i++) dst[i] += src[i];
}

}  // namespace

uint64_t structures_mask(const std::vector<std::string> &names) {
    static const std::map<std::string, int> abi = {
        {"zero", 0}, {"ra", 1}, {"sp", 2}, {"gp", 3}, {"tp", 4}, {"t0", 5}, {"t1", 6}, {"t2", 7},
        {"s0", 8}, {"fp", 8}, {"s1", 9}, {"a0", 10}, {"a1", 11}, {"a2", 12}, {"a3", 13}, {"a4", 14},
        {"a5", 15}, {"a6", 16}, {"a7", 17}, {"s2", 18}, {"s3", 19}, {"s4", 20}, {"s5", 21}, {"s6", 22},
        {"s7", 23}, {"s8", 24}, {"s9", 25}, {"s10", 26}, {"s11", 27}, {"t3", 28}, {"t4", 29}, {"t5", 30},
        {"t6", 31}};
    uint64_t m = 0;
    for (std::string s : names) {
        for (auto &ch : s) ch = (char)tolower((unsigned char)ch);
        if (s == "int_reg" || s == "intreg" || s == "regs" || s == "regfile") {
            m |= 0xFFFFFFFEULL;
        } else if (s == "pc") {
            m |= 1ULL << FI_T_PC;
        } else if (s == "mem" || s == "memory") {
            m |= 1ULL << FI_T_MEM;
        } else if (s == "result" || s == "fu" || s == "inst_result") {
            m |= 1ULL << FI_T_RESULT;
        } else if (abi.count(s)) {
            m |= 1ULL << abi.at(s);
        } else if (s.size() > 1 && s[0] == 'x' && s.find_first_not_of("0123456789", 1) == std::string::npos &&
                   std::stoi(s.substr(1)) < 32) {
            m |= 1ULL << std::stoi(s.substr(1));
        } else {
            throw std::runtime_error("unknown fault structure '" + s + "'");
        }
    }
    return m & ~1ULL;
}

uint64_t bits_mask(const std::string &spec) {
    if (spec.empty()) return ~0ULL;
    if (spec.find_first_of(",-") == std::string::npos) return std::stoull(spec, nullptr, 0);
    uint64_t m = 0;
    size_t pos = 0;
    while (pos <= spec.size()) {
        const size_t end = std::min(spec.find(',', pos), spec.size());
        const std::string part = spec.substr(pos, end - pos);
        pos = end + 1;
        if (part.empty()) continue;
        const size_t dash = part.find('-');
        const unsigned long lo = std::stoul(part.substr(0, dash), nullptr, 0);
        const unsigned long hi = dash == std::string::npos ? lo : std::stoul(part.substr(dash + 1), nullptr, 0);
        if (lo > hi || hi > 63) throw std::runtime_error("bad bit range '" + part + "'");
        for (unsigned long b = lo; b <= hi; b++) m |= 1ULL << b;
    }
    return m;
}

// gem5 OpClass names (src/cpu/FuncUnit.py:43) -> mask of enum values; a bare
// number is taken as the enum value
uint64_t opclass_mask(const std::vector<std::string> &names) {
    static const std::map<std::string, int> cls = {
        {"No_OpClass", 0}, {"IntAlu", 1}, {"IntMult", 2}, {"IntDiv", 3}, {"FloatAdd", 4}, {"FloatCmp", 5},
        {"FloatCvt", 6}, {"FloatMult", 7}, {"FloatMultAcc", 8}, {"FloatDiv", 9}, {"FloatMisc", 10},
        {"FloatSqrt", 11}, {"MemRead", 52}, {"MemWrite", 53}, {"FloatMemRead", 54}, {"FloatMemWrite", 55}};
    uint64_t m = 0;
    for (std::string s : names) {
        if (s.size() > 2 && s.compare(s.size() - 2, 2, "Op") == 0) s.resize(s.size() - 2);
        if (cls.count(s)) m |= 1ULL << cls.at(s);
        else if (!s.empty() && s.find_first_not_of("0123456789") == std::string::npos && std::stoi(s) < 64)
            m |= 1ULL << std::stoi(s);
        else throw std::runtime_error("unknown OpClass '" + s + "'");
    }
    return m;
}

Campaign::Campaign(const CampaignParams &p) : p_(p) {
    if (p_.cmd.empty()) p_.cmd.push_back(p_.workload);
    if (p_.num_gpus == 0 && p_.devices.empty()) throw std::runtime_error("num_gpus must be >= 1");
    const std::vector<uint8_t> elf = read_file(p_.workload);
    std::vector<const char *> argv, envp;
    for (auto &s : p_.cmd) argv.push_back(s.c_str());
    argv.push_back(nullptr);
    for (auto &s : p_.env) envp.push_back(s.c_str());
    envp.push_back(nullptr);
    const uint64_t smask = structures_mask(p_.structures);
    // Process.input: the stdio names are the host's stdin (fd_array.cc:50-75),
    // anything else a file opened relative to the working directory
    std::vector<uint8_t> input;
    const bool input_file = !(p_.input == "cin" || p_.input == "stdin");
    if (input_file) {
        if (p_.input.empty()) throw std::runtime_error("input '': gem5 polls fd -1 and retries read(0) forever");
        std::ifstream f(p_.input, std::ios::binary);
        if (!f) throw std::runtime_error("cannot open input " + p_.input);
        input.assign(std::istreambuf_iterator<char>(f), {});
    }
    // /proc/self/exe: realpath(Process.executable) (syscall_emul.hh:1089-1111);
    // unresolvable on this host -> unset (readlinkat escapes as host)
    std::string exe;
    {
        const std::string x = p_.executable.empty() ? p_.workload : p_.executable;
        if (char *rp = realpath(x.c_str(), nullptr)) { exe = rp; free(rp); }
    }
    if (p_.cpu_type != "atomic" && p_.cpu_type != "timing")
        throw std::runtime_error("cpu_type: 'atomic' or 'timing', not '" + p_.cpu_type + "'");
    const bool timing = p_.cpu_type == "timing";
    std::vector<int32_t> devs = p_.devices;
    if (devs.empty())
        for (uint32_t g = 0; g < p_.num_gpus; g++) devs.push_back((int32_t)(p_.first_device + g));
    for (size_t g = 0; g < devs.size(); g++) {
        fi_config cfg{};
        cfg.device = devs[g];
        cfg.private_pages = p_.private_pages;
        cfg.hang_factor_x16 = (uint32_t)(p_.max_insts_factor * 16 + 0.5);
        fi_engine *e = nullptr;
        fi_status s = fi_create(&cfg, &e);
        if (s != FI_OK) {
            std::string msg = fi_last_error(e);
            if (e) fi_destroy(e);
            throw std::runtime_error("fi_create(device " + std::to_string(cfg.device) + "): " + msg);
        }
        engines_.push_back(e);
        if (p_.checkpoint.empty())
            check(e, fi_load_elf(e, elf.data(), elf.size(), argv.data(), envp.data()), "fi_load_elf");
        else
            check(e, fi_load_checkpoint(e, p_.checkpoint.c_str(), elf.data(), elf.size()), "fi_load_checkpoint");
        if (!exe.empty()) check(e, fi_set_exe_path(e, exe.c_str()), "fi_set_exe_path");
        if (input_file) check(e, fi_set_stdin(e, input.data(), input.size()), "fi_set_stdin");
        check(e, fi_set_cpu_model(e, timing ? FI_CPU_TIMING : FI_CPU_ATOMIC, nullptr), "fi_set_cpu_model");
        fi_golden_info gi{};
        check(e, fi_golden_run(e, &gi), "fi_golden_run");
        if (timing) {
            fi_tick_info ti{};
            check(e, fi_tick_golden(e, &ti), "fi_tick_golden");
            if (ti.status[0]) throw std::runtime_error(std::string("cpu_type timing: ") + ti.status);
        }
        check(e, fi_set_campaign(e, p_.seed, smask, p_.burst), "fi_set_campaign");
        check(e, fi_set_bits(e, bits_mask(p_.bits)), "fi_set_bits");
        check(e, fi_set_protect(e, p_.protect_mask), "fi_set_protect");
        check(e, fi_set_protect_opclasses(e, opclass_mask(p_.protect_opclasses)), "fi_set_protect_opclasses");
        if (p_.shadow_fu_model) {
            fi_issue_params ip;
            fi_issue_default_params(&ip);
            ip.priority_to_shadow = p_.priority_to_shadow ? 1 : 0;
            ip.issue_width = p_.issue_width;
            ip.load_latency = p_.load_latency;
            check(e, fi_set_issue_model(e, &ip), "fi_set_issue_model");
        }
        if (g == 0) {
            golden_.ninst = gi.ninst;
            golden_.ncycles = gi.ncycles;
            golden_.exit_code = gi.exit_code;
            std::string buf(gi.stdout_len, '\0');
            uint64_t len = 0;
            check(e, fi_golden_stdout(e, reinterpret_cast<uint8_t *>(&buf[0]), buf.size(), &len),
                  "fi_golden_stdout");
            golden_.stdout_bytes = buf;
        } else if (gi.ninst != golden_.ninst || gi.exit_code != golden_.exit_code) {
            throw std::runtime_error("golden runs differ between devices");
        }
    }
}

Campaign::~Campaign() {
    for (auto *e : engines_) fi_destroy(e);
}

void Campaign::setProtectOpClasses(const std::vector<std::string> &opclasses) {
    p_.protect_opclasses = opclasses;
    const uint64_t m = opclass_mask(opclasses);
    for (auto *e : engines_) check(e, fi_set_protect_opclasses(e, m), "fi_set_protect_opclasses");
}

void Campaign::setProtectMask(uint64_t mask) {
    p_.protect_mask = mask;
    for (auto *e : engines_) check(e, fi_set_protect(e, mask), "fi_set_protect");
}

void Campaign::run() {
    const uint32_t G = (uint32_t)engines_.size();
    const uint64_t T = p_.trials;
    out_.assign(T, fi_outcome{});
    std::vector<fi_histogram> h(G);
    std::vector<std::string> err(G);
    memset(&hist_, 0, sizeof(hist_));
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (uint32_t g = 0; g < G; g++) {
        th.emplace_back([&, g] {
            const uint64_t lo = T * g / G, hi = T * (g + 1) / G;
            memset(&h[g], 0, sizeof(fi_histogram));
            fi_status s = p_.cpu_type == "timing"
                              ? fi_run_tick_trials(engines_[g], p_.first_trial + lo, hi - lo, out_.data() + lo, &h[g])
                              : fi_run_trials(engines_[g], p_.first_trial + lo, hi - lo, out_.data() + lo, &h[g]);
            if (s != FI_OK) err[g] = fi_last_error(engines_[g]);
        });
    }
    for (auto &t : th) t.join();
    seconds_ = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (uint32_t g = 0; g < G; g++) {
        if (!err[g].empty()) throw std::runtime_error("fi_run_trials(gpu " + std::to_string(g) + "): " + err[g]);
        hist_add(hist_, h[g]);
    }
    if (!p_.output.empty()) writeOutput();
}

std::string Campaign::summaryJson() const {
    std::ostringstream o;
    uint64_t cls[FI_N_CLASS] = {};
    for (int s = 0; s < FI_N_STRUCT; s++)
        for (int b = 0; b < 64; b++)
            for (int c = 0; c < FI_N_CLASS; c++) cls[c] += hist_.counts[s][b][c];
    o << "{\"workload\": \"" << p_.workload << "\", \"trials\": " << hist_.trials << ", \"first_trial\": "
      << p_.first_trial << ", \"seed\": " << p_.seed << ", \"burst\": " << p_.burst
      << ", \"protect_mask\": " << p_.protect_mask << ", \"num_gpus\": " << engines_.size()
      << ", \"golden_ninst\": " << golden_.ninst << ", \"golden_exit\": " << golden_.exit_code;
    for (int c = 0; c < FI_N_CLASS; c++) o << ", \"" << kClass[c] << "\": " << cls[c];
    o << ", \"crash_sub\": {";
    bool first = true;
    for (int i = 1; i < kNCrash; i++)
        if (hist_.crash_sub[i]) { o << (first ? "" : ", ") << "\"" << kCrash[i] << "\": " << hist_.crash_sub[i]; first = false; }
    o << "}, \"escape_sub\": {";
    first = true;
    for (int i = 1; i < kNEscape; i++)
        if (hist_.escape_sub[i]) { o << (first ? "" : ", ") << "\"" << kEscape[i] << "\": " << hist_.escape_sub[i]; first = false; }
    o << "}, \"guest_insts\": " << hist_.guest_insts << ", \"seconds\": " << seconds_
      << ", \"trials_per_s\": " << (seconds_ > 0 ? (double)hist_.trials / seconds_ : 0.0) << "}";
    return o.str();
}

void Campaign::writeOutput() const {
    {
        std::ofstream f(p_.output + ".outcomes.bin", std::ios::binary);
        if (!f) throw std::runtime_error("cannot write " + p_.output + ".outcomes.bin");
        f.write(reinterpret_cast<const char *>(out_.data()), (std::streamsize)(out_.size() * sizeof(fi_outcome)));
    }
    {
        std::ofstream f(p_.output + ".hist.bin", std::ios::binary);
        f.write(reinterpret_cast<const char *>(&hist_), sizeof(hist_));
    }
    std::ofstream f(p_.output + ".json");
    f << summaryJson() << "\n";
}

}  // namespace shrewd
