// fi_engine.cpp -- host side of the MI355X fault-injection engine (C ABI in
// include/fi_engine.h).
//
// Host responsibilities are the ones gem5 performs once per run before the
// tick loop starts: load the static ELF and build the SE process image
// (src/base/loader/elf_object.cc:374-404, src/sim/process.cc:289-306,
// src/arch/riscv/process.cc:71-261), then hand everything to the device.
// Every guest instruction -- golden run included -- executes in the HIP
// kernels (hip/fi_kernels.hip).  There is no CPU interpreter here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <vector>

#include "fi_checkpoint.h"
#include "fi_debug.h"
#include "fi_tick.h"
#include "fi_types.h"
#include "rv64_isa.h"

constexpr uint64_t kRndLen = 1ULL << 20;   // getrandom bytes precomputed per engine

namespace fi {
hipError_t launch_sample(const SampleCtx &c, uint64_t n, fi_site *sites, uint64_t *keys, uint32_t *perm,
                         hipStream_t st);
hipError_t launch_keys(const fi_site *sites, uint64_t n, uint64_t *keys, uint32_t *perm, hipStream_t st);
hipError_t launch_forward(const fi_site *sites, uint64_t n, const FwdCtx &c, uint64_t *keys, uint64_t *eff,
                          hipStream_t st);
hipError_t launch_predecode(const uint8_t *text, uint64_t code_off, uint64_t code_end, uint64_t nhalf, PreInst *pre,
                           hipStream_t st);
hipError_t launch_debug_decode(const uint32_t *raws, uint64_t n, PreInst *out, hipStream_t st);
hipError_t launch_trials(const DevCtx &c, hipStream_t st);
hipError_t launch_trials_solo(const DevCtx &c, hipStream_t st);
hipError_t launch_span_init(unsigned long long *span, uint64_t n, hipStream_t st);
hipError_t launch_debug_loop(const DevCtx &c, const fi_debug_loop *in, uint64_t n, fi_debug_loop_out *out,
                             hipStream_t st);
hipError_t launch_hist(const fi_site *sites, const fi_outcome *out, uint64_t n, fi_histogram *h,
                       const unsigned long long *stats, hipStream_t st);
hipError_t launch_hist_stats(const unsigned long long *stats, fi_histogram *h, hipStream_t st);
hipError_t sort_pairs_bytes(uint64_t n, size_t &bytes);
hipError_t launch_pack_runs(const uint64_t *keys, const uint32_t *cnt, uint64_t cap, uint32_t *wrange,
                            uint32_t *n_waves, hipStream_t st);
hipError_t launch_redo_collect(const fi_outcome *out, uint64_t n, uint32_t *idx, uint32_t *cnt,
                               unsigned long long *stats, hipStream_t st);
hipError_t launch_redo_gather(const fi_site *sites, const uint32_t *idx, uint64_t n, fi_site *rsites, uint64_t *keys,
                              uint32_t *perm, hipStream_t st);
hipError_t launch_redo_scatter(const uint32_t *idx, uint64_t n, const fi_outcome *rout, fi_outcome *out,
                               hipStream_t st);
hipError_t launch_surv_keys(const LaneSave *save, const uint32_t *list, const uint32_t *cnt, uint64_t cap,
                            uint64_t text_lo, uint64_t *keys, uint32_t *vals, uint32_t *n_odd, uint32_t solo,
                            uint64_t golden_ninst, uint32_t nb, const LoopEst *loops, uint32_t n_loops,
                            uint64_t hang_cap, hipStream_t st);
hipError_t launch_odd_split(const uint32_t *cnt, const uint32_t *n_odd, uint32_t *split, uint32_t grid,
                            hipStream_t st);
std::string translate_blocks(const std::vector<PreInst> &pre, uint64_t text_lo, const std::vector<uint32_t> &trace,
                             const std::vector<uint64_t> &extra_pcs, std::vector<uint32_t> &leaders_out,
                             uint32_t &n_insts, bool odd_streams, std::vector<LoopEst> *loops_out = nullptr);
std::vector<fi_issue_op> issue_ops_from_trace(const std::vector<PreInst> &pre, const std::vector<uint32_t> &trace);
std::string jit_compile(const std::string &body, const char *arch, std::vector<char> &code, bool &cached, int part,
                        bool use_cache);
bool jit_has_odd(const std::string &body);
bool jit_parallel_ok();
hipError_t sort_pairs(void *tmp, size_t bytes, const uint64_t *kin, uint64_t *kout, const uint32_t *vin,
                      uint32_t *vout, uint64_t n, int end_bit, hipStream_t st);
}  // namespace fi

using namespace fi;

// trials per wave when fi_config.lanes_per_wave is 0: 32 of
// a wave's 64 lanes -- twice the waves in the first epoch (3,125 for 100k
// trials: ~3 per SIMD instead of 1.5) and half the divergence per wave;
// profiles/r06w_sweep_lanes_*.jsonl: crc32 4.37 -> 4.13 ms, intmix 243 ->
// 225 ms, qsort even against 64; 16 loses on crc32
static constexpr uint32_t kDefaultLanes = 32;
static constexpr uint32_t kPreTail = 4;   // zero PreInst entries past the text (fi_trial.hip solo_pre_run)
static constexpr uint32_t kDefaultResumeLanes = 8;   // measured: profiles/README.md (r01b sweep)
// trials per launch while the translated kernels are still being built, so
// that a long campaign picks the build up at a chunk boundary.  Not smaller:
// a chunk lasts at least as long as its longest trial (the hang trials), so
// the static kernels' throughput grows with the chunk (crc32, 100k trials:
// 0.36 s in 16k chunks; profiles/r04e_bench.json)
static constexpr uint64_t kJitWindowChunk = 131072;

// The background build of the translated kernels (fi_golden_run starts it;
// run_chunks installs the result at a chunk boundary): the 64-lane, solo and,
// with odd-pc streams, solo-odd kernels as one code object each, compiled in
// parallel processes (fi_jit.cpp).  Until it lands the static kernels run
// every trial -- the same outcomes, bit for bit, more slowly.
struct JitJob {
    std::string body, arch;
    bool odd = false;
    bool use_cache = true;   // FI_CFG_JIT_NO_CACHE: always compile (cold-start measurements, tests)
    std::vector<char> code[3];
    std::string err;
    bool cached = true;
    uint64_t us = 0;
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
};
static const char *const kTxKernel[3] = {"fi_trial_kernel_tx", "fi_trial_kernel_tx_solo",
                                         "fi_trial_kernel_tx_solo_odd"};

static void jit_job_run(std::shared_ptr<JitJob> j) {
    const auto t0 = std::chrono::steady_clock::now();
    const int np = j->odd ? 3 : 2;
    std::string err[3];
    bool cached[3] = {true, true, true};
    if (jit_parallel_ok()) {
        std::vector<std::thread> th;
        for (int k = 0; k < np; k++)
            th.emplace_back([&, k] { err[k] = jit_compile(j->body, j->arch.c_str(), j->code[k], cached[k], k + 1, j->use_cache); });
        for (auto &t : th) t.join();
    } else {   // in-process hipRTC: one build at a time
        for (int k = 0; k < np; k++) err[k] = jit_compile(j->body, j->arch.c_str(), j->code[k], cached[k], k + 1, j->use_cache);
    }
    std::lock_guard<std::mutex> lk(j->mu);
    for (int k = 0; k < np && j->err.empty(); k++) j->err = err[k];
    j->cached = cached[0] && cached[1] && cached[2];
    j->us = (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
    j->done = true;
    j->cv.notify_all();
}

struct fi_engine {
    fi_config cfg{};
    std::string err;
    int dev = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double last_ms = 0;
    // per-launch timing of the interpreter kernel (bench roofline)
    std::vector<std::pair<hipEvent_t, hipEvent_t>> tpool;
    unsigned long long *d_span = nullptr;   // per timer slot: [min wave start, max wave end] (kSpanSlots pairs)
    std::vector<uint32_t> tkind;
    size_t tused = 0;

    // process image (host copy)
    bool loaded = false;
    std::map<uint64_t, std::vector<uint8_t>> pages;   // vpn -> 4 KiB
    uint64_t entry = 0, sp0 = 0, stack_min0 = 0, svma_lo = 0, svma_hi = 0;
    uint64_t text_lo = 0, text_hi = 0, code_lo = 0, code_hi = 0;
    std::vector<uint64_t> mem_pages;   // memory fault candidates (sorted)
    struct Seg { uint64_t lo, hi; bool w; };
    std::vector<Seg> segs;             // PT_LOAD page ranges of the ELF (w = PF_W)
    // checkpoint start state beyond registers, pages and the stack VMA
    bool fp0_on = false, vm0_on = false;
    uint64_t fp0[32] = {};
    uint32_t fcsr0 = 0;
    uint64_t tick0 = 0;
    VmState vm0{};
    uint64_t *d_fp0 = nullptr;
    VmState *d_vm0 = nullptr;

    // device image: snapshot 0 = the process-start image; the golden run
    // appends snapshots 1..n-1
    PreInst *d_pre = nullptr;
    uint8_t *d_zero = nullptr, *d_text = nullptr, *d_sink = nullptr;
    uint64_t *d_mem_pages = nullptr;
    std::vector<SnapState> snaps;
    std::vector<PageEnt> tab;
    std::vector<uint8_t> pool;            // host copy of the snapshot frames
    uint32_t n_start_frames = 0;          // frames [0, n) = process-start pages
    SnapState *d_snaps = nullptr;
    PageEnt *d_tab = nullptr;
    uint8_t *d_pool = nullptr;
    uint64_t snap_I = 1ULL << 62;
    // memory liveness index of the golden run (build_mem_index)
    bool mem_live = false;
    uint32_t mw_n = 0;
    uint64_t *d_mw_addr = nullptr, *d_mw_ev = nullptr;
    // first-access forwarding: per register x1..x31, the golden trace's
    // accesses in order, entry = (2 * numInst + !ecall) << 1 | reads
    uint32_t *d_fw_off = nullptr, *d_fw_ev = nullptr;
    bool fw_ok = false;
    uint64_t *d_eff = nullptr;       // [cap] effective inject time per trial (kFwDead: dead at injection)
    uint32_t *d_mw_off = nullptr;
    bool pre_ok = true;
    // load-time build of the trial kernel with the translated golden blocks
    hipModule_t tx_mod[3] = {nullptr, nullptr, nullptr};
    std::shared_ptr<JitJob> jit;     // the build in flight (nullptr: none)
    // builds this engine started: a finished one is joined when a build is
    // installed (jit_install), one still running by fi_destroy
    std::vector<std::pair<std::thread, std::shared_ptr<JitJob>>> jit_threads;
    std::vector<PreInst> jit_pre;    // golden pre-decoded text with the leader flags, uploaded when it lands
    uint64_t jit_blocks = 0, jit_insts = 0;
    hipFunction_t tx_fn = nullptr, tx_fn_solo = nullptr;
    hipFunction_t tx_fn_odd = nullptr;   // solo kernel with the odd-pc blocks (nullptr: none translated)
    // the solo-odd kernel runs beside the solo kernel on its own stream
    hipStream_t stream_odd = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    std::string tx_status = "no golden run";
    std::string tx_body;   // last generated translation (diagnostics)

    // golden
    bool have_golden = false;
    fi_golden_info golden{};
    uint32_t gdetail = 0, gsub = 0;
    std::vector<uint8_t> gout, gerr;
    uint8_t *d_gout = nullptr, *d_gerr = nullptr;

    // campaign
    uint64_t seed = 0x5EED0001ULL, structures = 0;
    uint32_t burst = 1;
    uint64_t bits = ~0ULL;      // eligible lowest-bit positions (fi_set_bits)
    uint64_t clk_period = 500, rnd_seed = 5489;   // fi_set_clock
    uint8_t *d_rnd = nullptr;   // getrandom's byte stream (kRndLen bytes)
    std::string exe_path;       // fi_set_exe_path
    uint8_t *d_exe = nullptr;
    bool stdin_on = false;      // fi_set_stdin: Process.input is a file (else "cin")
    std::vector<uint8_t> stdin_data;
    uint8_t *d_stdin = nullptr;
    uint64_t *d_inpos = nullptr;   // per work slot: fd 0's file offset
    uint64_t protect = 0;
    uint64_t protect_opc = 0;   // SHREWD replication by OpClass (fi_set_protect_opclasses)
    // SHREWD FU contention (fi_set_issue_model): shadow issued per golden numInst index
    bool issue_on = false;
    fi_issue_params issue_p{};
    fi_issue_stats issue_stats{};
    std::vector<uint8_t> shadow;
    uint32_t *d_shadow = nullptr;    // the same as a bitmap, [ninst / 32 + 1]
    std::vector<PreInst> g_pre;      // golden pre-decoded text and trace (empty: unavailable)
    std::vector<uint32_t> g_trace;
    // tick-domain injection (fi_set_cpu_model FI_CPU_TIMING; fi_tick.cpp, fi_timing.cpp)
    int cpu_model = FI_CPU_ATOMIC;
    fi_timing_params tparams{};
    std::vector<uint64_t> alloc_order;   // process-start pages in allocation order (fi_load_elf's writes)
    bool golden_unmapped = false;        // the golden run freed frames (munmap / brk shrink)
    std::vector<fi_timing_op> t_ops;     // the golden run's attempts as requests
    std::vector<TickAttempt> t_att;
    std::vector<fi_timing_ticks> t_ticks;
    fi_timing_stats t_stats{};
    std::string t_status = "no golden run";
    uint32_t clk_esc = 0;                // DevCtx::clk_esc while tick trials run

    // work buffers, sized for `cap` trials per launch
    uint64_t cap = 0;
    fi_site *d_sites = nullptr, *d_sites_alt = nullptr;   // the chunk being run / the one being finished
    uint64_t *d_keys = nullptr, *d_keys2 = nullptr;
    uint32_t *d_perm = nullptr, *d_perm2 = nullptr;
    void *d_tmp = nullptr;
    size_t tmp_bytes = 0;
    fi_outcome *d_out = nullptr, *d_out_alt = nullptr;
    fi_histogram *d_hist = nullptr;
    unsigned long long *d_stats = nullptr;
    uint64_t *d_wave_dbg = nullptr;
    uint64_t *d_fregs = nullptr;     // FP registers of the work slots
    bool golden_fp = false;          // the golden run wrote FP state: no snapshot start / early exit
    uint64_t clk_until = 0;          // 1 + numInst of the golden run's last curTick read (0: none; DevCtx::clk_until)
    uint8_t *d_priv = nullptr;
    uint64_t *d_priv_vpn = nullptr;
    // overflow pages (DevCtx::ov_*): ov_blocks blocks of ov_pages
    uint8_t *d_ov = nullptr;
    uint64_t *d_ov_vpn = nullptr;
    uint32_t *d_ov_of = nullptr, *d_ov_next = nullptr;
    uint32_t ov_blocks = 0, ov_pages = 0;
    VmState *d_vm = nullptr;         // [cap] per-slot SE memory map (trials that made a VM syscall)
    uint64_t brk0 = 0;               // roundUp(maxAddr, page): the process-start brk point
    // epochs: suspended lanes, survivor lists, counts, sort buffers
    LaneSave *d_save = nullptr;
    uint32_t *d_surv[2] = {nullptr, nullptr};
    uint32_t *d_cnt = nullptr;
    uint64_t *d_skeys = nullptr, *d_skeys2 = nullptr;
    uint32_t *d_svals = nullptr, *d_svals2 = nullptr;
    uint32_t *d_wrange = nullptr, *d_nwaves = nullptr;   // packed resume (FI_CFG_PACK_RUNS)
    uint32_t *d_split = nullptr;   // per epoch: odd-pc survivors, then the solo kernel's share of the list
    LoopEst *d_loops = nullptr;    // counted loops of the golden text (the solo order's work-left estimate)
    uint32_t n_loops = 0;
    uint32_t *d_dmap = nullptr;    // per slot: rewritten-code map (DevCtx::dmap, kDmapWords words)
    // second pass of the trials that ran out of private pages (chunk_end)
    uint32_t *d_redo_idx = nullptr, *d_redo_cnt = nullptr, *h_redo_cnt = nullptr;   // two of each: a chunk and its predecessor
    hipEvent_t ev_cnt[2] = {nullptr, nullptr};   // a chunk's redo count has reached h_redo_cnt
    // pinned staging of a chunk's outcomes on their way to the caller's (pageable) array: a copy
    // straight into pageable memory would hold the host until the stream reaches it
    fi_outcome *h_stage[2] = {nullptr, nullptr};
    hipEvent_t ev_stage[2] = {nullptr, nullptr};
    fi_site *d_redo_sites = nullptr;
    fi_outcome *d_redo_out = nullptr;
};

static fi_status fail(fi_engine *e, fi_status code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (e) e->err = buf;
    return code;
}

#define HIPCHK(call)                                                                          \
    do {                                                                                      \
        hipError_t _e = (call);                                                               \
        if (_e != hipSuccess) return fail(e, FI_E_HIP, "%s: %s", #call, hipGetErrorString(_e)); \
    } while (0)

template <typename T>
static void dfree(T *&p) {
    if (p) { (void)hipFree((void *)p); p = nullptr; }
}

// Diagnostics (SHREWD_FI_TRACE): a native backtrace on SIGSEGV.
#include <execinfo.h>
#include <csignal>
#include <unistd.h>
static void segv_trace(int sig) {
    void *bt[64];
    const int n = backtrace(bt, 64);
    const char msg[] = "[fi] fatal signal, native backtrace:\n";
    (void)!write(2, msg, sizeof msg - 1);
    backtrace_symbols_fd(bt, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

extern "C" {

// errors of calls that have no engine yet (fi_create), per host thread
static thread_local std::string g_create_err;

// getrandom's bytes: gem5's Random(globalSeed) generator (std::mt19937_64,
// base/random.hh:125) drawn once per byte, % 255 (Random::random<uint8_t>)
static fi_status upload_rnd(fi_engine *e) {
    std::vector<uint8_t> tab(kRndLen);
    std::mt19937_64 gen((uint32_t)e->rnd_seed);
    for (auto &b : tab) b = (uint8_t)(gen() % 255);
    if (!e->d_rnd) HIPCHK(hipMalloc(&e->d_rnd, kRndLen));
    HIPCHK(hipMemcpy(e->d_rnd, tab.data(), kRndLen, hipMemcpyHostToDevice));
    return FI_OK;
}

// private pages per slot of the second pass (and so the overflow blocks): 16 P, at least 256
static uint64_t redo_pages(uint64_t P) { return std::max<uint64_t>(P * 16ull, 256); }

fi_status fi_create(const fi_config *cfg, fi_engine **out) {
    if (!out) { g_create_err = "fi_create: out is NULL"; return FI_E_ARG; }
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        g_create_err = "fi_create: no HIP device visible (the engine has no CPU fallback)";
        return FI_E_NODEVICE;
    }
    if (getenv("SHREWD_FI_TRACE")) signal(SIGSEGV, segv_trace);
    fi_engine *e = new fi_engine();
    if (cfg) e->cfg = *cfg;
    // diagnostics (A/B runs of an unchanged caller): FI_CFG_* bits to add
    if (const char *x = getenv("SHREWD_FI_EXTRA_FLAGS")) e->cfg.flags |= (uint32_t)strtoul(x, nullptr, 0);
    if (e->cfg.private_pages == 0) e->cfg.private_pages = 16;
    if (e->cfg.hang_factor_x16 == 0) e->cfg.hang_factor_x16 = 32;
    if (e->cfg.lanes_per_wave == 0) e->cfg.lanes_per_wave = kDefaultLanes;
    if (e->cfg.resume_lanes == 0) e->cfg.resume_lanes = kDefaultResumeLanes;
    for (uint32_t l : {e->cfg.lanes_per_wave, e->cfg.resume_lanes}) {
        if (l > 64 || (l & (l - 1))) {
            g_create_err = "fi_create: lanes_per_wave / resume_lanes must be a power of two <= 64";
            delete e;
            return FI_E_ARG;
        }
    }
    e->dev = e->cfg.device;
    if (e->dev < 0 || e->dev >= n) {
        g_create_err = "fi_create: device " + std::to_string(e->dev) + " out of range (" + std::to_string(n) + " visible)";
        delete e;
        return FI_E_ARG;
    }
    if (hipSetDevice(e->dev) != hipSuccess || hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&e->stream_odd, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&e->ev0) != hipSuccess || hipEventCreate(&e->ev1) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_join, hipEventDisableTiming) != hipSuccess) {
        g_create_err = "fi_create: HIP stream/event creation failed on device " + std::to_string(e->dev);
        delete e;
        return FI_E_HIP;
    }
    if (upload_rnd(e) != FI_OK) {
        g_create_err = "fi_create: " + e->err;
        delete e;
        return FI_E_HIP;
    }
    if (e->cfg.max_trials_per_launch == 0) {
        // auto: a campaign's trials in as few launches as half the free HBM
        // holds (each launch ends in its own serial tail of long trials), at
        // (4 KiB + 8 B) per private page, the per-slot buffers of ensure_work
        // (both site / outcome buffers of the chunks in flight, the redo
        // lists, the rewritten-code map) and the overflow pool's share
        // (one block of P' - P pages per 2048 slots)
        size_t free_b = 0, total_b = 0;
        const uint64_t P = e->cfg.private_pages, P2 = redo_pages(P);
        const uint64_t slot_b = 3 * sizeof(fi_site) + 3 * sizeof(fi_outcome) + 8 * 8 + 8 * 4 + 10 * 8 +
                                sizeof(LaneSave) + sizeof(VmState) + 33 * 8 + kDmapWords * 4 + 4 + 64;
        const uint64_t per = P * (kPage + 8) + slot_b + (P2 > P ? (P2 - P) * (kPage + 8) / 2048 + 1 : 0);
        uint64_t cap = 65536;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) cap = (uint64_t)free_b / 2 / per;
        e->cfg.max_trials_per_launch = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(cap, 65536), 1u << 21);
    }
    *out = e;
    return FI_OK;
}

static void free_work(fi_engine *e) {
    dfree(e->d_sites); dfree(e->d_sites_alt); dfree(e->d_out_alt); dfree(e->d_keys); dfree(e->d_keys2); dfree(e->d_perm); dfree(e->d_perm2);
    dfree(e->d_tmp); dfree(e->d_out); dfree(e->d_hist); dfree(e->d_stats); dfree(e->d_wave_dbg); dfree(e->d_fregs);
    dfree(e->d_inpos);
    dfree(e->d_save); dfree(e->d_surv[0]); dfree(e->d_surv[1]); dfree(e->d_cnt);
    dfree(e->d_eff);
    dfree(e->d_skeys); dfree(e->d_skeys2); dfree(e->d_svals); dfree(e->d_svals2); dfree(e->d_wrange); dfree(e->d_nwaves); dfree(e->d_split); dfree(e->d_dmap); dfree(e->d_priv); dfree(e->d_priv_vpn); dfree(e->d_vm);
    dfree(e->d_ov); dfree(e->d_ov_vpn); dfree(e->d_ov_of); dfree(e->d_ov_next);
    e->ov_blocks = e->ov_pages = 0;
    dfree(e->d_redo_idx); dfree(e->d_redo_cnt); dfree(e->d_redo_sites); dfree(e->d_redo_out);
    for (auto &h : e->h_stage)
        if (h) { (void)hipHostFree(h); h = nullptr; }
    e->cap = 0;
}
static void free_snaps(fi_engine *e) { dfree(e->d_snaps); dfree(e->d_tab); dfree(e->d_pool); }
static void free_mem_index(fi_engine *e) {
    dfree(e->d_mw_addr); dfree(e->d_mw_off); dfree(e->d_mw_ev);
    e->mw_n = 0;
    e->mem_live = false;
}
static void free_fw(fi_engine *e) {
    dfree(e->d_fw_off); dfree(e->d_fw_ev); dfree(e->d_loops);
    e->fw_ok = false;
    e->n_loops = 0;
}
static void free_tx(fi_engine *e) {
    for (auto &m : e->tx_mod) {
        if (m) (void)hipModuleUnload(m);
        m = nullptr;
    }
    e->tx_fn = e->tx_fn_solo = e->tx_fn_odd = nullptr;
    e->jit.reset();   // a build in flight finishes on its own (its thread holds the job; fi_destroy joins it)
}

// Install a finished background build (at a chunk boundary, before anything
// of the chunk is queued on st): load the code objects and flag the block
// leaders in the pre-decoded text.  wait = block until the build is done.
static void jit_install(fi_engine *e, hipStream_t st, bool wait) {
    std::shared_ptr<JitJob> j = e->jit;
    if (!j) return;
    {
        std::unique_lock<std::mutex> lk(j->mu);
        if (wait) j->cv.wait(lk, [&] { return j->done; });
        if (!j->done) return;
    }
    e->jit.reset();
    // join the builds that have finished (this one, and any an earlier golden
    // run left behind): a long-lived engine keeps no finished threads
    for (size_t i = 0; i < e->jit_threads.size();) {
        bool fin;
        {
            std::lock_guard<std::mutex> lk(e->jit_threads[i].second->mu);
            fin = e->jit_threads[i].second->done;
        }
        if (fin) {
            if (e->jit_threads[i].first.joinable()) e->jit_threads[i].first.join();
            e->jit_threads.erase(e->jit_threads.begin() + (long)i);
        } else {
            i++;
        }
    }
    if (!j->err.empty()) {
        e->tx_status = j->err;
        return;
    }
    hipFunction_t *fn[3] = {&e->tx_fn, &e->tx_fn_solo, &e->tx_fn_odd};
    for (int k = 0; k < (j->odd ? 3 : 2); k++) {
        if (hipModuleLoadData(&e->tx_mod[k], j->code[k].data()) != hipSuccess ||
            hipModuleGetFunction(fn[k], e->tx_mod[k], kTxKernel[k]) != hipSuccess) {
            free_tx(e);
            e->tx_status = "code object did not load";
            return;
        }
    }
    if (hipMemcpyAsync(e->d_pre, e->jit_pre.data(), e->jit_pre.size() * sizeof(PreInst), hipMemcpyHostToDevice, st) !=
        hipSuccess) {
        free_tx(e);
        e->tx_status = "pre-decoded text upload failed";
        return;
    }
    e->tx_status = "";
    e->golden.translated_blocks = e->jit_blocks;
    e->golden.translated_insts = e->jit_insts;
    e->golden.translate_us = j->cached ? 0 : j->us;
}
static void free_image(fi_engine *e) {
    dfree(e->d_pre); dfree(e->d_zero); dfree(e->d_sink);
    dfree(e->d_text); dfree(e->d_mem_pages); dfree(e->d_gout); dfree(e->d_gerr);
    dfree(e->d_fp0); dfree(e->d_vm0);
    e->fp0_on = e->vm0_on = false;
    e->tick0 = 0;
    free_snaps(e);
    free_mem_index(e);
    free_fw(e);
    free_tx(e);
    dfree(e->d_shadow);
    e->g_pre.clear(); e->g_trace.clear(); e->shadow.clear();
    e->have_golden = false;
    e->loaded = false;
}

void fi_destroy(fi_engine *e) {
    if (!e) return;
    // a background build still running (a short campaign on a cold cache):
    // wait for it, so that no thread outlives the engine and no fi_jitc child
    // is left behind -- exiting under a running build races the static
    // destructors of the JIT cache and of hipRTC
    for (auto &t : e->jit_threads)
        if (t.first.joinable()) t.first.join();
    (void)hipSetDevice(e->dev);
    free_work(e);
    free_image(e);
    dfree(e->d_rnd); dfree(e->d_exe); dfree(e->d_stdin);
    for (auto &tp : e->tpool) { (void)hipEventDestroy(tp.first); (void)hipEventDestroy(tp.second); }
    dfree(e->d_span);
    if (e->ev0) (void)hipEventDestroy(e->ev0);
    if (e->ev1) (void)hipEventDestroy(e->ev1);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    if (e->stream_odd) (void)hipStreamDestroy(e->stream_odd);
    if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
    if (e->ev_join) (void)hipEventDestroy(e->ev_join);
    if (e->h_redo_cnt) (void)hipHostFree(e->h_redo_cnt);
    for (auto ev : e->ev_cnt)
        if (ev) (void)hipEventDestroy(ev);
    for (auto ev : e->ev_stage)
        if (ev) (void)hipEventDestroy(ev);
    delete e;
}

const char *fi_last_error(fi_engine *e) { return e ? e->err.c_str() : g_create_err.c_str(); }

// ------------------------------------------------------------------ image
static uint16_t le16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static uint32_t le32(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
static uint64_t le64(const uint8_t *p) { return (uint64_t)le32(p) | ((uint64_t)le32(p + 4) << 32); }

// SETranslatingPortProxy(Always) write: allocates pages on demand.
static void img_write(fi_engine *e, uint64_t addr, const uint8_t *src, uint64_t n) {
    for (uint64_t i = 0; i < n;) {
        const uint64_t a = addr + i;
        auto &pg = e->pages[a >> 12];
        if (pg.empty()) {
            pg.assign(kPage, 0);
            // SETranslatingPortProxy (Always) allocates the frame on this first
            // write: frames go out in this order (sim/process.cc:318-343)
            e->alloc_order.push_back(a >> 12);
        }
        const uint64_t off = a & (kPage - 1);
        const uint64_t k = std::min<uint64_t>(n - i, kPage - off);
        if (src) memcpy(pg.data() + off, src + i, k);
        else memset(pg.data() + off, 0, k);
        i += k;
    }
}
static void img_push64(fi_engine *e, uint64_t &sp, uint64_t v) {
    uint8_t b[8];
    for (int i = 0; i < 8; i++) b[i] = (uint8_t)(v >> (8 * i));
    img_write(e, sp, b, 8);
    sp += 8;
}

// std::mt19937_64 with gem5's global seed 5489 (src/base/random.hh:211-217):
// AT_RANDOM byte i = gen() % 256 (RiscvProcess::argsInit, process.cc:171-175).
struct Mt64 {
    uint64_t mt[312];
    int idx;
    explicit Mt64(uint64_t seed) {
        mt[0] = seed;
        for (int i = 1; i < 312; i++) mt[i] = 6364136223846793005ULL * (mt[i - 1] ^ (mt[i - 1] >> 62)) + (uint64_t)i;
        idx = 312;
    }
    uint64_t operator()() {
        if (idx >= 312) {
            for (int i = 0; i < 312; i++) {
                const uint64_t x = (mt[i] & 0xFFFFFFFF80000000ULL) | (mt[(i + 1) % 312] & 0x7FFFFFFFULL);
                uint64_t xa = x >> 1;
                if (x & 1) xa ^= 0xB5026F5AA96619E9ULL;
                mt[i] = mt[(i + 156) % 312] ^ xa;
            }
            idx = 0;
        }
        uint64_t y = mt[idx++];
        y ^= (y >> 29) & 0x5555555555555555ULL;
        y ^= (y << 17) & 0x71D67FFFEDA60000ULL;
        y ^= (y << 37) & 0xFFF7EEE000000000ULL;
        y ^= y >> 43;
        return y;
    }
};

// The issue model over the golden trace (fi_issue.cpp), indexed by numInst
// (ecall events are replayed but numInst does not count them), uploaded as a
// bitmap for the result-fault commit (fi_trial.hip:replicated).
static fi_status compute_shadow(fi_engine *e) {
    if (e->g_trace.empty() && e->golden.ninst)
        return fail(e, FI_E_STATE, "issue model: the golden trace is unavailable (trace overflow or rewritten text)");
    const std::vector<fi_issue_op> ops = issue_ops_from_trace(e->g_pre, e->g_trace);
    std::vector<uint8_t> all(ops.size());
    fi_issue_stats st{};
    const fi_status s = fi_issue_model_run(ops.data(), ops.size(), &e->issue_p, all.data(), &st);
    if (s) return fail(e, s, "issue model: invalid parameters");
    e->shadow.clear();
    e->shadow.reserve(e->golden.ninst);
    for (size_t i = 0; i < ops.size(); i++)
        if (!(e->g_trace[i] & 0x80000000u)) e->shadow.push_back(all[i]);
    if (e->shadow.size() != e->golden.ninst)
        return fail(e, FI_E_STATE, "issue model: trace holds %zu instructions, golden run %llu", e->shadow.size(),
                    (unsigned long long)e->golden.ninst);
    std::vector<uint32_t> bits(e->shadow.size() / 32 + 1, 0);
    for (size_t k = 0; k < e->shadow.size(); k++)
        if (e->shadow[k]) bits[k >> 5] |= 1u << (k & 31);
    dfree(e->d_shadow);
    HIPCHK(hipMalloc(&e->d_shadow, bits.size() * 4));
    HIPCHK(hipMemcpy(e->d_shadow, bits.data(), bits.size() * 4, hipMemcpyHostToDevice));
    e->issue_stats = st;
    return FI_OK;
}

static fi_status upload_snaps(fi_engine *e) {
    free_snaps(e);
    HIPCHK(hipMalloc(&e->d_snaps, e->snaps.size() * sizeof(SnapState)));
    HIPCHK(hipMalloc(&e->d_tab, std::max<size_t>(1, e->tab.size()) * sizeof(PageEnt)));
    // (+64: solo translated code reads shared frames with dword-granular scalar
    // loads that may run up to 11 bytes past an access at a frame's end)
    HIPCHK(hipMalloc(&e->d_pool, std::max<size_t>(kPage, e->pool.size()) + 64));
    HIPCHK(hipMemcpy(e->d_snaps, e->snaps.data(), e->snaps.size() * sizeof(SnapState), hipMemcpyHostToDevice));
    if (!e->tab.empty())
        HIPCHK(hipMemcpy(e->d_tab, e->tab.data(), e->tab.size() * sizeof(PageEnt), hipMemcpyHostToDevice));
    if (!e->pool.empty()) HIPCHK(hipMemcpy(e->d_pool, e->pool.data(), e->pool.size(), hipMemcpyHostToDevice));
    return FI_OK;
}

static fi_status finish_load(fi_engine *e, const uint64_t regs[32], uint64_t pc);

fi_status fi_load_elf(fi_engine *e, const uint8_t *elf, size_t len, const char *const *argv, const char *const *envp) {
    if (!e || !elf || !argv || !argv[0]) return fail(e, FI_E_ARG, "fi_load_elf: elf and argv[0] required");
    HIPCHK(hipSetDevice(e->dev));
    free_image(e);
    e->pages.clear();
    e->mem_pages.clear();
    e->segs.clear();
    e->alloc_order.clear();
    if (len < 64 || memcmp(elf, "\x7f" "ELF", 4) || elf[4] != 2 || elf[5] != 1 || le16(elf + 18) != 243)
        return fail(e, FI_E_ELF, "not an ELF64 little-endian RISC-V executable");
    e->entry = le64(elf + 24);
    const uint64_t phoff = le64(elf + 32);
    const uint32_t phentsize = le16(elf + 54), phnum = le16(elf + 56);
    if (phoff + (uint64_t)phentsize * phnum > len) return fail(e, FI_E_ELF, "program headers out of file");
    uint64_t max_addr = 0, phdr_vaddr = 0;
    uint64_t xlo = ~0ULL, xhi = 0, clo = ~0ULL, chi = 0;
    std::vector<uint64_t> wpages;
    for (uint32_t i = 0; i < phnum; i++) {
        const uint8_t *ph = elf + phoff + (uint64_t)i * phentsize;
        if (le32(ph) != 1) continue;   // PT_LOAD
        const uint32_t flags = le32(ph + 4);
        const uint64_t off = le64(ph + 8), vaddr = le64(ph + 16), paddr = le64(ph + 24);
        const uint64_t filesz = le64(ph + 32), memsz = le64(ph + 40);
        if (memsz == 0) continue;                       // elf_object.cc:378-381
        if (off + filesz > len) return fail(e, FI_E_ELF, "segment %u beyond file", i);
        img_write(e, paddr, elf + off, filesz);          // loaded at p_paddr (elf_object.cc:383)
        if (memsz > filesz) img_write(e, paddr + filesz, nullptr, memsz - filesz);
        max_addr = std::max(max_addr, paddr + memsz);
        e->segs.push_back({paddr & ~(kPage - 1), (paddr + memsz + kPage - 1) & ~(kPage - 1), (flags & 2) != 0});
        if (off <= phoff && off + filesz > phoff) phdr_vaddr = vaddr + (phoff - off);
        if (flags & 1) {
            xlo = std::min(xlo, paddr & ~(kPage - 1));
            xhi = std::max(xhi, (paddr + memsz + kPage - 1) & ~(kPage - 1));
            clo = std::min(clo, paddr);
            chi = std::max(chi, paddr + memsz);
        }
        if (flags & 2)
            for (uint64_t pg = paddr & ~(kPage - 1); pg < paddr + memsz; pg += kPage) wpages.push_back(pg);
    }
    if (xlo == ~0ULL) return fail(e, FI_E_ELF, "no executable segment");
    if ((xlo >> 32) != ((xhi - 1) >> 32)) return fail(e, FI_E_ELF, "executable segments cross a 4 GiB boundary");
    e->text_lo = xlo;
    e->text_hi = xhi;
    e->code_lo = clo;
    e->code_hi = chi;

    // RiscvProcess::argsInit<uint64_t> (src/arch/riscv/process.cc:134-261)
    std::vector<std::string> av, ev;
    for (int i = 0; argv[i]; i++) av.emplace_back(argv[i]);
    for (int i = 0; envp && envp[i]; i++) ev.emplace_back(envp[i]);
    const int nauxv = 8;
    uint64_t stack_min = kStackBase;
    uint64_t stack_top = stack_min - 16;
    for (auto &s : av) stack_top -= s.size() + 1;
    for (auto &s : ev) stack_top -= s.size() + 1;
    stack_top &= ~7ULL;
    const uint64_t at_random = stack_top;   // AT_RANDOM points here (process.cc:156)
    const uint64_t arrays = (1 + av.size()) * 8 + (1 + ev.size()) * 8 + 8 + 2 * 8 * nauxv;
    stack_top -= arrays;
    stack_top &= ~15ULL;
    const uint64_t stack_size = kStackBase - stack_top;
    e->svma_lo = stack_top & ~(kPage - 1);
    e->svma_hi = e->svma_lo + ((stack_size + kPage - 1) & ~(kPage - 1));
    stack_min -= 16;
    Mt64 rng(5489);
    uint8_t rnd[16];
    for (int i = 0; i < 16; i++) rnd[i] = (uint8_t)(rng() % 256);
    img_write(e, stack_min, rnd, 16);
    std::vector<uint64_t> argp, envptr;
    for (auto &s : av) { stack_min -= s.size() + 1; img_write(e, stack_min, (const uint8_t *)s.c_str(), s.size() + 1); argp.push_back(stack_min); }
    for (auto &s : ev) { stack_min -= s.size() + 1; img_write(e, stack_min, (const uint8_t *)s.c_str(), s.size() + 1); envptr.push_back(stack_min); }
    stack_min &= ~7ULL;
    stack_min -= arrays;
    stack_min &= ~15ULL;
    uint64_t sp = stack_min;
    img_push64(e, sp, av.size());
    for (uint64_t p : argp) img_push64(e, sp, p);
    img_push64(e, sp, 0);
    for (uint64_t p : envptr) img_push64(e, sp, p);
    img_push64(e, sp, 0);
    const uint64_t aux[8][2] = {{9, e->entry}, {5, phnum}, {4, phentsize}, {3, phdr_vaddr},
                                {6, kPage}, {23, 0}, {25, at_random}, {0, 0}};
    for (auto &a : aux) { img_push64(e, sp, a[0]); img_push64(e, sp, a[1]); }
    e->sp0 = stack_min;
    e->stack_min0 = stack_min & ~(kPage - 1);
    for (uint64_t pg = e->stack_min0;; pg += kPage) {
        wpages.push_back(pg);
        if (pg == (kStackBase & ~(kPage - 1))) break;
    }
    std::sort(wpages.begin(), wpages.end());
    wpages.erase(std::unique(wpages.begin(), wpages.end()), wpages.end());
    e->mem_pages = wpages;
    e->brk0 = (max_addr + kPage - 1) & ~(kPage - 1);   // Process brk point (process.cc: roundUp(maxAddr))
    // RiscvProcess::argsInit leaves every register 0 but sp; pc = e_entry
    uint64_t regs[32] = {};
    regs[2] = e->sp0;
    return finish_load(e, regs, e->entry);
}

// ---- snapshot 0: the start image in e->pages (frames sorted by vpn) and the
// initial architectural state; the text pre-decoded on the device.  The
// common tail of fi_load_elf and fi_load_checkpoint.
static fi_status finish_load(fi_engine *e, const uint64_t regs[32], uint64_t pc) {
    const std::vector<uint64_t> &wpages = e->mem_pages;
    e->pool.clear();
    e->tab.clear();
    e->snaps.clear();
    for (auto &kv : e->pages) {
        PageEnt pe{};
        pe.vpn = kv.first;
        pe.frame = (uint32_t)(e->pool.size() / kPage);
        e->tab.push_back(pe);
        e->pool.insert(e->pool.end(), kv.second.begin(), kv.second.end());
    }
    e->n_start_frames = (uint32_t)e->tab.size();
    SnapState s0{};
    for (int r = 1; r < 32; r++) s0.regs[r] = regs[r];
    s0.pc = pc;
    s0.stack_min = e->stack_min0;
    s0.tab_off = 0;
    s0.tab_n = (uint32_t)e->tab.size();
    e->snaps.push_back(s0);
    e->snap_I = 1ULL << 62;
    e->pre_ok = true;
    {
        fi_status st = upload_snaps(e);
        if (st) return st;
    }
    HIPCHK(hipMalloc(&e->d_zero, kPage + 64));   // (+64: as the frame pool)
    HIPCHK(hipMalloc(&e->d_sink, kPage));
    HIPCHK(hipMalloc(&e->d_mem_pages, std::max<size_t>(1, wpages.size()) * 8));
    HIPCHK(hipMemset(e->d_zero, 0, kPage + 64));
    if (!wpages.empty()) HIPCHK(hipMemcpy(e->d_mem_pages, wpages.data(), wpages.size() * 8, hipMemcpyHostToDevice));
    const uint64_t tbytes = e->text_hi - e->text_lo;
    std::vector<uint8_t> text(tbytes, 0);
    for (uint64_t a = e->text_lo; a < e->text_hi; a += kPage) {
        auto it = e->pages.find(a >> 12);
        if (it != e->pages.end()) memcpy(text.data() + (a - e->text_lo), it->second.data(), kPage);
    }
    HIPCHK(hipMalloc(&e->d_text, tbytes));
    HIPCHK(hipMemcpy(e->d_text, text.data(), tbytes, hipMemcpyHostToDevice));
    // + kPreTail zero entries (kind K_SLOW): the solo interpreter prefetches
    // the fall-through entry of the text's last instruction without a clamp
    HIPCHK(hipMalloc(&e->d_pre, (tbytes / 2 + kPreTail) * sizeof(PreInst)));
    HIPCHK(hipMemset(e->d_pre + tbytes / 2, 0, kPreTail * sizeof(PreInst)));
    HIPCHK(launch_predecode(e->d_text, e->code_lo - e->text_lo, e->code_hi - e->text_lo, tbytes / 2, e->d_pre,
                            e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    e->loaded = true;
    return FI_OK;
}

// ------------------------------------------------------------------ work buffers
fi_status fi_load_checkpoint(fi_engine *e, const char *cpt_dir, const uint8_t *elf, size_t len) {
    if (!e || !cpt_dir || !elf) return fail(e, FI_E_ARG, "fi_load_checkpoint: checkpoint directory and ELF required");
    const char *argv[] = {"checkpoint", nullptr};
    fi_status st = fi_load_elf(e, elf, len, argv, nullptr);   // executable range, entry checks
    if (st) return st;
    CptImage img;
    const std::string err = read_gem5_checkpoint(cpt_dir, img);
    if (!err.empty()) return fail(e, FI_E_ARG, "fi_load_checkpoint: %s", err.c_str());
    // the engine's SE model keeps RiscvProcess64's stack (process.cc:71-82)
    if (img.stack_base != kStackBase || img.max_stack != kMaxStack)
        return fail(e, FI_E_ARG, "fi_load_checkpoint: stack base / max stack differ from RiscvProcess64's");
    if (img.vmas.size() > kMaxVma)
        return fail(e, FI_E_ARG, "fi_load_checkpoint: %zu VMAs (at most %u)", img.vmas.size(), kMaxVma);
    const std::vector<fi_engine::Seg> segs = e->segs;   // (fi_load_elf's; free_image keeps them)
    free_image(e);
    e->pages.clear();
    e->alloc_order.clear();   // a checkpoint's frames: not in process-start order (no tick model)
    for (auto &kv : img.pages) e->pages[kv.first] = kv.second;
    // memory-fault candidates, as at process start (the ELF's writable
    // segments and the stack): every mapped page no read-only PT_LOAD covers
    e->mem_pages.clear();
    for (auto &kv : img.pages) {
        const uint64_t a = kv.first << 12;
        bool ro = false, w = false;
        for (const fi_engine::Seg &g : segs)
            if (a >= g.lo && a < g.hi) (g.w ? w : ro) = true;
        if (w || !ro) e->mem_pages.push_back(a);
    }
    e->brk0 = img.brk;
    e->svma_lo = e->svma_hi = 0;
    for (size_t i = 0; i < img.vmas.size(); i++)
        if (img.vma_names[i] == "stack") { e->svma_lo = img.vmas[i].first; e->svma_hi = img.vmas[i].second; }
    // a VMA list other than argsInit's lone stack VMA, or another mmap end:
    // the trials start from it (DevCtx::vm0)
    const bool plain = img.vmas.size() == 1 && img.vma_names[0] == "stack" && img.mmap_end == 0x4000000000000000ULL;
    e->vm0_on = !plain;
    if (e->vm0_on) {
        e->vm0 = VmState{};
        e->vm0.brk = img.brk; e->vm0.mmap_end = img.mmap_end;
        e->vm0.nvma = (uint32_t)img.vmas.size();
        for (size_t i = 0; i < img.vmas.size(); i++) { e->vm0.vma[i][0] = img.vmas[i].first; e->vm0.vma[i][1] = img.vmas[i].second; }
    }
    e->fp0_on = img.fp_state;
    memcpy(e->fp0, img.fregs, sizeof e->fp0);
    e->fcsr0 = img.fflags | (img.frm << 5);
    e->tick0 = img.tick0;
    e->sp0 = img.regs[2];
    e->stack_min0 = img.stack_min & ~(kPage - 1);
    fi_status st2 = finish_load(e, img.regs, img.pc);
    if (st2) return st2;
    if (e->vm0_on) {
        HIPCHK(hipMalloc(&e->d_vm0, sizeof(VmState)));
        HIPCHK(hipMemcpy(e->d_vm0, &e->vm0, sizeof(VmState), hipMemcpyHostToDevice));
    }
    if (e->fp0_on) {
        HIPCHK(hipMalloc(&e->d_fp0, 32 * 8));
        HIPCHK(hipMemcpy(e->d_fp0, e->fp0, 32 * 8, hipMemcpyHostToDevice));
    }
    return FI_OK;
}

// Private pages per trial of the second pass (chunk_end) and, with the
// overflow pool, a trial's capacity in the first: 16 P, at least 256.

static fi_status ensure_work(fi_engine *e, uint64_t n) {
    if (n <= e->cap) return FI_OK;
    free_work(e);
    const uint64_t c = n;
    HIPCHK(hipMalloc(&e->d_sites, c * sizeof(fi_site)));
    HIPCHK(hipMalloc(&e->d_sites_alt, c * sizeof(fi_site)));
    HIPCHK(hipMalloc(&e->d_keys, c * 8));
    HIPCHK(hipMalloc(&e->d_keys2, c * 8));
    HIPCHK(hipMalloc(&e->d_perm, c * 4));
    HIPCHK(hipMalloc(&e->d_perm2, c * 4));
    HIPCHK(sort_pairs_bytes(c, e->tmp_bytes));
    HIPCHK(hipMalloc(&e->d_tmp, std::max<size_t>(e->tmp_bytes, 16)));
    HIPCHK(hipMalloc(&e->d_out, c * sizeof(fi_outcome)));
    HIPCHK(hipMalloc(&e->d_out_alt, c * sizeof(fi_outcome)));
    HIPCHK(hipMalloc(&e->d_eff, c * 8));
    HIPCHK(hipMalloc(&e->d_hist, sizeof(fi_histogram)));
    HIPCHK(hipMalloc(&e->d_stats, kNStats * sizeof(unsigned long long)));
    HIPCHK(hipMalloc(&e->d_wave_dbg, c * 10 * sizeof(uint64_t)));
    HIPCHK(hipMalloc(&e->d_priv, c * e->cfg.private_pages * kPage));
    HIPCHK(hipMalloc(&e->d_priv_vpn, c * e->cfg.private_pages * 8));
    HIPCHK(hipMalloc(&e->d_save, c * sizeof(LaneSave)));
    HIPCHK(hipMalloc(&e->d_vm, c * sizeof(VmState)));
    HIPCHK(hipMalloc(&e->d_fregs, c * 32 * sizeof(uint64_t)));
    HIPCHK(hipMalloc(&e->d_inpos, c * sizeof(uint64_t)));
    HIPCHK(hipMalloc(&e->d_surv[0], c * 4));
    HIPCHK(hipMalloc(&e->d_surv[1], c * 4));
    HIPCHK(hipMalloc(&e->d_cnt, 16 * 4));
    HIPCHK(hipMalloc(&e->d_skeys, c * 8));
    HIPCHK(hipMalloc(&e->d_skeys2, c * 8));
    HIPCHK(hipMalloc(&e->d_svals, c * 4));
    HIPCHK(hipMalloc(&e->d_svals2, c * 4));
    HIPCHK(hipMalloc(&e->d_wrange, c * 8));
    HIPCHK(hipMalloc(&e->d_nwaves, 16 * 4));
    HIPCHK(hipMalloc(&e->d_split, 64 * 4));
    HIPCHK(hipMalloc(&e->d_dmap, c * kDmapWords * 4));
    HIPCHK(hipMalloc(&e->d_redo_idx, 2 * c * 4));
    HIPCHK(hipMalloc(&e->d_redo_cnt, 16));
    HIPCHK(hipMalloc(&e->d_redo_sites, c * sizeof(fi_site)));
    HIPCHK(hipMalloc(&e->d_redo_out, c * sizeof(fi_outcome)));
    if (!e->h_redo_cnt) HIPCHK(hipHostMalloc(&e->h_redo_cnt, 16));
    for (auto &ev : e->ev_cnt)
        if (!ev) HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    // (the pinned staging of host-bound outcomes is made on first use:
    // chunk_end; device-resident runs never need it)
    for (int i = 0; i < 2; i++)
        if (!e->ev_stage[i]) HIPCHK(hipEventCreateWithFlags(&e->ev_stage[i], hipEventDisableTiming));
    // overflow pool: a trial past P pages takes a block of P' - P more (P' the
    // redo pass's page count), one block per 2048 slots (at least 64)
    {
        const uint64_t P = e->cfg.private_pages, P2 = redo_pages(P);
        if (!(e->cfg.flags & FI_CFG_NO_OVERFLOW) && P2 > P) {
            e->ov_pages = (uint32_t)(P2 - P);
            e->ov_blocks = (uint32_t)std::max<uint64_t>(64, c / 2048);
            HIPCHK(hipMalloc(&e->d_ov, (uint64_t)e->ov_blocks * e->ov_pages * kPage));
            HIPCHK(hipMalloc(&e->d_ov_vpn, (uint64_t)e->ov_blocks * e->ov_pages * 8));
            HIPCHK(hipMalloc(&e->d_ov_of, c * 4));
            HIPCHK(hipMalloc(&e->d_ov_next, 16));
        }
    }
    e->cap = c;
    return FI_OK;
}

// The rewritten-code map's granule: one byte, coarser for large code so that
// a slot's map stays within kDmapWords x 32 bits (the solo kernel's LDS
// copy, fi_trial.hip kDmapWords).  (Byte granules: a store next to a loop's
// instructions leaves the loop's translated blocks usable.)
static void dmap_params(const fi_engine *e, uint32_t &shift, uint32_t &words) {
    const uint64_t cb = e->code_hi > e->code_lo ? e->code_hi - e->code_lo : 1;
    shift = 0;
    while ((cb >> shift) >= kDmapWords * 32) shift++;
    words = (uint32_t)((((cb + (1ULL << shift) - 1) >> shift) + 31) / 32);
}

static DevCtx base_ctx(fi_engine *e) {
    DevCtx c{};
    c.pre = e->d_pre; c.text_lo = e->text_lo; c.text_hi = e->text_hi; c.pre_ok = e->pre_ok ? 1 : 0;
    c.text_bytes = (uint32_t)(e->text_hi - e->text_lo);
    c.code_lo = e->code_lo; c.code_hi = e->code_hi;
    c.snaps = e->d_snaps; c.snap_tab = e->d_tab; c.pool = e->d_pool; c.zero_page = e->d_zero;
    const bool start = !(e->cfg.flags & FI_CFG_NO_SNAPSHOT_START);
    c.n_snap = (uint32_t)e->snaps.size();
    c.snap_start = (start && !e->golden_fp) ? 1 : 0;
    c.snap_interval = e->snap_I;
    c.early_exit = (!(e->cfg.flags & FI_CFG_NO_EARLY_EXIT) && e->snaps.size() > 1 && !e->golden_fp) ? 1 : 0;
    if (c.early_exit && !(e->cfg.flags & FI_CFG_NO_SDC_EXIT)) c.early_exit = 3;   // bit 1: SDC early exit
    c.hang_proof = (e->cfg.flags & FI_CFG_NO_HANG_PROOF) ? 0 : 1;
    c.gout = e->d_gout; c.gerr = e->d_gerr; c.gout_len = e->gout.size(); c.gerr_len = e->gerr.size();
    c.gexit = e->golden.exit_code;
    c.gdetail = e->gdetail;
    c.gsub = e->gsub;
    c.gninst = e->golden.ninst;
    c.priv_pages = e->cfg.private_pages;
    c.hang_cap = e->golden.ninst * e->cfg.hang_factor_x16 / 16 + 1000;
    c.protect_mask = e->protect;
    c.protect_opc = e->protect_opc;
    c.shadow_bits = e->issue_on ? e->d_shadow : nullptr;
    c.priv_frames = e->d_priv; c.priv_vpn = e->d_priv_vpn;
    c.ov_frames = e->d_ov; c.ov_vpn = e->d_ov_vpn; c.ov_of = e->d_ov_of; c.ov_next = e->d_ov_next;
    c.ov_blocks = e->ov_blocks; c.ov_pages = e->ov_pages;
    c.tx_sink = e->d_sink;
    c.fregs = e->d_fregs;
    c.wave_dbg = e->d_wave_dbg;
    c.stats = e->d_stats;
    c.brk0 = e->brk0; c.svma_lo = e->svma_lo; c.svma_hi = e->svma_hi; c.vm = e->d_vm;
    c.simt_min = (e->cfg.flags & FI_CFG_SIMT) ? 8u : 0u;
    c.rnd_tab = e->d_rnd; c.rnd_len = e->d_rnd ? kRndLen : 0; c.clk_period = e->clk_period;
    c.exe_path = e->d_exe; c.exe_len = e->d_exe ? e->exe_path.size() : 0;
    c.tick0 = e->tick0;
    c.clk_until = e->clk_until;
    c.clk_esc = e->clk_esc;
    c.stdin_data = e->stdin_on ? e->d_stdin : nullptr;
    c.stdin_len = e->stdin_on ? e->stdin_data.size() : 0;
    c.in_pos = e->d_inpos;
    c.fp0 = e->fp0_on ? e->d_fp0 : nullptr;
    c.fcsr0 = e->fcsr0;
    c.vm0 = e->vm0_on ? e->d_vm0 : nullptr;
    c.dmap = e->d_dmap;
    dmap_params(e, c.dmap_shift, c.dmap_words);
    c.lanes = e->cfg.lanes_per_wave;
    c.mem_live = (e->mem_live && !(e->cfg.flags & FI_CFG_NO_EARLY_EXIT)) ? 1 : 0;
    c.mw_n = e->mw_n; c.mw_addr = e->d_mw_addr; c.mw_off = e->d_mw_off; c.mw_ev = e->d_mw_ev;
    return c;
}

// One golden (fault-free, record-mode) launch: a single lane from snapshot 0.
// P private pages; rec_* capture snapshots every rec_I instructions (0 = off).
static fi_status golden_launch(fi_engine *e, uint32_t P, uint64_t rec_I, uint32_t rec_max, SnapState *d_rs,
                               uint8_t *d_rp, uint64_t *d_rv, uint32_t *d_trace, uint32_t trace_cap, uint8_t *d_ro,
                               uint8_t *d_re, uint64_t rec_cap, fi_outcome &o, unsigned long long *stats,
                               MemEv *d_mem = nullptr, uint32_t mem_cap = 0) {
    uint8_t *d_gpriv = nullptr;
    uint64_t *d_gvpn = nullptr;
    HIPCHK(hipMalloc(&d_gpriv, (uint64_t)P * kPage));
    HIPCHK(hipMalloc(&d_gvpn, (uint64_t)P * 8));
    uint64_t *d_gfregs = nullptr;
    HIPCHK(hipMalloc(&d_gfregs, 33 * sizeof(uint64_t)));   // 32 FP registers + fd 0's offset
    DevCtx c = base_ctx(e);
    c.fregs = d_gfregs;
    c.in_pos = d_gfregs + 32;
    c.dmap = nullptr;
    c.ov_blocks = 0;   // (the golden run has its own P pages, no overflow pool)
    c.record = 1;
    c.early_exit = 0;
    c.snap_start = 0;
    c.rec_out = d_ro; c.rec_err = d_re; c.rec_cap = rec_cap;
    c.hang_cap = 1ULL << 30;   // golden safety cap
    c.priv_pages = P; c.priv_frames = d_gpriv; c.priv_vpn = d_gvpn;
    c.rec_snaps = d_rs; c.rec_pages = d_rp; c.rec_vpns = d_rv; c.rec_interval = rec_I; c.rec_max_snaps = rec_max;
    c.rec_trace = d_trace; c.rec_trace_cap = d_trace ? trace_cap : 0;
    c.rec_mem = d_mem; c.rec_mem_cap = d_mem ? mem_cap : 0;
    c.mem_live = 0;
    c.out = e->d_out;
    c.n = 1;
    c.n_slots = 1;
    c.sites = nullptr; c.perm = nullptr;
    hipError_t err = hipMemsetAsync(e->d_stats, 0, kNStats * sizeof(unsigned long long), e->stream);
    if (err == hipSuccess) err = hipEventRecord(e->ev0, e->stream);
    if (err == hipSuccess) err = launch_trials(c, e->stream);
    if (err == hipSuccess) err = hipEventRecord(e->ev1, e->stream);
    if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
    float ms = 0;
    if (err == hipSuccess) err = hipEventElapsedTime(&ms, e->ev0, e->ev1);
    if (err == hipSuccess) err = hipMemcpy(&o, e->d_out, sizeof o, hipMemcpyDeviceToHost);
    if (err == hipSuccess) err = hipMemcpy(stats, e->d_stats, kNStats * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    (void)hipFree(d_gpriv);
    (void)hipFree(d_gfregs);
    (void)hipFree(d_gvpn);
    if (err != hipSuccess) return fail(e, FI_E_HIP, "golden launch: %s", hipGetErrorString(err));
    e->last_ms = ms;
    if (o.cls != FI_MASKED)
        return fail(e, FI_E_GOLDEN, "golden run did not exit normally (class %u sub %u detail %#x after %llu insts)",
                    o.cls, o.sub, o.detail, (unsigned long long)o.ninst);
    return FI_OK;
}

// Memory liveness index (DevCtx::mw_*): the golden run's data accesses split
// into 8-byte words, per word in time order as numInst << 16 | bytes read << 8
// | bytes written.  A trial's memory fault looks its word up at injection
// (fi_trial.hip:mem_dead).  complete = the access trace did not overflow and
// every golden instruction came from the pre-decoded text.
static fi_status build_mem_index(fi_engine *e, const std::vector<MemEv> &mev, bool complete) {
    free_mem_index(e);
    if (!complete) return FI_OK;
    std::vector<std::pair<uint64_t, uint64_t>> ent;   // (word, event)
    const uint64_t kMaxEnt = 1ULL << 26;
    for (const MemEv &ev : mev) {
        const uint64_t len = ev.len_kind & ((1u << 30) - 1), kind = ev.len_kind >> 30;
        const uint64_t end = ev.addr + len;
        if (end < ev.addr) return FI_OK;
        for (uint64_t a = ev.addr; a < end;) {
            const uint64_t wd = a & ~7ULL, we = std::min(end, wd + 8);
            uint64_t bm = 0;
            for (uint64_t b = a; b < we; b++) bm |= 1ULL << (b - wd);
            ent.emplace_back(wd, ((uint64_t)(ev.t & ~kMemEvProxy) << 16) | ((kind & 1) ? bm << 8 : 0) |
                                     ((kind & 2) ? bm : 0));
            if (ent.size() > kMaxEnt) return FI_OK;
            a = we;
        }
    }
    std::stable_sort(ent.begin(), ent.end(), [](const auto &x, const auto &y) { return x.first < y.first; });
    std::vector<uint64_t> addr, evs;
    std::vector<uint32_t> off;
    evs.reserve(ent.size());
    for (size_t i = 0; i < ent.size(); i++) {
        if (i == 0 || ent[i].first != ent[i - 1].first) {
            addr.push_back(ent[i].first);
            off.push_back((uint32_t)i);
        }
        evs.push_back(ent[i].second);
    }
    off.push_back((uint32_t)ent.size());
    HIPCHK(hipMalloc(&e->d_mw_addr, std::max<size_t>(addr.size(), 1) * 8));
    HIPCHK(hipMalloc(&e->d_mw_off, off.size() * 4));
    HIPCHK(hipMalloc(&e->d_mw_ev, std::max<size_t>(evs.size(), 1) * 8));
    if (!addr.empty()) HIPCHK(hipMemcpy(e->d_mw_addr, addr.data(), addr.size() * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->d_mw_off, off.data(), off.size() * 4, hipMemcpyHostToDevice));
    if (!evs.empty()) HIPCHK(hipMemcpy(e->d_mw_ev, evs.data(), evs.size() * 8, hipMemcpyHostToDevice));
    e->mw_n = (uint32_t)addr.size();
    e->mem_live = true;
    return FI_OK;
}

// The golden run under TimingSimpleCPU (fi_tick.cpp, fi_timing.cpp): its
// attempts as requests, then their ticks.  t_status says why not, if not.
static void tick_prepare(fi_engine *e, const std::vector<MemEv> &mev, bool mev_ok) {
    e->t_ops.clear(); e->t_att.clear(); e->t_ticks.clear(); e->t_stats = fi_timing_stats{};
    if (e->cpu_model != FI_CPU_TIMING) { e->t_status = "the CPU model is AtomicSimpleCPU (fi_set_cpu_model)"; return; }
    if (e->alloc_order.empty()) { e->t_status = "a checkpoint start: its frame order is not known"; return; }
    if (e->clk_until) { e->t_status = "the golden run reads curTick: its output depends on the CPU model"; return; }
    if (e->golden_unmapped) { e->t_status = "the golden run unmaps memory: freed frames are reused"; return; }
    if (!mev_ok || e->g_trace.empty()) { e->t_status = "the golden access record is incomplete"; return; }
    TickGoldenIn in{&e->g_trace, &e->g_pre, e->text_lo, &mev, &e->alloc_order, e->stack_min0, e->svma_lo,
                    e->svma_hi, kStackBase, kMaxStack, e->golden.ninst, e->golden.ncycles};
    std::string why = build_tick_attempts(in, e->t_ops, e->t_att);
    if (why.empty()) {
        e->t_ticks.resize(e->t_ops.size());
        if (fi_timing_model_run(e->t_ops.data(), e->t_ops.size(), &e->tparams, e->t_ticks.data(), &e->t_stats))
            why = "the timing model rejected the golden requests (a state gem5 asserts on)";
    }
    if (!why.empty()) {
        e->t_ops.clear(); e->t_att.clear(); e->t_ticks.clear();
        e->t_status = why;
        return;
    }
    e->t_status = "";
}

fi_status fi_golden_run(fi_engine *e, fi_golden_info *out) {
    if (!e) return FI_E_ARG;
    if (!e->loaded) return fail(e, FI_E_STATE, "fi_golden_run: no workload loaded");
    HIPCHK(hipSetDevice(e->dev));
    fi_status st = ensure_work(e, 64);
    if (st) return st;
    // back to the process-start image only
    e->t_status = "no golden run";
    e->t_ops.clear(); e->t_att.clear(); e->t_ticks.clear();
    e->snaps.resize(1);
    e->tab.resize(e->n_start_frames);
    e->pool.resize((uint64_t)e->n_start_frames * kPage);
    e->snap_I = 1ULL << 62;
    e->pre_ok = true;
    e->have_golden = false;
    st = upload_snaps(e);
    if (st) return st;

    // ---- pass 1: the golden run itself (output, instruction count, footprint)
    const uint64_t rec_cap = 1 << 24;
    const uint32_t kGoldenPages = 4096;   // 16 MiB of written pages
    uint8_t *d_rec_out = nullptr, *d_rec_err = nullptr;
    HIPCHK(hipMalloc(&d_rec_out, rec_cap));
    HIPCHK(hipMalloc(&d_rec_err, rec_cap));
    fi_outcome o;
    unsigned long long stats[kNStats];
    st = golden_launch(e, kGoldenPages, 0, 0, nullptr, nullptr, nullptr, nullptr, 0, d_rec_out, d_rec_err, rec_cap, o,
                       stats);
    if (st) { (void)hipFree(d_rec_out); (void)hipFree(d_rec_err); return st; }
    const double golden_ms = e->last_ms;
    const uint64_t ol = stats[4], el = stats[5];
    const uint64_t gpages = stats[2];
    if (ol > rec_cap || el > rec_cap) {
        (void)hipFree(d_rec_out); (void)hipFree(d_rec_err);
        return fail(e, FI_E_GOLDEN, "golden output exceeds %llu bytes", (unsigned long long)rec_cap);
    }
    if (gpages >= kGoldenPages) {
        (void)hipFree(d_rec_out); (void)hipFree(d_rec_err);
        return fail(e, FI_E_GOLDEN, "golden run writes more than %u pages", kGoldenPages);
    }
    e->gout.assign(ol, 0);
    e->gerr.assign(el, 0);
    if (ol) HIPCHK(hipMemcpy(e->gout.data(), d_rec_out, ol, hipMemcpyDeviceToHost));
    if (el) HIPCHK(hipMemcpy(e->gerr.data(), d_rec_err, el, hipMemcpyDeviceToHost));
    dfree(e->d_gout); dfree(e->d_gerr);
    HIPCHK(hipMalloc(&e->d_gout, std::max<uint64_t>(ol, 1)));
    HIPCHK(hipMalloc(&e->d_gerr, std::max<uint64_t>(el, 1)));
    if (ol) HIPCHK(hipMemcpy(e->d_gout, e->gout.data(), ol, hipMemcpyHostToDevice));
    if (el) HIPCHK(hipMemcpy(e->d_gerr, e->gerr.data(), el, hipMemcpyHostToDevice));
    e->golden = fi_golden_info{};
    e->golden.ninst = o.ninst;
    e->golden.ncycles = stats[3];
    e->golden.exit_code = o.exit_code;
    e->golden.stdout_len = ol;
    e->golden.stderr_len = el;
    e->golden.fetch_bytes = stats[0];
    e->golden.data_bytes = stats[1];
    e->gdetail = o.detail;
    e->gsub = o.sub;
    e->golden_fp = stats[22] != 0;
    e->clk_until = stats[52];

    // ---- pass 2: the same run again, capturing a snapshot every I committed
    // instructions (state + every page written so far), within ~1 GiB
    uint64_t I = std::max<uint64_t>(e->cfg.snapshot_interval ? e->cfg.snapshot_interval : 256, 16);
    const uint32_t P = (uint32_t)std::max<uint64_t>(gpages, 1);
    while (o.ninst / I + 2 > 65536 || (o.ninst / I + 2) * P * kPage > (1ULL << 30)) I *= 2;
    const uint32_t rec_max = (uint32_t)(o.ninst / I + 2);
    SnapState *d_rs = nullptr;
    uint8_t *d_rp = nullptr;
    uint64_t *d_rv = nullptr;
    HIPCHK(hipMalloc(&d_rs, (uint64_t)rec_max * sizeof(SnapState)));
    HIPCHK(hipMalloc(&d_rp, (uint64_t)rec_max * P * kPage));
    HIPCHK(hipMalloc(&d_rv, (uint64_t)rec_max * P * 8));
    // golden trace for the register liveness pass: one entry per committed
    // instruction and ecall (capped; without it every register counts as live)
    const uint32_t trace_cap = (uint32_t)std::min<uint64_t>(o.ninst + 4096, 1ULL << 26);
    uint32_t *d_trace = nullptr;
    HIPCHK(hipMalloc(&d_trace, (uint64_t)trace_cap * 4));
    // and its data accesses for the memory liveness index
    const uint32_t mem_cap = (uint32_t)std::min<uint64_t>(2 * o.ninst + 4096, 1ULL << 24);
    MemEv *d_mem = nullptr;
    HIPCHK(hipMalloc(&d_mem, (uint64_t)mem_cap * sizeof(MemEv)));
    fi_outcome o2;
    st = golden_launch(e, P, I, rec_max, d_rs, d_rp, d_rv, d_trace, trace_cap, d_rec_out, d_rec_err, rec_cap, o2,
                       stats, d_mem, mem_cap);
    (void)hipFree(d_rec_out);
    (void)hipFree(d_rec_err);
    std::vector<SnapState> rs;
    std::vector<uint8_t> rp;
    std::vector<uint64_t> rv;
    std::vector<uint32_t> trace;
    std::vector<PreInst> pre;
    uint32_t ns = 0;
    const uint64_t n_events = stats[15];
    if (!st && n_events <= trace_cap) {
        trace.resize(n_events);
        pre.resize((e->text_hi - e->text_lo) / 2);
        hipError_t err = hipMemcpy(trace.data(), d_trace, n_events * 4, hipMemcpyDeviceToHost);
        if (err == hipSuccess) err = hipMemcpy(pre.data(), e->d_pre, pre.size() * sizeof(PreInst), hipMemcpyDeviceToHost);
        for (auto &p : pre) p.flags &= (uint8_t)~(kPreLeader | kPreOddLeader);
        if (err != hipSuccess) st = fail(e, FI_E_HIP, "trace download: %s", hipGetErrorString(err));
    }
    (void)hipFree(d_trace);
    const uint64_t n_mem = stats[25];
    std::vector<MemEv> mev;
    if (!st && n_mem <= mem_cap) {
        mev.resize(n_mem);
        hipError_t err = n_mem ? hipMemcpy(mev.data(), d_mem, n_mem * sizeof(MemEv), hipMemcpyDeviceToHost) : hipSuccess;
        if (err != hipSuccess) st = fail(e, FI_E_HIP, "access trace download: %s", hipGetErrorString(err));
    }
    (void)hipFree(d_mem);
    if (!st) {
        ns = (uint32_t)std::min<unsigned long long>(stats[13], rec_max);
        rs.resize(ns);
        rp.resize((uint64_t)ns * P * kPage);
        rv.resize((uint64_t)ns * P);
        hipError_t err = hipMemcpy(rs.data(), d_rs, ns * sizeof(SnapState), hipMemcpyDeviceToHost);
        if (err == hipSuccess) err = hipMemcpy(rp.data(), d_rp, rp.size(), hipMemcpyDeviceToHost);
        if (err == hipSuccess) err = hipMemcpy(rv.data(), d_rv, rv.size() * 8, hipMemcpyDeviceToHost);
        if (err != hipSuccess) st = fail(e, FI_E_HIP, "snapshot download: %s", hipGetErrorString(err));
    }
    (void)hipFree(d_rs); (void)hipFree(d_rp); (void)hipFree(d_rv);
    if (st) return st;
    if (o2.ninst != o.ninst || o2.detail != o.detail || stats[13] != o.ninst / I + 1)
        return fail(e, FI_E_GOLDEN, "golden capture pass diverged from the golden run");

    // ---- host: deduplicate frames and build one sorted page table per snapshot
    std::map<uint64_t, uint32_t> cur;   // vpn -> frame of its latest version
    for (uint32_t i = 0; i < e->n_start_frames; i++) cur[e->tab[i].vpn] = e->tab[i].frame;
    std::vector<SnapState> snaps;
    std::vector<PageEnt> tab;
    for (uint32_t k = 0; k < ns; k++) {
        SnapState S = rs[k];
        for (uint32_t i = 0; i < S.tab_n; i++) {
            const uint64_t vpn = rv[(uint64_t)k * P + i];
            const uint8_t *pg = rp.data() + (((uint64_t)k * P + i) << 12);
            auto it = cur.find(vpn);
            if (it != cur.end() && !memcmp(e->pool.data() + ((uint64_t)it->second << 12), pg, kPage)) continue;
            const uint32_t f = (uint32_t)(e->pool.size() / kPage);
            e->pool.insert(e->pool.end(), pg, pg + kPage);
            cur[vpn] = f;
            // the pre-decoded text stays valid only if the golden run never rewrites it
            const uint64_t va = vpn << 12;
            if (va < e->code_hi && va + kPage > e->code_lo) {   // bytes of the code range in this page
                const uint64_t a = std::max(va, e->code_lo), b = std::min(va + kPage, e->code_hi);
                auto org = e->pages.find(vpn);
                if (org == e->pages.end() || memcmp(org->second.data() + (a - va), pg + (a - va), b - a))
                    e->pre_ok = false;
            }
        }
        S.tab_off = (uint32_t)tab.size();
        S.tab_n = (uint32_t)cur.size();
        for (auto &kv : cur) {
            PageEnt pe{};
            pe.vpn = kv.first;
            pe.frame = kv.second;
            tab.push_back(pe);
        }
        snaps.push_back(S);
    }
    // ---- register liveness at each snapshot: backward over the golden trace,
    // live = (live - writes) | reads; an ecall reads a0..a7.  Unknown entries
    // (trace overflow, pc outside the pre-decoded text) leave every register live.
    bool live_ok = !trace.empty() || n_events == 0;
    std::vector<uint32_t> rmask(trace.size()), wmask(trace.size());
    for (size_t i = 0; live_ok && i < trace.size(); i++) {
        const uint32_t h = trace[i] & 0x7FFFFFFFu;
        if (h >= pre.size() || !(pre[h].flags & kPreValid)) { live_ok = false; break; }
        const PreInst &p = pre[h];
        uint32_t r = 0, w = 0;
        if ((p.flags & kPreRs1) && p.rs1) r |= 1u << p.rs1;
        if ((p.flags & kPreRs2) && p.rs2) r |= 1u << p.rs2;
        if ((trace[i] & 0x80000000u) || p.op == OP_m5op) r |= 0x3FC00u;   // x10..x17 (an M5Op's ABI arguments)
        else if ((p.flags & kPreRd) && p.rd) w |= 1u << p.rd;
        rmask[i] = r;
        wmask[i] = w;
    }
    {
        uint32_t live = 0;
        int64_t ev = (int64_t)trace.size() - 1;
        for (int64_t k = (int64_t)snaps.size() - 1; k >= 0; k--) {
            if (!live_ok) { snaps[k].live = 0xFFFFFFFEu; continue; }
            for (; ev >= (int64_t)snaps[k].trace_pos; ev--) live = (live & ~wmask[ev]) | rmask[ev];
            snaps[k].live = live & ~1u;
        }
    }
    e->snaps = snaps;
    e->tab = tab;
    e->snap_I = I;
    e->g_pre.clear(); e->g_trace.clear();
    if (live_ok && !trace.empty()) { e->g_pre = pre; e->g_trace = trace; }
    // ---- first-access index (DESIGN.md §4 "first-access forwarding"): a
    // register flipped at numInst t is neither read nor written by the golden
    // run before its next access, so flipping it at that access instead gives
    // the same machine; written first (or never touched again) it is dead.
    free_fw(e);
    {
        const bool ok = live_ok && !trace.empty() && o.ninst < (1ULL << 29);
        std::vector<uint32_t> off(33, 0), ev;
        if (ok) {
            for (size_t i = 0; i < trace.size(); i++)
                for (uint32_t m = (rmask[i] | wmask[i]) & ~1u; m; m &= m - 1) off[__builtin_ctz(m) + 1]++;
            for (int r = 0; r < 32; r++) off[r + 1] += off[r];
            ev.resize(off[32]);
            std::vector<uint32_t> at(off.begin(), off.end() - 1);
            uint64_t t = 0;
            for (size_t i = 0; i < trace.size(); i++) {
                const bool ecall = (trace[i] & 0x80000000u) != 0;
                const uint32_t key = (uint32_t)(2 * t + (ecall ? 0 : 1));
                for (uint32_t m = (rmask[i] | wmask[i]) & ~1u; m; m &= m - 1) {
                    const int r = __builtin_ctz(m);
                    ev[at[r]++] = (key << 1) | ((rmask[i] >> r) & 1u);
                }
                if (!ecall) t++;
            }
            HIPCHK(hipMalloc(&e->d_fw_off, 33 * 4));
            HIPCHK(hipMalloc(&e->d_fw_ev, std::max<size_t>(ev.size(), 1) * 4));
            HIPCHK(hipMemcpy(e->d_fw_off, off.data(), 33 * 4, hipMemcpyHostToDevice));
            if (!ev.empty()) HIPCHK(hipMemcpy(e->d_fw_ev, ev.data(), ev.size() * 4, hipMemcpyHostToDevice));
            e->fw_ok = true;
        }
    }
    st = upload_snaps(e);
    if (st) return st;
    st = build_mem_index(e, mev, live_ok && n_mem <= mem_cap);
    if (st) return st;
    e->golden_unmapped = stats[62] != 0;
    tick_prepare(e, mev, !trace.empty() && n_mem <= mem_cap);

    // ---- translate the golden basic blocks and build the trial kernel with
    // them (hipRTC); the static kernel stays the fallback
    free_tx(e);
    if (e->cfg.flags & FI_CFG_NO_TRANSLATE) e->tx_status = "disabled (FI_CFG_NO_TRANSLATE)";
    else if (!e->pre_ok) e->tx_status = "golden run rewrites its text";
    else if (!live_ok || trace.empty()) e->tx_status = "golden trace unavailable";
    else {
        // (snapshot pcs are not leaders: they fall all over the hot loops and
        // would cut the blocks into single instructions; a wave that starts
        // mid-block steps to the next leader in the interpreter)
        const std::vector<uint64_t> pcs;
        std::vector<uint32_t> leaders;
        std::vector<LoopEst> loops;
        uint32_t n_tx = 0;
        std::string body = translate_blocks(pre, e->text_lo, trace, pcs, leaders, n_tx, true, &loops);
        if (n_tx > 24000) {   // the odd-pc streams make it too large: without them
            leaders.clear();
            loops.clear();
            body = translate_blocks(pre, e->text_lo, trace, pcs, leaders, n_tx, false, &loops);
        }
        if (!loops.empty() && !(e->cfg.flags & FI_CFG_NO_LOOP_ORDER)) {
            HIPCHK(hipMalloc(&e->d_loops, loops.size() * sizeof(LoopEst)));
            HIPCHK(hipMemcpy(e->d_loops, loops.data(), loops.size() * sizeof(LoopEst), hipMemcpyHostToDevice));
            e->n_loops = (uint32_t)loops.size();
        }
        e->tx_body = body;
        hipDeviceProp_t prop;
        HIPCHK(hipGetDeviceProperties(&prop, e->dev));
        if (const char *dump = getenv("SHREWD_FI_DUMP_TX")) {   // diagnostics: the generated blocks
            if (FILE *f = fopen(dump, "w")) { fputs(body.c_str(), f); fclose(f); }
        }
        if (leaders.empty()) {   // nothing hot: the static kernels (pre-decoded + general interpreter) run everything
            e->tx_status = "nothing to translate (no code run twice)";
        } else if (n_tx > 24000) {   // more than the load-time compiler handles in reasonable time
            e->tx_status = "translation too large";
        } else {
            auto j = std::make_shared<JitJob>();
            j->body = body;
            j->arch = prop.gcnArchName;
            j->odd = jit_has_odd(body);
            j->use_cache = !(e->cfg.flags & FI_CFG_JIT_NO_CACHE);
            for (uint32_t h : leaders) pre[h & 0x7FFFFFFFu].flags |= (h >> 31) ? kPreOddLeader : kPreLeader;
            e->jit_pre = std::move(pre);
            e->jit_blocks = leaders.size();
            e->jit_insts = n_tx;
            e->jit = j;
            e->tx_status = "compiling";
            e->jit_threads.emplace_back(std::thread(jit_job_run, j), j);
        }
    }
    e->last_ms = golden_ms;
    e->golden.snapshots = e->snaps.size();
    e->golden.snapshot_interval = I;
    e->golden.snapshot_frames = e->pool.size() / kPage;
    e->have_golden = true;
    if (e->issue_on) {   // the model follows the new golden run
        st = compute_shadow(e);
        if (st) return st;
    }
    if (out) *out = e->golden;
    return FI_OK;
}

fi_status fi_golden_stdout(fi_engine *e, uint8_t *buf, uint64_t cap, uint64_t *len) {
    if (!e || !e->have_golden) return fail(e, FI_E_STATE, "no golden run");
    if (buf && cap) memcpy(buf, e->gout.data(), std::min<uint64_t>(cap, e->gout.size()));
    if (len) *len = e->gout.size();
    return FI_OK;
}

fi_status fi_golden_stderr(fi_engine *e, uint8_t *buf, uint64_t cap, uint64_t *len) {
    if (!e || !e->have_golden) return fail(e, FI_E_STATE, "no golden run");
    if (buf && cap) memcpy(buf, e->gerr.data(), std::min<uint64_t>(cap, e->gerr.size()));
    if (len) *len = e->gerr.size();
    return FI_OK;
}

fi_status fi_set_campaign(fi_engine *e, uint64_t seed, uint64_t structures, uint32_t burst) {
    if (!e) return FI_E_ARG;
    structures &= ~1ULL;
    structures &= (1ULL << FI_N_STRUCT) - 1;
    if (!structures) return fail(e, FI_E_ARG, "no fault structures selected");
    if (burst < 1 || burst > 64) return fail(e, FI_E_ARG, "burst must be 1..64");
    e->seed = seed; e->structures = structures; e->burst = burst;
    e->bits = ~0ULL;
    return FI_OK;
}

fi_status fi_set_exe_path(fi_engine *e, const char *path) {
    if (!e) return FI_E_ARG;
    if (e->have_golden) return fail(e, FI_E_STATE, "fi_set_exe_path: set before fi_golden_run (the golden run sees it)");
    HIPCHK(hipSetDevice(e->dev));
    e->exe_path = path ? path : "";
    if (e->exe_path.size() >= 4096) { e->exe_path.clear(); return FI_E_ARG; }   // PATH_MAX
    dfree(e->d_exe);
    if (!e->exe_path.empty()) {
        HIPCHK(hipMalloc(&e->d_exe, e->exe_path.size()));
        HIPCHK(hipMemcpy(e->d_exe, e->exe_path.data(), e->exe_path.size(), hipMemcpyHostToDevice));
    }
    return FI_OK;
}

fi_status fi_set_stdin(fi_engine *e, const uint8_t *data, uint64_t len) {
    if (!e) return FI_E_ARG;
    if (e->have_golden) return fail(e, FI_E_STATE, "fi_set_stdin: set before fi_golden_run (the golden run reads it)");
    if (data && len >= (1ULL << 40)) return fail(e, FI_E_ARG, "fi_set_stdin: input larger than 1 TiB");
    HIPCHK(hipSetDevice(e->dev));
    dfree(e->d_stdin);
    e->stdin_data.clear();
    e->stdin_on = data != nullptr;
    if (!data) return FI_OK;
    e->stdin_data.assign(data, data + len);
    HIPCHK(hipMalloc(&e->d_stdin, std::max<uint64_t>(len, 1)));
    if (len) HIPCHK(hipMemcpy(e->d_stdin, data, len, hipMemcpyHostToDevice));
    return FI_OK;
}

fi_status fi_set_clock(fi_engine *e, uint64_t period_ticks, uint64_t random_seed) {
    if (!e || !period_ticks) return FI_E_ARG;
    if (e->have_golden) return fail(e, FI_E_STATE, "fi_set_clock: set before fi_golden_run (the golden run sees it)");
    HIPCHK(hipSetDevice(e->dev));
    e->clk_period = period_ticks;
    e->rnd_seed = random_seed;
    return upload_rnd(e);
}

fi_status fi_set_bits(fi_engine *e, uint64_t bits_mask) {
    if (!e) return FI_E_ARG;
    if (!e->structures) return fail(e, FI_E_STATE, "fi_set_campaign first");
    const uint64_t valid = e->burst == 1 ? ~0ULL : ((2ULL << (64 - e->burst)) - 1);
    if (!(bits_mask & valid)) return fail(e, FI_E_ARG, "no eligible bit position for a %u-bit burst", e->burst);
    e->bits = bits_mask;
    return FI_OK;
}

fi_status fi_set_protect(fi_engine *e, uint64_t protect_mask) {
    if (!e) return FI_E_ARG;
    e->protect = protect_mask;
    return FI_OK;
}

fi_status fi_set_protect_opclasses(fi_engine *e, uint64_t opclass_mask) {
    if (!e) return FI_E_ARG;
    e->protect_opc = opclass_mask;
    return FI_OK;
}

fi_status fi_set_issue_model(fi_engine *e, const fi_issue_params *p) {
    if (!e) return FI_E_ARG;
    if (!p) {
        e->issue_on = false;
        return FI_OK;
    }
    if (!e->have_golden) return fail(e, FI_E_STATE, "fi_set_issue_model: no golden run");
    const fi_issue_params keep = e->issue_p;
    e->issue_p = *p;
    const fi_status st = compute_shadow(e);
    if (st) { e->issue_p = keep; return st; }
    e->issue_on = true;
    return FI_OK;
}

fi_status fi_shadow_map(fi_engine *e, uint8_t *shadow, uint64_t cap, uint64_t *n, fi_issue_stats *stats) {
    if (!e) return FI_E_ARG;
    if (!e->issue_on) return fail(e, FI_E_STATE, "fi_shadow_map: the issue model is off");
    if (shadow && cap) memcpy(shadow, e->shadow.data(), std::min<uint64_t>(cap, e->shadow.size()));
    if (n) *n = e->shadow.size();
    if (stats) *stats = e->issue_stats;
    return FI_OK;
}

static SampleCtx sample_ctx(fi_engine *e, uint64_t first) {
    SampleCtx s{};
    s.seed = e->seed;
    s.structures = e->structures;
    s.bits = e->bits & (e->burst == 1 ? ~0ULL : ((2ULL << (64 - e->burst)) - 1));
    if (e->mem_pages.empty()) s.structures &= ~(1ULL << FI_T_MEM);
    s.golden_ninst = e->golden.ninst;
    s.first = first;
    s.burst = e->burst;
    s.n_struct = (uint32_t)__builtin_popcountll(s.structures);
    s.mem_pages = e->d_mem_pages;
    s.n_mem_pages = e->mem_pages.size();
    return s;
}

fi_status fi_sample_sites(fi_engine *e, uint64_t first, uint64_t n, fi_site *out) {
    if (!e || !out) return FI_E_ARG;
    if (!e->have_golden) return fail(e, FI_E_STATE, "golden run required before sampling");
    if (!e->structures) return fail(e, FI_E_STATE, "fi_set_campaign first");
    HIPCHK(hipSetDevice(e->dev));
    const uint64_t chunk = e->cfg.max_trials_per_launch;
    fi_status st = ensure_work(e, std::min<uint64_t>(std::max<uint64_t>(n, 1), chunk));
    if (st) return st;
    for (uint64_t done = 0; done < n;) {
        const uint64_t k = std::min<uint64_t>(n - done, e->cap);
        HIPCHK(launch_sample(sample_ctx(e, first + done), k, e->d_sites, e->d_keys, e->d_perm, e->stream));
        HIPCHK(hipMemcpyAsync(out + done, e->d_sites, k * sizeof(fi_site), hipMemcpyDeviceToHost, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        done += k;
    }
    return FI_OK;
}

// The trial kernel: the load-time build with translated blocks when there is
// one, else the static (interpreter-only) kernel.
// solo: the one-trial-per-wave build, one workgroup (kSoloLanes identical lanes) per slot.
static hipError_t launch_trial_kernel(fi_engine *e, DevCtx &c, hipStream_t st, bool solo) {
    void *args[] = {&c};
    if (solo) {
        if (!e->tx_fn_solo) return launch_trials_solo(c, st);
        return hipModuleLaunchKernel(e->tx_fn_solo, (unsigned)c.n, 1, 1, kSoloLanes, 1, 1, 0, st, args, nullptr);
    }
    if (!e->tx_fn) return launch_trials(c, st);
    const uint32_t gl = (c.resume && c.resume_waves) ? 1u : c.lanes;   // grid for the fewest lanes per wave
    return hipModuleLaunchKernel(e->tx_fn, (unsigned)((c.n + gl - 1) / gl), 1, 1, 64, 1, 1, 0, st, args,
                                 nullptr);
}

// The event pair of the next trial-kernel dispatch (kind: 0 the 64-lane
// kernel, 1 solo, 2 solo-odd; fi_debug_dispatch_ms).
static constexpr size_t kTimerSlots = 4096;   // dispatch timers kept between fi_kernel_timer_reset calls (a ring)
static std::pair<hipEvent_t, hipEvent_t> &timer_slot(fi_engine *e, uint32_t kind) {
    if (e->tused == kTimerSlots) e->tused = 0;
    if (e->tused == e->tpool.size()) {
        hipEvent_t a = nullptr, b = nullptr;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        e->tpool.emplace_back(a, b);
        e->tkind.push_back(0);
    }
    e->tkind[e->tused] = kind;
    return e->tpool[e->tused++];
}

// One pass over sites[0..k) (keys/perm set) with P private pages per slot:
// forwarding, sort by inject time, the epochs.  Outcomes to d_out.
static fi_status run_pass(fi_engine *e, fi_site *sites, uint64_t k, fi_outcome *d_out, uint32_t P, hipStream_t st) {
    int end_bit = 64 - __builtin_clzll(std::max<uint64_t>(e->golden.ninst, 1));
    // (a dead site ends at injection: an early exit, so not with FI_CFG_NO_EARLY_EXIT)
    const bool fwd = e->fw_ok && !(e->cfg.flags & (FI_CFG_NO_FORWARD | FI_CFG_NO_EARLY_EXIT));
    if (fwd) {
        FwdCtx fc{};
        fc.reg_off = e->d_fw_off; fc.reg_ev = e->d_fw_ev;
        // memory sites only when the golden run's mappings are static (no VM
        // syscalls: golden_fp covers them) and its access index is complete
        const bool memf = e->mem_live && !e->golden_fp && e->snaps.size() > 1;
        fc.mw_n = memf ? e->mw_n : 0;
        fc.mw_addr = e->d_mw_addr; fc.mw_off = e->d_mw_off; fc.mw_ev = e->d_mw_ev;
        fc.snaps = e->d_snaps; fc.snap_tab = e->d_tab; fc.n_snap = (uint32_t)e->snaps.size();
        fc.snap_interval = e->snap_I; fc.text_lo = e->text_lo; fc.text_hi = e->text_hi;
        HIPCHK(launch_forward(sites, k, fc, e->d_keys, e->d_eff, st));
    }
    HIPCHK(sort_pairs(e->d_tmp, e->tmp_bytes, e->d_keys, e->d_keys2, e->d_perm, e->d_perm2, k, end_bit, st));
    DevCtx c = base_ctx(e);
    c.sites = sites;
    c.perm = e->d_perm2;
    c.eff = fwd ? e->d_eff : nullptr;
    c.out = d_out;
    c.n = k;
    c.n_slots = (uint32_t)k;
    c.save = e->d_save;
    c.priv_pages = P;
    if (P != e->cfg.private_pages) c.ov_blocks = 0;   // the second pass has its own P' (chunk_end)
    if (c.ov_blocks) HIPCHK(hipMemsetAsync(e->d_ov_next, 0, 4, st));
    HIPCHK(hipMemsetAsync(e->d_cnt, 0, 16 * 4, st));
    HIPCHK(hipMemsetAsync(e->d_wave_dbg, 0, k * 10 * sizeof(uint64_t), st));
    const bool pack = (e->cfg.flags & FI_CFG_PACK_RUNS) != 0;
    int n_cu = 0;
    HIPCHK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, e->dev));
    const uint32_t spread = (e->cfg.flags & FI_CFG_FIXED_RESUME) ? 0u : (uint32_t)std::max(1, n_cu) * 4u;   // SIMDs
    if (pack) HIPCHK(hipMemsetAsync(e->d_nwaves, 0, 16 * 4, st));
    // epochs: each wave runs a bounded number of loop
    // iterations, then its live lanes are suspended, sorted by pc and resumed
    // densely packed; the last epoch runs to completion.  All asynchronous:
    // resume grids are sized for every slot and surplus waves exit at once.
    std::vector<uint32_t> budgets;
    if (e->cfg.flags & FI_CFG_NO_EPOCHS) {
        budgets = {0};
    } else {
        const uint32_t b = e->cfg.epoch_iters ? e->cfg.epoch_iters : 384;
        // default: one 64-lane epoch, then every survivor to completion on the
        // solo kernel (profiles/r02c epoch_sweep: 2 epochs beat 3 and 4; with
        // first-access forwarding a 1024-iteration first epoch beat 4096:
        // crc32 12.7M vs 9.8M, qsort +3 %, intmix even, profiles/r02l_ab.txt;
        // with the round-5 solo kernel 384 beats 1024: crc32 4.77 vs 4.96 ms,
        // qsort 30.9 vs 32.2 ms, intmix 257 vs 253 ms, profiles/ep_sweep_r05*.jsonl)
        const uint32_t n_ep = e->cfg.epochs ? std::max(2u, std::min(e->cfg.epochs, 14u)) : 2u;
        for (uint32_t i = 0; i + 1 < n_ep; i++) budgets.push_back(b << (2 * std::min(i, 2u)));
        budgets.push_back(0);
    }
    // the odd-pc survivors of a resumed solo epoch run on the solo-odd kernel
    // (at most kOddGrid of them; the rest stay with the solo kernel), on its
    // own stream beside the solo kernel
    constexpr uint32_t kOddGrid = 2048;
    const bool odd_on = e->tx_fn_odd && e->tx_fn_solo && !(e->cfg.flags & FI_CFG_NO_ODD_KERNEL);
    if (odd_on) HIPCHK(hipMemsetAsync(e->d_split, 0, 64 * 4, st));
    for (size_t ep = 0; ep < budgets.size(); ep++) {
        const bool solo = (e->cfg.flags & FI_CFG_SOLO_ALL) || (ep > 0 && !(e->cfg.flags & FI_CFG_NO_SOLO));
        const bool odd = odd_on && solo && ep > 0 && ep < 16;
        c.wave_budget = budgets[ep];
        c.surv = e->d_surv[ep & 1];
        c.surv_n = e->d_cnt + ep;
        c.lanes = ep == 0 ? e->cfg.lanes_per_wave : e->cfg.resume_lanes;
        c.wrange = nullptr;
        c.n_waves = nullptr;
        c.resume_waves = ep == 0 ? 0u : spread;
        if (ep == 0) {
            c.resume = nullptr;
            c.resume_n = nullptr;
        } else {
            // survivors not yet injected form a tier right after the first
            // (fi_surv_keys_kernel; profiles/r04au: intmix -3 %, qsort -3 %
            // per step against the two-tier order)
            const uint32_t skey = (solo && !pack) ? 3u : 0u;
            // solo keys: tier above numInst, which stays below the hang cap -- a
            // key of nb + 2 bits (+ 1 for the odd-pc flag) sorts in fewer passes
            const uint32_t nb = 64u - (uint32_t)__builtin_clzll(std::max<uint64_t>(c.hang_cap, 1));
            HIPCHK(launch_surv_keys(e->d_save, e->d_surv[(ep - 1) & 1], e->d_cnt + ep - 1, k, c.text_lo, e->d_skeys,
                                    e->d_svals, odd ? e->d_split + 4 * ep : nullptr, skey, e->golden.ninst, nb,
                                    e->d_loops, e->n_loops, c.hang_cap, st));
            HIPCHK(sort_pairs(e->d_tmp, e->tmp_bytes, e->d_skeys, e->d_skeys2, e->d_svals, e->d_svals2, k,
                              skey ? (int)std::min(64u, nb + 3u) : 64, st));
            c.resume = e->d_svals2;
            c.resume_n = e->d_cnt + ep - 1;
            if (odd) {   // odd survivors sort last: the solo kernel takes [0, split), the solo-odd kernel the rest
                const uint32_t grid = (uint32_t)std::min<uint64_t>(k, kOddGrid);
                HIPCHK(launch_odd_split(c.resume_n, e->d_split + 4 * ep, e->d_split + 4 * ep + 1, grid, st));
                DevCtx co = c;
                co.lanes = 1; co.resume_waves = 0; co.wrange = nullptr; co.n_waves = nullptr;
                co.resume_lo = e->d_split + 4 * ep + 1;
                c.resume_n = e->d_split + 4 * ep + 1;
                HIPCHK(hipEventRecord(e->ev_fork, st));
                HIPCHK(hipStreamWaitEvent(e->stream_odd, e->ev_fork, 0));
                auto &tq = timer_slot(e, 2);
                co.span = e->d_span ? e->d_span + 2 * (e->tused - 1) : nullptr;
                HIPCHK(hipEventRecord(tq.first, e->stream_odd));
                void *args[] = {&co};
                HIPCHK(hipModuleLaunchKernel(e->tx_fn_odd, grid, 1, 1, kSoloLanes, 1, 1, 0, e->stream_odd, args, nullptr));
                HIPCHK(hipEventRecord(tq.second, e->stream_odd));
                HIPCHK(hipEventRecord(e->ev_join, e->stream_odd));
            }
            if (pack && !solo) {
                // one wave per same-pc run of survivors (<= 64 lanes); the grid
                // covers the worst case (every survivor alone), surplus waves exit
                HIPCHK(launch_pack_runs(e->d_skeys2, c.resume_n, k, e->d_wrange + 0, e->d_nwaves + ep, st));
                c.wrange = e->d_wrange;
                c.n_waves = e->d_nwaves + ep;
                c.lanes = 1;
                c.resume_waves = 0;
            }
        }
        // every dispatch of the trial kernel is bracketed by its own event
        // pair on the launch stream (the bench's per-dispatch kernel time)
        auto &tp = timer_slot(e, solo ? 1 : 0);
        c.span = e->d_span ? e->d_span + 2 * (e->tused - 1) : nullptr;
        HIPCHK(hipEventRecord(tp.first, st));
        if (solo) { c.lanes = 1; c.resume_waves = 0; c.wrange = nullptr; c.n_waves = nullptr; }
        HIPCHK(launch_trial_kernel(e, c, st, solo));
        HIPCHK(hipEventRecord(tp.second, st));
        if (odd) HIPCHK(hipStreamWaitEvent(st, e->ev_join, 0));
    }
    return FI_OK;
}

// Chunks are pipelined on the launch stream with no host wait between them
// (DESIGN.md §4e): chunk i runs its pass and lists its resource escapes
// (FI_ESC_RESOURCE: an engine capacity limit -- the overflow pool ran dry --
// not gem5 behaviour) and copies their count to pinned memory; the host then
// enqueues chunk i+1 and only after that reads chunk i's count, while the GPU
// is busy with chunk i+1.  Chunk i's second pass (redo_pages-fold pages, in
// batches that reuse the same frames: batch x P' <= k x P), its histogram and
// its host copy follow chunk i+1 on the stream; their outcomes replace the
// escapes.  Sites and outcome buffers alternate between the two chunks in
// flight.  FI_CFG_NO_REDO keeps the escapes.
struct Chunk {
    uint64_t k = 0;
    fi_site *sites = nullptr;
    fi_outcome *out = nullptr;
    fi_outcome *host_out = nullptr;   // run_common: where the outcomes go on the host
    uint32_t slot = 0;                // redo list / count / event pair
};

static fi_status chunk_begin(fi_engine *e, const Chunk &ch, hipStream_t st) {
    fi_status s = run_pass(e, ch.sites, ch.k, ch.out, e->cfg.private_pages, st);
    if (s) return s;
    if (!(e->cfg.flags & FI_CFG_NO_REDO)) {
        uint32_t *cnt = e->d_redo_cnt + ch.slot;
        HIPCHK(hipMemsetAsync(cnt, 0, 4, st));
        HIPCHK(launch_redo_collect(ch.out, ch.k, e->d_redo_idx + ch.slot * e->cap, cnt, e->d_stats, st));
        HIPCHK(hipMemcpyAsync(e->h_redo_cnt + ch.slot, cnt, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipEventRecord(e->ev_cnt[ch.slot], st));
    }
    return FI_OK;
}

static fi_status chunk_end(fi_engine *e, const Chunk &ch, fi_histogram *d_hist, hipStream_t st) {
    if (!(e->cfg.flags & FI_CFG_NO_REDO)) {
        HIPCHK(hipEventSynchronize(e->ev_cnt[ch.slot]));   // (normally long done: a chunk later was enqueued first)
        const uint64_t nr = e->h_redo_cnt[ch.slot];
        const uint32_t *idx = e->d_redo_idx + ch.slot * e->cap;
        if (nr) {
            const uint64_t P = e->cfg.private_pages;
            const uint64_t pool = e->cap * P;   // page frames a pass has
            const uint64_t P2 = std::min<uint64_t>(pool, redo_pages(P));
            const uint64_t B = std::max<uint64_t>(1, pool / P2);
            for (uint64_t d = 0; d < nr; d += B) {
                const uint64_t b = std::min(B, nr - d);
                HIPCHK(launch_redo_gather(ch.sites, idx + d, b, e->d_redo_sites, e->d_keys, e->d_perm, st));
                fi_status s = run_pass(e, e->d_redo_sites, b, e->d_redo_out, (uint32_t)P2, st);
                if (s) return s;
                HIPCHK(launch_redo_scatter(idx + d, b, e->d_redo_out, ch.out, st));
            }
        }
    }
    HIPCHK(launch_hist(ch.sites, ch.out, ch.k, d_hist, nullptr, st));
    if (ch.host_out) {
        if (!e->h_stage[ch.slot]) HIPCHK(hipHostMalloc(&e->h_stage[ch.slot], e->cap * sizeof(fi_outcome)));
        HIPCHK(hipMemcpyAsync(e->h_stage[ch.slot], ch.out, ch.k * sizeof(fi_outcome), hipMemcpyDeviceToHost, st));
        HIPCHK(hipEventRecord(e->ev_stage[ch.slot], st));
    }
    return FI_OK;
}

// A chunk's staged outcomes to the caller's array, once their copy has landed.
static fi_status chunk_deliver(fi_engine *e, Chunk &ch) {
    if (!ch.host_out || !ch.k) return FI_OK;
    HIPCHK(hipEventSynchronize(e->ev_stage[ch.slot]));
    memcpy(ch.host_out, e->h_stage[ch.slot], ch.k * sizeof(fi_outcome));
    ch.k = 0;
    return FI_OK;
}

static void hist_add(fi_histogram *dst, const fi_histogram *src) {
    const uint64_t *s = (const uint64_t *)src;
    uint64_t *d = (uint64_t *)dst;
    for (size_t i = 0; i < sizeof(fi_histogram) / 8; i++) d[i] += s[i];
}

// Trials [first, first + n) (sampled on the device) or the given sites, in
// chunks of at most e->cap; outcomes to out_dev (device, n entries) or
// out_host (through the alternating device buffers), histogram added to
// d_hist.  The event pair ev0 / ev1 spans the whole call.
static fi_status run_chunks(fi_engine *e, uint64_t first, const fi_site *sites, uint64_t n, fi_outcome *out_dev,
                            fi_outcome *out_host, fi_histogram *d_hist, hipStream_t st) {
    HIPCHK(hipMemsetAsync(e->d_stats, 0, kNStats * sizeof(unsigned long long), st));
    HIPCHK(hipEventRecord(e->ev0, st));
    Chunk prev, staged[2];   // (staged: chunks whose outcomes still sit in h_stage)
    bool have_prev = false;
    uint32_t i = 0;
    for (uint64_t done = 0; done < n; i++) {
        jit_install(e, st, false);   // the translated kernels, once their build has landed
        Chunk ch;
        ch.k = std::min<uint64_t>({n - done, e->cap, e->jit ? kJitWindowChunk : e->cap});
        ch.slot = i & 1;
        ch.sites = ch.slot ? e->d_sites_alt : e->d_sites;
        ch.out = out_dev ? out_dev + done : ch.slot ? e->d_out_alt : e->d_out;
        ch.host_out = out_host ? out_host + done : nullptr;
        if (sites) {
            HIPCHK(hipMemcpyAsync(ch.sites, sites + done, ch.k * sizeof(fi_site), hipMemcpyHostToDevice, st));
            HIPCHK(launch_keys(ch.sites, ch.k, e->d_keys, e->d_perm, st));
        } else {
            HIPCHK(launch_sample(sample_ctx(e, first + done), ch.k, ch.sites, e->d_keys, e->d_perm, st));
        }
        fi_status s = chunk_begin(e, ch, st);
        if (s) return s;
        if (have_prev) {
            if ((s = chunk_deliver(e, staged[prev.slot]))) return s;   // (two chunks ago: long landed)
            if ((s = chunk_end(e, prev, d_hist, st))) return s;
            staged[prev.slot] = prev;
        }
        prev = ch;
        have_prev = true;
        done += ch.k;
    }
    if (have_prev) {
        fi_status s = chunk_deliver(e, staged[prev.slot]);
        if (!s) s = chunk_end(e, prev, d_hist, st);
        if (s) return s;
        staged[prev.slot] = prev;
    }
    HIPCHK(hipEventRecord(e->ev1, st));
    HIPCHK(launch_hist_stats(e->d_stats, d_hist, st));
    for (auto &c : staged) {
        fi_status s = chunk_deliver(e, c);
        if (s) return s;
    }
    return FI_OK;
}

static fi_status run_common(fi_engine *e, uint64_t first, const fi_site *sites, uint64_t n, fi_outcome *out,
                            fi_histogram *hist) {
    if (!e) return FI_E_ARG;
    if (!e->have_golden) return fail(e, FI_E_STATE, "golden run required");
    if (!sites && !e->structures) return fail(e, FI_E_STATE, "fi_set_campaign first");
    HIPCHK(hipSetDevice(e->dev));
    const uint64_t chunk = e->cfg.max_trials_per_launch;
    fi_status s = ensure_work(e, std::min<uint64_t>(std::max<uint64_t>(n, 1), chunk));
    if (s) return s;
    HIPCHK(hipMemsetAsync(e->d_hist, 0, sizeof(fi_histogram), e->stream));
    s = run_chunks(e, first, sites, n, nullptr, out, e->d_hist, e->stream);
    if (s) return s;
    HIPCHK(hipStreamSynchronize(e->stream));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e->ev0, e->ev1));
    e->last_ms = ms;
    if (hist) {
        fi_histogram h;
        HIPCHK(hipMemcpy(&h, e->d_hist, sizeof h, hipMemcpyDeviceToHost));
        hist_add(hist, &h);
    }
    return FI_OK;
}

fi_status fi_wait_translation(fi_engine *e, fi_golden_info *out) {
    if (!e) return FI_E_ARG;
    if (!e->have_golden) return fail(e, FI_E_STATE, "no golden run");
    HIPCHK(hipSetDevice(e->dev));
    jit_install(e, e->stream, true);
    HIPCHK(hipStreamSynchronize(e->stream));
    if (out) *out = e->golden;
    return FI_OK;
}

fi_status fi_run_trials(fi_engine *e, uint64_t first, uint64_t n, fi_outcome *out, fi_histogram *hist) {
    return run_common(e, first, nullptr, n, out, hist);
}

fi_status fi_run_sites(fi_engine *e, const fi_site *sites, uint64_t n, fi_outcome *out, fi_histogram *hist) {
    if (!sites && n) return FI_E_ARG;
    return run_common(e, 0, sites, n, out, hist);
}

// ---------------------------------------------------- tick-domain injection
fi_status fi_set_cpu_model(fi_engine *e, int model, const fi_timing_params *p) {
    if (!e) return FI_E_ARG;
    if (model != FI_CPU_ATOMIC && model != FI_CPU_TIMING) return fail(e, FI_E_ARG, "unknown CPU model %d", model);
    if (e->have_golden) return fail(e, FI_E_STATE, "fi_set_cpu_model: set before fi_golden_run");
    e->cpu_model = model;
    if (p) e->tparams = *p; else fi_timing_default_params(&e->tparams);
    return FI_OK;
}

fi_status fi_tick_golden(fi_engine *e, fi_tick_info *out) {
    if (!e || !out) return FI_E_ARG;
    *out = fi_tick_info{};
    snprintf(out->status, sizeof out->status, "%s", e->t_status.c_str());
    out->attempts = e->t_ops.size();
    out->golden_ticks = e->t_stats.ticks;
    out->stats = e->t_stats;
    return FI_OK;
}

fi_status fi_tick_trace(fi_engine *e, fi_timing_op *ops, fi_timing_ticks *ticks, uint64_t cap, uint64_t *n) {
    if (!e) return FI_E_ARG;
    if (!e->t_status.empty()) return fail(e, FI_E_STATE, "tick model: %s", e->t_status.c_str());
    const uint64_t k = std::min<uint64_t>(cap, e->t_ops.size());
    if (ops && k) memcpy(ops, e->t_ops.data(), k * sizeof *ops);
    if (ticks && k) memcpy(ticks, e->t_ticks.data(), k * sizeof *ticks);
    if (n) *n = e->t_ops.size();
    return FI_OK;
}

static uint64_t splitmix_host(uint64_t &s) {   // the sampler's SplitMix64 (fi_kernels.hip)
    uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static uint64_t mulhi64(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a * b) >> 64); }

static fi_status tick_ready(fi_engine *e) {
    if (!e->have_golden) return fail(e, FI_E_STATE, "golden run required");
    if (!e->t_status.empty()) return fail(e, FI_E_STATE, "tick model: %s", e->t_status.c_str());
    return FI_OK;
}

fi_status fi_sample_tick_sites(fi_engine *e, uint64_t first, uint64_t n, fi_tick_site *out) {
    if (!e || (!out && n)) return FI_E_ARG;
    fi_status st = tick_ready(e);
    if (st) return st;
    if (!e->structures) return fail(e, FI_E_STATE, "fi_set_campaign first");
    if (e->structures & (1ULL << FI_T_MEM)) return fail(e, FI_E_ARG, "tick sites: memory words are not supported");
    const uint64_t structures = e->structures;
    const uint32_t nt = (uint32_t)__builtin_popcountll(structures), burst = e->burst;
    const uint64_t valid = burst == 1 ? ~0ULL : ((2ULL << (64 - burst)) - 1);
    for (uint64_t i = 0; i < n; i++) {   // fi_sample_kernel's draw with the golden run's ticks for numInst
        const uint64_t id = first + i;
        uint64_t s = e->seed ^ (id * 0xD6E8FEB86659FD93ULL);
        const uint64_t r0 = splitmix_host(s), r1 = splitmix_host(s), r2 = splitmix_host(s);
        fi_tick_site &o = out[i];
        o.tick = mulhi64(r0, e->t_stats.ticks);
        const uint64_t k = mulhi64(r1, nt);
        uint64_t m = structures;
        for (uint64_t j = 0; j < k; j++) m &= m - 1;
        o.target = (uint32_t)__builtin_ctzll(m);
        uint64_t b;
        if ((e->bits & valid) == valid) {
            b = mulhi64(r2, 65 - burst);
        } else {
            uint64_t mm = e->bits & valid;
            const uint64_t kk = mulhi64(r2, (uint64_t)__builtin_popcountll(mm));
            for (uint64_t j = 0; j < kk; j++) mm &= mm - 1;
            b = (uint64_t)__builtin_ctzll(mm);
        }
        o.mask = (burst == 64 ? ~0ULL : ((1ULL << burst) - 1)) << b;
        o.trial = (uint32_t)id;
    }
    return FI_OK;
}

fi_status fi_map_tick_sites(fi_engine *e, const fi_tick_site *ts, uint64_t n, fi_site *sites, uint8_t *disp,
                            fi_outcome *host_out) {
    if (!e || (n && (!ts || !sites || !disp))) return FI_E_ARG;
    fi_status st = tick_ready(e);
    if (st) return st;
    for (uint64_t i = 0; i < n; i++) {
        const fi_tick_site &t = ts[i];
        const bool target_ok = (t.target >= 1 && t.target <= FI_T_PC) || t.target == FI_T_RESULT;
        if (!t.mask || !target_ok || t.tick >= e->t_stats.ticks)
            return fail(e, FI_E_ARG, "tick site %llu: target %u, tick %llu (golden run %llu ticks)",
                        (unsigned long long)i, t.target, (unsigned long long)t.tick,
                        (unsigned long long)e->t_stats.ticks);
        const TickMapped m = map_tick_site(e->t_att, e->t_ticks, e->golden.ninst, t.tick, t.target, t.mask, t.trial);
        disp[i] = (uint8_t)m.disp;
        sites[i] = m.site;
        if (host_out) {
            fi_outcome o{};
            if (m.disp == 1) {   // the golden run itself
                o.cls = FI_MASKED; o.sub = (uint8_t)e->gsub; o.exit_code = (uint8_t)e->golden.exit_code;
                o.flags = 1; o.detail = e->gdetail; o.ninst = e->golden.ninst;
            } else if (m.disp == 2) {
                const TickAttempt &A = e->t_att[m.attempt];
                o.cls = FI_ESCAPE; o.sub = FI_ESC_TIMING; o.exit_code = (uint8_t)m.reason;
                o.flags = 1; o.detail = (uint32_t)A.pc; o.ninst = A.n;
            }
            host_out[i] = o;
        }
    }
    return FI_OK;
}

fi_status fi_run_tick_sites(fi_engine *e, const fi_tick_site *ts, uint64_t n, fi_outcome *out, fi_histogram *hist) {
    if (!e || (n && !ts)) return FI_E_ARG;
    fi_status st = tick_ready(e);
    if (st) return st;
    if (e->protect || e->protect_opc)
        return fail(e, FI_E_ARG, "tick sites: selective replication (fi_set_protect*) is not supported");
    std::vector<fi_site> sites(n);
    std::vector<uint8_t> disp(n);
    std::vector<fi_outcome> res(n);
    st = fi_map_tick_sites(e, ts, n, sites.data(), disp.data(), res.data());
    if (st) return st;
    std::vector<fi_site> run;
    std::vector<uint64_t> idx;
    for (uint64_t i = 0; i < n; i++)
        if (disp[i] == 0) { run.push_back(sites[i]); idx.push_back(i); }
    fi_histogram dh{};
    if (!run.empty()) {
        std::vector<fi_outcome> ro(run.size());
        e->clk_esc = 1;   // this engine's clock is AtomicSimpleCPU's: a curTick read escapes
        st = run_common(e, 0, run.data(), run.size(), ro.data(), &dh);
        e->clk_esc = 0;
        if (st) return st;
        for (size_t q = 0; q < idx.size(); q++) res[idx[q]] = ro[q];
    }
    if (out) memcpy(out, res.data(), n * sizeof *out);
    if (hist) {   // by the tick site's own structure and bit (fi_hist_kernel's layout)
        for (uint64_t i = 0; i < n; i++) {
            const fi_outcome &o = res[i];
            const uint32_t cls = o.cls < FI_N_CLASS ? o.cls : FI_ESCAPE;
            hist->counts[ts[i].target][__builtin_ctzll(ts[i].mask)][cls]++;
            if (cls == FI_CRASH) hist->crash_sub[o.sub & 15]++;
            if (cls == FI_ESCAPE) hist->escape_sub[o.sub & 7]++;
            hist->trials++;
            hist->guest_insts += o.ninst;
        }
        hist->fetch_bytes += dh.fetch_bytes; hist->data_bytes += dh.data_bytes;
        hist->cow_pages += dh.cow_pages; hist->device_insts += dh.device_insts;
    }
    return FI_OK;
}

fi_status fi_run_tick_trials(fi_engine *e, uint64_t first, uint64_t n, fi_outcome *out, fi_histogram *hist) {
    if (!e) return FI_E_ARG;
    std::vector<fi_tick_site> ts(n);
    fi_status st = fi_sample_tick_sites(e, first, n, ts.data());
    if (st) return st;
    return fi_run_tick_sites(e, ts.data(), n, out, hist);
}

fi_status fi_run_trials_device(fi_engine *e, uint64_t first, uint64_t n, void *d_out, void *d_hist, void *stream) {
    if (!e || !d_out || !d_hist) return FI_E_ARG;
    if (!e->have_golden) return fail(e, FI_E_STATE, "golden run required");
    if (!e->structures) return fail(e, FI_E_STATE, "fi_set_campaign first");
    HIPCHK(hipSetDevice(e->dev));
    hipStream_t st = stream ? (hipStream_t)stream : e->stream;
    const uint64_t chunk = e->cfg.max_trials_per_launch;
    fi_status s = ensure_work(e, std::min<uint64_t>(std::max<uint64_t>(n, 1), chunk));
    if (s) return s;
    return run_chunks(e, first, nullptr, n, (fi_outcome *)d_out, nullptr, (fi_histogram *)d_hist, st);
}

fi_status fi_sync(fi_engine *e) {
    if (!e) return FI_E_ARG;
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipEventSynchronize(e->ev1));
    float ms = 0;
    if (hipEventElapsedTime(&ms, e->ev0, e->ev1) == hipSuccess) e->last_ms = ms;
    return FI_OK;
}

double fi_last_kernel_ms(fi_engine *e) { return e ? e->last_ms : 0.0; }

const char *fi_translate_status(fi_engine *e) { return e ? e->tx_status.c_str() : "no engine"; }

// hipRTC build of the trial kernel with `body` as translated blocks, no
// device needed (tests; inspecting generated code offline).
fi_status fi_debug_jit_compile(const char *body, const char *arch, void *code, uint64_t cap, uint64_t *len,
                               char *err, uint64_t err_cap) {
    std::vector<char> co;
    bool cached = false;
    const std::string msg = jit_compile(body ? body : "", arch ? arch : "gfx950", co, cached, 0, true);
    if (err && err_cap) {
        const uint64_t n = std::min<uint64_t>(err_cap - 1, msg.size());
        memcpy(err, msg.data(), n);
        err[n] = 0;
    }
    if (!msg.empty()) return FI_E_HIP;
    if (code && cap) memcpy(code, co.data(), std::min<uint64_t>(cap, co.size()));
    if (len) *len = co.size();
    return FI_OK;
}

// One part of the load-time build as an engine runs it (part 1..3, the disk
// cache on or off, FI_CFG_JIT_NO_CACHE), no device needed: *cached = 1 when
// the code object came from the cache.  Tests of the per-node build lock.
fi_status fi_debug_jit_build(const char *body, const char *arch, int part, int use_cache, uint64_t *len,
                             int *cached, char *err, uint64_t err_cap) {
    std::vector<char> co;
    bool c = false;
    const std::string msg = jit_compile(body ? body : "", arch ? arch : "gfx950", co, c, part, use_cache != 0);
    if (err && err_cap) {
        const uint64_t n = std::min<uint64_t>(err_cap - 1, msg.size());
        memcpy(err, msg.data(), n);
        err[n] = 0;
    }
    if (len) *len = co.size();
    if (cached) *cached = c ? 1 : 0;
    return msg.empty() ? FI_OK : FI_E_HIP;
}

fi_status fi_debug_waves(fi_engine *e, uint64_t *out, uint64_t n_waves) {
    if (!e || !out) return FI_E_ARG;
    if (n_waves > e->cap) return fail(e, FI_E_ARG, "more waves than the work buffers hold");
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipMemcpy(out, e->d_wave_dbg, n_waves * 10 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return FI_OK;
}

fi_status fi_debug_epochs(fi_engine *e, uint32_t *out16) {
    if (!e || !out16 || !e->d_cnt) return FI_E_ARG;
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipMemcpy(out16, e->d_cnt, 16 * 4, hipMemcpyDeviceToHost));
    return FI_OK;
}

fi_status fi_debug_golden_trace(fi_engine *e, void *pre_out, uint64_t pre_cap, uint64_t *n_pre, uint32_t *trace_out,
                                uint64_t trace_cap, uint64_t *n_trace, uint64_t *text_lo) {
    if (!e) return FI_E_ARG;
    if (pre_out) memcpy(pre_out, e->g_pre.data(), std::min<uint64_t>(pre_cap, e->g_pre.size()) * sizeof(PreInst));
    if (trace_out) memcpy(trace_out, e->g_trace.data(), std::min<uint64_t>(trace_cap, e->g_trace.size()) * 4);
    if (n_pre) *n_pre = e->g_pre.size();
    if (n_trace) *n_trace = e->g_trace.size();
    if (text_lo) *text_lo = e->text_lo;
    return FI_OK;
}

fi_status fi_debug_loop_est(const void *pre, uint64_t n_pre, uint64_t text_lo, const uint32_t *trace,
                            uint64_t n_trace, void *out, uint64_t cap, uint64_t *n) {
    if (!pre || !trace) return FI_E_ARG;
    std::vector<PreInst> p((const PreInst *)pre, (const PreInst *)pre + n_pre);
    std::vector<uint32_t> t(trace, trace + n_trace), leaders;
    std::vector<LoopEst> loops;
    uint32_t n_tx = 0;
    (void)translate_blocks(p, text_lo, t, {}, leaders, n_tx, true, &loops);
    static_assert(sizeof(LoopEst) == 16, "LoopEst is 16 bytes (fi_debug.h)");
    if (out) memcpy(out, loops.data(), std::min<uint64_t>(cap, loops.size()) * sizeof(LoopEst));
    if (n) *n = loops.size();
    return FI_OK;
}

fi_status fi_debug_translate(const void *pre, uint64_t n_pre, uint64_t text_lo, const uint32_t *trace,
                             uint64_t n_trace, char *out, uint64_t cap, uint64_t *len) {
    if (!pre || !trace) return FI_E_ARG;
    std::vector<PreInst> p((const PreInst *)pre, (const PreInst *)pre + n_pre);
    std::vector<uint32_t> t(trace, trace + n_trace);
    std::vector<uint32_t> leaders;
    uint32_t n_tx = 0;
    const std::string body = translate_blocks(p, text_lo, t, {}, leaders, n_tx, true);
    if (out && cap) {
        const uint64_t n = std::min<uint64_t>(cap - 1, body.size());
        memcpy(out, body.data(), n);
        out[n] = 0;
    }
    if (len) *len = body.size();
    return FI_OK;
}

fi_status fi_debug_translation(fi_engine *e, char *buf, uint64_t cap, uint64_t *len) {
    if (!e) return FI_E_ARG;
    if (buf && cap) {
        const uint64_t n = std::min<uint64_t>(cap - 1, e->tx_body.size());
        memcpy(buf, e->tx_body.data(), n);
        buf[n] = 0;
    }
    if (len) *len = e->tx_body.size();
    return FI_OK;
}

fi_status fi_debug_stats(fi_engine *e, uint64_t *out64) {
    if (!e || !out64) return FI_E_ARG;
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipMemcpy(out64, e->d_stats, kNStats * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return FI_OK;
}

fi_status fi_get_config(fi_engine *e, fi_config *out) {
    if (!e || !out) return FI_E_ARG;
    *out = e->cfg;
    return FI_OK;
}

fi_status fi_kernel_timer_reset(fi_engine *e) {
    if (!e) return FI_E_ARG;
    e->tused = 0;
    if (!e->d_span) {
        HIPCHK(hipSetDevice(e->dev));
        HIPCHK(hipMalloc(&e->d_span, kTimerSlots * 2 * sizeof(unsigned long long)));
    }
    // every slot's min starts at ~0, its max at 0 (layout: slot i at [2i, 2i + 1])
    HIPCHK(hipMemsetAsync(e->d_span, 0, kTimerSlots * 2 * sizeof(unsigned long long), e->stream));
    HIPCHK(launch_span_init(e->d_span, kTimerSlots, e->stream));
    return FI_OK;
}

fi_status fi_kernel_timer_read(fi_engine *e, double *total_ms, uint32_t *launches) {
    if (!e) return FI_E_ARG;
    double t = 0;
    for (size_t i = 0; i < e->tused; i++) {
        HIPCHK(hipEventSynchronize(e->tpool[i].second));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, e->tpool[i].first, e->tpool[i].second));
        t += ms;
    }
    if (total_ms) *total_ms = t;
    if (launches) *launches = (uint32_t)e->tused;
    return FI_OK;
}

// ------------------------------------------------------------------ debug hooks (tests)
fi_status fi_debug_dispatch_ms(fi_engine *e, float *ms, uint32_t cap, uint32_t *n) {
    if (!e || (!ms && cap)) return FI_E_ARG;
    for (size_t i = 0; i < e->tused && i < cap; i++) {
        HIPCHK(hipEventSynchronize(e->tpool[i].second));
        HIPCHK(hipEventElapsedTime(&ms[i], e->tpool[i].first, e->tpool[i].second));
    }
    if (n) *n = (uint32_t)e->tused;
    return FI_OK;
}

fi_status fi_debug_dispatch_span_ms(fi_engine *e, float *ms, uint32_t cap, uint32_t *n) {
    if (!e || (!ms && cap)) return FI_E_ARG;
    const size_t k = std::min<size_t>(e->tused, cap);
    if (k) {
        if (!e->d_span) return fail(e, FI_E_STATE, "fi_debug_dispatch_span_ms: fi_kernel_timer_reset first");
        HIPCHK(hipStreamSynchronize(e->stream));
        HIPCHK(hipStreamSynchronize(e->stream_odd));
        std::vector<unsigned long long> h(2 * k);
        HIPCHK(hipMemcpy(h.data(), e->d_span, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < k; i++)   // (s_memrealtime runs at 100 MHz; no trial ran: 0)
            ms[i] = h[2 * i + 1] > h[2 * i] ? (float)((h[2 * i + 1] - h[2 * i]) * 1e-5) : 0.0f;
    }
    if (n) *n = (uint32_t)e->tused;
    return FI_OK;
}
fi_status fi_debug_dispatch_kinds(fi_engine *e, uint32_t *kinds, uint32_t cap, uint32_t *n) {
    if (!e || (!kinds && cap)) return FI_E_ARG;
    for (size_t i = 0; i < e->tused && i < cap; i++) kinds[i] = e->tkind[i];
    if (n) *n = (uint32_t)e->tused;
    return FI_OK;
}

fi_status fi_debug_decode(fi_engine *e, const uint32_t *raws, uint64_t n, void *out16) {
    if (!e || !raws || !out16) return FI_E_ARG;
    HIPCHK(hipSetDevice(e->dev));
    uint32_t *d_raw = nullptr;
    PreInst *d_o = nullptr;
    HIPCHK(hipMalloc(&d_raw, n * 4));
    HIPCHK(hipMalloc(&d_o, n * sizeof(PreInst)));
    HIPCHK(hipMemcpy(d_raw, raws, n * 4, hipMemcpyHostToDevice));
    HIPCHK(launch_debug_decode(d_raw, n, d_o, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipMemcpy(out16, d_o, n * sizeof(PreInst), hipMemcpyDeviceToHost));
    (void)hipFree(d_raw);
    (void)hipFree(d_o);
    return FI_OK;
}

fi_status fi_debug_loop_outcome(fi_engine *e, const fi_debug_loop *in, uint64_t n, fi_debug_loop_out *out) {
    if (!e || (n && (!in || !out))) return FI_E_ARG;
    if (e->snaps.empty()) return fail(e, FI_E_STATE, "fi_debug_loop_outcome: fi_golden_run first");
    if (!n) return FI_OK;
    HIPCHK(hipSetDevice(e->dev));
    fi_debug_loop *d_in = nullptr;
    fi_debug_loop_out *d_out = nullptr;
    HIPCHK(hipMalloc(&d_in, n * sizeof *in));
    HIPCHK(hipMalloc(&d_out, n * sizeof *out));
    HIPCHK(hipMemcpy(d_in, in, n * sizeof *in, hipMemcpyHostToDevice));
    DevCtx c = base_ctx(e);
    HIPCHK(launch_debug_loop(c, d_in, n, d_out, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipMemcpy(out, d_out, n * sizeof *out, hipMemcpyDeviceToHost));
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return FI_OK;
}

}  // extern "C"
