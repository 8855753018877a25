"""Host-side mirror of the gem5 `FaultCampaign` SimObject over the C ABI.

`FaultCampaign` keeps the parameter names and meaning of the SimObject
declared in src/gem5ext/FaultCampaign.py (a gem5 SimObject in the style of
src/cpu/o3/BaseO3CPU.py:64-72,226-227 of the reference) so a config script can
drive the engine with or without gem5 present.  Every call goes to
libshrewd_fi.so (HIP kernels); there is no CPU execution path -- when no
MI355X is visible the engine refuses to start (FI_E_NODEVICE).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Iterable, Sequence

import numpy as np

from . import build as _build

FI_OK, FI_E_ARG, FI_E_NODEVICE, FI_E_HIP, FI_E_ELF, FI_E_STATE, FI_E_GOLDEN = 0, -1, -2, -3, -4, -5, -6
CLASS_NAMES = ["masked", "sdc", "crash", "hang", "detected", "escape"]
CRASH_NAMES = {1: "panic_unknown_inst", 2: "panic_illegal_inst", 3: "panic_page_fault",
               4: "fatal_syscall_range", 5: "fatal_syscall_unimpl", 6: "fatal_proxy", 7: "abort_fd_assert",
               8: "sigtrap", 9: "fatal_stack_limit", 10: "panic_amo_line", 11: "abort_sc_line", 12: "panic_se_handler",
               13: "panic_m5op", 14: "abort_vset_sew"}
ESCAPE_NAMES = {1: "inst", 2: "syscall", 3: "csr", 4: "host", 5: "resource", 6: "undefined", 7: "timing"}
# FI_ESC_TIMING reasons (exit_code): tick sites that are not a numInst injection (include/fi_engine.h FI_TK_*)
TICK_ESCAPE_NAMES = {1: "after_noncounting_tick", 2: "pc_straddle_first_fetch", 3: "pc_word_and_alignment",
                     4: "pc_aligned_mid_decode", 5: "pc_two_values", 6: "pc_on_fault_attempt",
                     7: "pc_macro_op_access", 8: "reads_curtick"}
CPU_ATOMIC, CPU_TIMING = 0, 1
HANG_NAMES = {1: "max_insts", 2: "m5_quiesce"}
END_NAMES = {0: "exit", 1: "m5_exit", 2: "m5_fail"}     # sub-codes of masked / sdc: how the run ended
T_PC, T_MEM, T_RESULT, N_STRUCT = 32, 33, 34, 35

OUTCOME_DT = np.dtype([("cls", "u1"), ("sub", "u1"), ("exit_code", "u1"), ("flags", "u1"),
                       ("detail", "<u4"), ("ninst", "<u8")])
SITE_DT = np.dtype([("inst", "<u8"), ("mask", "<u8"), ("addr", "<u8"), ("target", "<u4"), ("trial", "<u4")])
HIST_DT = np.dtype([("counts", "<u8", (N_STRUCT, 64, 6)), ("crash_sub", "<u8", (16,)), ("escape_sub", "<u8", (8,)),
                    ("trials", "<u8"), ("guest_insts", "<u8"), ("fetch_bytes", "<u8"), ("data_bytes", "<u8"),
                    ("cow_pages", "<u8"), ("device_insts", "<u8")])

ABI_NAMES = {"zero": 0, "ra": 1, "sp": 2, "gp": 3, "tp": 4, "t0": 5, "t1": 6, "t2": 7, "s0": 8, "fp": 8, "s1": 9,
             **{f"a{i}": 10 + i for i in range(8)}, **{f"s{i}": 16 + i for i in range(2, 12)},
             "t3": 28, "t4": 29, "t5": 30, "t6": 31}


# gem5 OpClass enum (src/cpu/FuncUnit.py:43), for protect_opclasses by name
OPCLASS_NAMES = ["No_OpClass", "IntAlu", "IntMult", "IntDiv", "FloatAdd", "FloatCmp", "FloatCvt", "FloatMult",
                 "FloatMultAcc", "FloatDiv", "FloatMisc", "FloatSqrt"]
OPCLASS_MEMREAD, OPCLASS_MEMWRITE, OPCLASS_FLOATMEMREAD, OPCLASS_FLOATMEMWRITE = 52, 53, 54, 55


def opclass_mask(opclasses: Iterable[str | int] | int) -> int:
    """gem5 OpClass names ('IntAlu', 'IntMult', ...) or enum values -> bitmask."""
    if isinstance(opclasses, int):
        return opclasses
    named = dict(zip(OPCLASS_NAMES, range(len(OPCLASS_NAMES))))
    named.update(MemRead=OPCLASS_MEMREAD, MemWrite=OPCLASS_MEMWRITE, FloatMemRead=OPCLASS_FLOATMEMREAD,
                 FloatMemWrite=OPCLASS_FLOATMEMWRITE)
    m = 0
    for c in opclasses:
        k = c if isinstance(c, int) else named[c.removesuffix("Op")]
        if not 0 <= k < 64:
            raise ValueError(f"OpClass {c!r} outside the 64-bit mask")
        m |= 1 << k
    return m


def structures_mask(structures: Iterable[str] | int) -> int:
    """'int_reg' (x1..x31), 'pc', 'mem', or register names ('x5', 'a0', 'sp') -> bitmask."""
    if isinstance(structures, int):
        return structures
    m = 0
    for s in structures:
        s = s.strip().lower()
        if s in ("int_reg", "intreg", "regs", "regfile"):
            m |= ((1 << 32) - 1) & ~1
        elif s == "pc":
            m |= 1 << T_PC
        elif s in ("mem", "memory"):
            m |= 1 << T_MEM
        elif s in ("result", "fu", "inst_result"):
            m |= 1 << T_RESULT
        elif s in ABI_NAMES:
            m |= 1 << ABI_NAMES[s]
        elif s.startswith("x") and s[1:].isdigit() and 0 <= int(s[1:]) < 32:
            m |= 1 << int(s[1:])
        else:
            raise ValueError(f"unknown fault structure {s!r}")
    return m & ~1


class EngineError(RuntimeError):
    pass


class _Config(C.Structure):
    _fields_ = [("device", C.c_int32), ("private_pages", C.c_uint32), ("hang_factor_x16", C.c_uint32),
                ("max_trials_per_launch", C.c_uint32), ("snapshot_interval", C.c_uint32), ("flags", C.c_uint32),
                ("epoch_iters", C.c_uint32), ("lanes_per_wave", C.c_uint32),
                ("resume_lanes", C.c_uint32), ("epochs", C.c_uint32)]


CFG_NO_SNAPSHOT_START = 1
CFG_NO_EARLY_EXIT = 2
CFG_NO_TRANSLATE = 4
CFG_NO_EPOCHS = 8
CFG_PACK_RUNS = 16
CFG_FIXED_RESUME = 32
CFG_NO_SOLO = 64
CFG_SOLO_ALL = 128
CFG_SIMT = 256
CFG_NO_FORWARD = 512
CFG_NO_SDC_EXIT = 1024
CFG_NO_REDO = 2048
CFG_NO_ODD_KERNEL = 4096
CFG_JIT_NO_CACHE = 8192
CFG_NO_HANG_PROOF = 16384
CFG_NO_OVERFLOW = 32768
CFG_NO_LOOP_ORDER = 65536


class GoldenInfo(C.Structure):
    _fields_ = [("ninst", C.c_uint64), ("ncycles", C.c_uint64), ("exit_code", C.c_uint32), ("pad", C.c_uint32),
                ("stdout_len", C.c_uint64), ("stderr_len", C.c_uint64), ("fetch_bytes", C.c_uint64),
                ("data_bytes", C.c_uint64), ("snapshots", C.c_uint64), ("snapshot_interval", C.c_uint64),
                ("snapshot_frames", C.c_uint64), ("translated_blocks", C.c_uint64),
                ("translated_insts", C.c_uint64), ("translate_us", C.c_uint64)]


class IssueParams(C.Structure):
    """fi_issue_params: the O3 issue model of SHREWD's FU contention."""
    _fields_ = [("issue_width", C.c_uint32), ("dispatch_width", C.c_uint32), ("commit_width", C.c_uint32),
                ("iq_entries", C.c_uint32), ("rob_entries", C.c_uint32), ("load_latency", C.c_uint32),
                ("priority_to_shadow", C.c_uint32), ("fu_count", C.c_uint32 * 6)]


class IssueStats(C.Structure):
    _fields_ = [("ops", C.c_uint64), ("cycles", C.c_uint64), ("shadow_available", C.c_uint64),
                ("shadow_not_available", C.c_uint64), ("shadow_same_fu", C.c_uint64),
                ("shadow_not_same_fu", C.c_uint64), ("class_available", C.c_uint64 * 12),
                ("class_not_available", C.c_uint64 * 12)]

    def as_dict(self) -> dict:
        d = {n: getattr(self, n) for n in ("ops", "cycles", "shadow_available", "shadow_not_available",
                                              "shadow_same_fu", "shadow_not_same_fu")}
        for n in ("class_available", "class_not_available"):
            d[n] = {OPCLASS_NAMES[k]: int(getattr(self, n)[k]) for k in range(1, 12) if getattr(self, n)[k]}
        return d


ISSUE_OP_DT = np.dtype([("src", "<u8"), ("dst", "<u8"), ("opclass", "u1"), ("kind", "u1"), ("pad", "u1", (6,))])

# ---- tick-domain injection under TimingSimpleCPU (include/fi_engine.h)
TIMING_OP_DT = np.dtype([("fetch", "<u8", (2,)), ("addr", "<u8", (2,)), ("size", "<u2", (2,)), ("nfetch", "u1"),
                         ("nfrag", "u1"), ("kind", "u1"), ("cmd", "u1"), ("pad", "u1", (8,))])
TIMING_TICKS_DT = np.dtype([("fetch_send", "<u8", (2,)), ("fetch_done", "<u8", (2,)), ("exec", "<u8"),
                            ("done", "<u8")])
# include/fi_debug.h fi_debug_loop / fi_debug_loop_out
DEBUG_LOOP_DT = np.dtype([("regs", "<u8", (32,)), ("left", "<u8"), ("lp_cnt", "<u4"), ("lp_m", "<u4"), ("lp_n", "<u4"),
                          ("lp_ld", "<u4", (4, 3)), ("pad", "<u4")])
DEBUG_LOOP_OUT_DT = np.dtype([("verdict", "<i4"), ("body_proof", "<u4"), ("k", "<u8"), ("fva", "<u8")])
TICK_SITE_DT = np.dtype([("tick", "<u8"), ("mask", "<u8"), ("target", "<u4"), ("trial", "<u4")])
TOP_EXEC, TOP_FAULT, TOP_END = 0, 1, 2
TCMD_READ, TCMD_WRITE, TCMD_SWAP, TCMD_LL, TCMD_SC = 0, 1, 2, 3, 4


class TimingParams(C.Structure):
    """fi_timing_params: the reference SE board (NoCache SystemXBar, DDR3-1600, 3 GHz)."""
    _fields_ = ([("cpu_period", C.c_uint64)] +
                [(n, C.c_uint32) for n in ("xbar_frontend", "xbar_forward", "xbar_response", "xbar_header",
                                           "xbar_width", "xbar_sf_lookup")] +
                [(n, C.c_uint64) for n in ("mc_frontend", "mc_backend", "mc_command_window")] +
                [(n, C.c_uint32) for n in ("read_buffer", "write_buffer", "write_high_pct", "write_low_pct",
                                           "min_writes_per_switch", "min_reads_per_switch")] +
                [(n, C.c_uint64) for n in ("tCK", "tBURST", "tRCD", "tCL", "tRP", "tRAS", "tRRD", "tXAW", "tRFC",
                                           "tWR", "tWTR", "tRTP", "tRTW", "tCS", "tREFI")] +
                [(n, C.c_uint32) for n in ("activation_limit", "ranks", "banks", "burst_bytes",
                                           "row_buffer_bytes", "max_accesses_per_row")] +
                [("mem_bytes", C.c_uint64)])


class TimingStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("ops", "ticks", "reads", "writes", "write_queue_hits", "row_hits",
                                          "activates", "refreshes", "xbar_retries", "mc_retries")]

    def as_dict(self) -> dict:
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class TickInfo(C.Structure):
    _fields_ = [("golden_ticks", C.c_uint64), ("attempts", C.c_uint64), ("stats", TimingStats),
                ("status", C.c_char * 160)]


def timing_params(**kw) -> TimingParams:
    """The reference board's timing parameters with overrides by field name."""
    p = TimingParams()
    lib().fi_timing_default_params(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, int(v))
    return p


def timing_model_run(ops: np.ndarray, params: TimingParams | None = None):
    """fi_timing_model_run (pure host code): -> (ticks TIMING_TICKS_DT[n], TimingStats)."""
    ops = np.ascontiguousarray(ops, TIMING_OP_DT)
    out = np.zeros(len(ops), TIMING_TICKS_DT)
    st = TimingStats()
    rc = lib().fi_timing_model_run(ops.ctypes.data, len(ops), C.byref(params or timing_params()),
                                   out.ctypes.data, C.byref(st))
    if rc != FI_OK:
        raise EngineError(f"fi_timing_model_run: {rc}")
    return out, st


ISSUE_PLAIN, ISSUE_LOAD, ISSUE_STORE, ISSUE_SERIAL = 0, 1, 2, 3
FU_NAMES = ("IntALU", "IntMultDiv", "FP_ALU", "FP_MultDiv", "RdWrPort", "IprPort")


def issue_params(**kw) -> IssueParams:
    """The reference's O3 defaults (BaseO3CPU.py, FuncUnitConfig.py) with
    overrides by field name; fu_count also by FU name (IntALU=4, ...)."""
    p = IssueParams()
    lib().fi_issue_default_params(C.byref(p))
    for k, v in kw.items():
        if k in FU_NAMES:
            p.fu_count[FU_NAMES.index(k)] = int(v)
        elif k == "fu_count":
            for i, c in enumerate(v):
                p.fu_count[i] = int(c)
        else:
            setattr(p, k, int(v))
    return p


def issue_model_run(ops: np.ndarray, params: IssueParams | None = None):
    """fi_issue_model_run (pure host code): -> (shadow uint8[n], IssueStats)."""
    ops = np.ascontiguousarray(ops, ISSUE_OP_DT)
    p = params if params is not None else issue_params()
    out = np.zeros(len(ops), np.uint8)
    st = IssueStats()
    rc = lib().fi_issue_model_run(ops.ctypes.data, len(ops), C.byref(p), out.ctypes.data, C.byref(st))
    if rc != FI_OK:
        raise EngineError(f"fi_issue_model_run: {rc}")
    return out, st


_lib = None


def library_path() -> str:
    return os.environ.get("SHREWD_FI_LIB", _build.OUT)


def build_library(force: bool = False) -> str:
    return _build.build(force=force)


def lib():
    global _lib
    if _lib is None:
        path = library_path()
        if not os.path.exists(path):
            raise EngineError(f"{path} missing: run `python -m shrewd_amd.build` (hipcc, gfx950)")
        L = C.CDLL(path)
        vp = C.c_void_p
        L.fi_create.argtypes = [C.POINTER(_Config), C.POINTER(vp)]
        L.fi_destroy.argtypes = [vp]
        L.fi_last_error.restype = C.c_char_p
        L.fi_last_error.argtypes = [vp]
        L.fi_load_elf.argtypes = [vp, C.c_char_p, C.c_size_t, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p)]
        L.fi_golden_run.argtypes = [vp, C.POINTER(GoldenInfo)]
        L.fi_wait_translation.argtypes = [vp, C.POINTER(GoldenInfo)]
        L.fi_load_checkpoint.argtypes = [vp, C.c_char_p, C.c_char_p, C.c_size_t]
        L.fi_golden_stdout.argtypes = [vp, C.c_char_p, C.c_uint64, C.POINTER(C.c_uint64)]
        L.fi_golden_stderr.argtypes = [vp, C.c_char_p, C.c_uint64, C.POINTER(C.c_uint64)]
        L.fi_set_campaign.argtypes = [vp, C.c_uint64, C.c_uint64, C.c_uint32]
        L.fi_set_bits.argtypes = [vp, C.c_uint64]
        L.fi_set_clock.argtypes = [vp, C.c_uint64, C.c_uint64]
        L.fi_set_exe_path.argtypes = [vp, C.c_char_p]
        L.fi_set_stdin.argtypes = [vp, C.c_char_p, C.c_uint64]
        L.fi_set_protect.argtypes = [vp, C.c_uint64]
        L.fi_set_protect_opclasses.argtypes = [vp, C.c_uint64]
        L.fi_sample_sites.argtypes = [vp, C.c_uint64, C.c_uint64, vp]
        L.fi_run_trials.argtypes = [vp, C.c_uint64, C.c_uint64, vp, vp]
        L.fi_run_sites.argtypes = [vp, vp, C.c_uint64, vp, vp]
        L.fi_run_trials_device.argtypes = [vp, C.c_uint64, C.c_uint64, vp, vp, vp]
        L.fi_sync.argtypes = [vp]
        L.fi_last_kernel_ms.restype = C.c_double
        L.fi_last_kernel_ms.argtypes = [vp]
        L.fi_debug_decode.argtypes = [vp, vp, C.c_uint64, vp]
        L.fi_debug_loop_outcome.argtypes = [vp, vp, C.c_uint64, vp]
        L.fi_kernel_timer_reset.argtypes = [vp]
        L.fi_get_config.argtypes = [vp, C.POINTER(_Config)]
        L.fi_debug_stats.argtypes = [vp, vp]
        L.fi_debug_softfp.argtypes = [C.c_int, C.c_int, C.c_int, vp, vp, vp, C.c_uint64, vp, vp, C.c_int]
        L.fi_debug_crypto.argtypes = [C.c_int, vp, vp, C.c_uint64, vp, C.c_int]
        L.fi_kernel_timer_read.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_uint32)]
        L.fi_debug_waves.argtypes = [vp, vp, C.c_uint64]
        L.fi_debug_epochs.argtypes = [vp, vp]
        L.fi_debug_dispatch_ms.argtypes = [vp, vp, C.c_uint32, C.POINTER(C.c_uint32)]
        L.fi_debug_dispatch_kinds.argtypes = [vp, vp, C.c_uint32, C.POINTER(C.c_uint32)]
        L.fi_debug_dispatch_span_ms.argtypes = [vp, vp, C.c_uint32, C.POINTER(C.c_uint32)]
        L.fi_debug_golden_trace.argtypes = [vp, vp, C.c_uint64, C.POINTER(C.c_uint64), vp, C.c_uint64,
                                            C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.fi_debug_translate.argtypes = [vp, C.c_uint64, C.c_uint64, vp, C.c_uint64, C.c_char_p, C.c_uint64,
                                         C.POINTER(C.c_uint64)]
        L.fi_debug_translation.argtypes = [vp, C.c_char_p, C.c_uint64, C.POINTER(C.c_uint64)]
        L.fi_issue_default_params.argtypes = [C.POINTER(IssueParams)]
        L.fi_issue_model_run.argtypes = [vp, C.c_uint64, C.POINTER(IssueParams), vp, C.POINTER(IssueStats)]
        L.fi_set_issue_model.argtypes = [vp, C.POINTER(IssueParams)]
        L.fi_shadow_map.argtypes = [vp, vp, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(IssueStats)]
        L.fi_timing_default_params.argtypes = [C.POINTER(TimingParams)]
        L.fi_timing_model_run.argtypes = [vp, C.c_uint64, C.POINTER(TimingParams), vp, C.POINTER(TimingStats)]
        L.fi_set_cpu_model.argtypes = [vp, C.c_int, C.POINTER(TimingParams)]
        L.fi_tick_golden.argtypes = [vp, C.POINTER(TickInfo)]
        L.fi_tick_trace.argtypes = [vp, vp, vp, C.c_uint64, C.POINTER(C.c_uint64)]
        L.fi_sample_tick_sites.argtypes = [vp, C.c_uint64, C.c_uint64, vp]
        L.fi_map_tick_sites.argtypes = [vp, vp, C.c_uint64, vp, vp, vp]
        L.fi_run_tick_sites.argtypes = [vp, vp, C.c_uint64, vp, vp]
        L.fi_run_tick_trials.argtypes = [vp, C.c_uint64, C.c_uint64, vp, vp]
        L.fi_translate_status.restype = C.c_char_p
        L.fi_translate_status.argtypes = [vp]
        _lib = L
    return _lib


def _cstrs(items: Sequence[str] | None):
    items = list(items or [])
    arr = (C.c_char_p * (len(items) + 1))()
    for i, s in enumerate(items):
        arr[i] = s.encode()
    arr[len(items)] = None
    return arr


class Engine:
    """Thin RAII wrapper of one fi_engine (one HIP device)."""

    def __init__(self, device: int = 0, private_pages: int = 16, hang_factor_x16: int = 32,
                 max_trials_per_launch: int = 0, snapshot_interval: int = 0, flags: int = 0,
                 epoch_iters: int = 0, lanes_per_wave: int = 0, resume_lanes: int = 0,
                 epochs: int = 0):
        self.L = lib()
        cfg = _Config(device, private_pages, hang_factor_x16, max_trials_per_launch, snapshot_interval, flags,
                      epoch_iters, lanes_per_wave, resume_lanes, epochs)
        h = C.c_void_p()
        st = self.L.fi_create(C.byref(cfg), C.byref(h))
        if st == FI_E_NODEVICE:
            raise EngineError("no HIP device visible: the engine has no CPU path")
        if st != FI_OK:
            raise EngineError(f"fi_create failed ({st})")
        self.h = h
        self.golden: GoldenInfo | None = None

    def close(self):
        if getattr(self, "h", None):
            self.L.fi_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def _chk(self, st: int, what: str):
        if st != FI_OK:
            raise EngineError(f"{what}: {self.L.fi_last_error(self.h).decode()} ({st})")

    def load_elf(self, elf: bytes, argv: Sequence[str], envp: Sequence[str] | None = None):
        self._chk(self.L.fi_load_elf(self.h, elf, len(elf), _cstrs(argv), _cstrs(envp)), "fi_load_elf")

    def load_checkpoint(self, directory: str, elf: bytes):
        """Start from a gem5 SE checkpoint (fi_load_checkpoint); elf = the workload."""
        self._chk(self.L.fi_load_checkpoint(self.h, directory.encode(), elf, len(elf)), "fi_load_checkpoint")

    def golden_run(self, wait_translation: bool = True) -> GoldenInfo:
        """fi_golden_run; wait_translation: also wait for the background build
        of the translated kernels (fi_wait_translation) -- otherwise trials
        start on the static kernels and pick the build up when it lands."""
        g = GoldenInfo()
        self._chk(self.L.fi_golden_run(self.h, C.byref(g)), "fi_golden_run")
        if wait_translation:
            self._chk(self.L.fi_wait_translation(self.h, C.byref(g)), "fi_wait_translation")
        self.golden = g
        return g

    def wait_translation(self) -> GoldenInfo:
        g = GoldenInfo()
        self._chk(self.L.fi_wait_translation(self.h, C.byref(g)), "fi_wait_translation")
        self.golden = g
        return g

    def _golden_stream(self, fn, what) -> bytes:
        n = C.c_uint64()
        self._chk(fn(self.h, None, 0, C.byref(n)), what)        # length first: no silent truncation
        buf = C.create_string_buffer(max(n.value, 1))
        self._chk(fn(self.h, buf, n.value, C.byref(n)), what)
        return buf.raw[:n.value]

    def golden_stdout(self) -> bytes:
        return self._golden_stream(self.L.fi_golden_stdout, "fi_golden_stdout")

    def golden_stderr(self) -> bytes:
        return self._golden_stream(self.L.fi_golden_stderr, "fi_golden_stderr")

    def set_bits(self, bits: int):
        """Eligible lowest flipped bit positions (mask; ~0 = all): fi_set_bits."""
        self._chk(self.L.fi_set_bits(self.h, bits & (2**64 - 1)), "fi_set_bits")

    def set_exe_path(self, path: str):
        """What readlinkat("/proc/self/exe") answers: the executable's realpath."""
        self._chk(self.L.fi_set_exe_path(self.h, path.encode()), "fi_set_exe_path")

    def set_stdin(self, data: bytes | None):
        """Process.input as a file: the bytes read(0) returns (fi_set_stdin);
        None = "cin", the host's stdin (reads of fd 0 escape as host).  Before
        golden_run()."""
        self._chk(self.L.fi_set_stdin(self.h, data, 0 if data is None else len(data)), "fi_set_stdin")

    def set_clock(self, period_ticks: int = 500, random_seed: int = 5489):
        """clock_gettime's ticks per CPU cycle and getrandom's gem5 Random seed."""
        self._chk(self.L.fi_set_clock(self.h, period_ticks, random_seed), "fi_set_clock")

    def set_campaign(self, seed: int, structures, burst: int = 1):
        self._chk(self.L.fi_set_campaign(self.h, seed & (2**64 - 1), structures_mask(structures), burst),
                  "fi_set_campaign")

    def set_protect(self, mask: int):
        self._chk(self.L.fi_set_protect(self.h, mask), "fi_set_protect")

    def set_protect_opclasses(self, opclasses):
        self._chk(self.L.fi_set_protect_opclasses(self.h, opclass_mask(opclasses)), "fi_set_protect_opclasses")

    def set_issue_model(self, params: IssueParams | dict | None = None, **kw):
        """SHREWD FU contention for result faults (fi_set_issue_model): None and
        no keywords -> off; a dict / keywords override the O3 defaults."""
        if params is None and not kw:
            self._chk(self.L.fi_set_issue_model(self.h, None), "fi_set_issue_model")
            return
        p = params if isinstance(params, IssueParams) else issue_params(**{**(params or {}), **kw})
        self._chk(self.L.fi_set_issue_model(self.h, C.byref(p)), "fi_set_issue_model")

    def shadow_map(self):
        """(uint8 per golden numInst index: shadow issued, IssueStats)"""
        n, st = C.c_uint64(), IssueStats()
        self._chk(self.L.fi_shadow_map(self.h, None, 0, C.byref(n), None), "fi_shadow_map")
        out = np.zeros(n.value, np.uint8)
        self._chk(self.L.fi_shadow_map(self.h, out.ctypes.data, n.value, C.byref(n), C.byref(st)), "fi_shadow_map")
        return out, st

    # ---- tick-domain injection under TimingSimpleCPU
    def set_cpu_model(self, model: int | str, params: TimingParams | None = None):
        """fi_set_cpu_model: 'atomic' (numInst sites) or 'timing' (tick sites on
        the reference board); before golden_run()."""
        if isinstance(model, str):
            model = {"atomic": CPU_ATOMIC, "timing": CPU_TIMING}[model.lower().removesuffix("simplecpu")]
        self._chk(self.L.fi_set_cpu_model(self.h, model, C.byref(params) if params is not None else None),
                  "fi_set_cpu_model")

    def tick_info(self) -> dict:
        t = TickInfo()
        self._chk(self.L.fi_tick_golden(self.h, C.byref(t)), "fi_tick_golden")
        return {"golden_ticks": int(t.golden_ticks), "attempts": int(t.attempts), "stats": t.stats.as_dict(),
                "status": t.status.decode()}

    def tick_trace(self):
        """(ops TIMING_OP_DT, ticks TIMING_TICKS_DT): the golden run's attempts."""
        n = C.c_uint64()
        self._chk(self.L.fi_tick_trace(self.h, None, None, 0, C.byref(n)), "fi_tick_trace")
        ops = np.zeros(n.value, TIMING_OP_DT)
        ticks = np.zeros(n.value, TIMING_TICKS_DT)
        self._chk(self.L.fi_tick_trace(self.h, ops.ctypes.data, ticks.ctypes.data, n.value, C.byref(n)),
                  "fi_tick_trace")
        return ops, ticks

    def sample_tick_sites(self, first: int, n: int) -> np.ndarray:
        out = np.zeros(n, TICK_SITE_DT)
        self._chk(self.L.fi_sample_tick_sites(self.h, first, n, out.ctypes.data), "fi_sample_tick_sites")
        return out

    def map_tick_sites(self, ts: np.ndarray):
        """-> (numInst sites, disposition 0 run / 1 golden / 2 escape, host outcomes)"""
        ts = np.ascontiguousarray(ts, TICK_SITE_DT)
        sites = np.zeros(len(ts), SITE_DT)
        disp = np.zeros(len(ts), np.uint8)
        ho = np.zeros(len(ts), OUTCOME_DT)
        self._chk(self.L.fi_map_tick_sites(self.h, ts.ctypes.data, len(ts), sites.ctypes.data, disp.ctypes.data,
                                           ho.ctypes.data), "fi_map_tick_sites")
        return sites, disp, ho

    def run_tick_sites(self, ts: np.ndarray):
        ts = np.ascontiguousarray(ts, TICK_SITE_DT)
        out = np.zeros(len(ts), OUTCOME_DT)
        hist = np.zeros(1, HIST_DT)
        self._chk(self.L.fi_run_tick_sites(self.h, ts.ctypes.data, len(ts), out.ctypes.data, hist.ctypes.data),
                  "fi_run_tick_sites")
        return out, hist[0]

    def run_tick_trials(self, first: int, n: int, want_outcomes: bool = True):
        out = np.zeros(n, OUTCOME_DT) if want_outcomes else None
        hist = np.zeros(1, HIST_DT)
        self._chk(self.L.fi_run_tick_trials(self.h, first, n, out.ctypes.data if out is not None else None,
                                            hist.ctypes.data), "fi_run_tick_trials")
        return out, hist[0]

    def sample(self, first: int, n: int) -> np.ndarray:
        out = np.zeros(n, SITE_DT)
        self._chk(self.L.fi_sample_sites(self.h, first, n, out.ctypes.data), "fi_sample_sites")
        return out

    def run_trials(self, first: int, n: int, want_outcomes: bool = True):
        out = np.zeros(n, OUTCOME_DT) if want_outcomes else None
        hist = np.zeros(1, HIST_DT)
        self._chk(self.L.fi_run_trials(self.h, first, n, out.ctypes.data if out is not None else None,
                                       hist.ctypes.data), "fi_run_trials")
        return out, hist[0]

    def run_sites(self, sites: np.ndarray):
        sites = np.ascontiguousarray(sites, SITE_DT)
        out = np.zeros(len(sites), OUTCOME_DT)
        hist = np.zeros(1, HIST_DT)
        self._chk(self.L.fi_run_sites(self.h, sites.ctypes.data, len(sites), out.ctypes.data, hist.ctypes.data),
                  "fi_run_sites")
        return out, hist[0]

    def run_trials_device(self, first: int, n: int, d_out: int, d_hist: int, stream: int | None = None):
        self._chk(self.L.fi_run_trials_device(self.h, first, n, d_out, d_hist, stream), "fi_run_trials_device")

    def sync(self):
        self._chk(self.L.fi_sync(self.h), "fi_sync")

    def translate_status(self) -> str:
        """"" when the translated path is on, else why not."""
        return self.L.fi_translate_status(self.h).decode()

    def debug_waves(self, n_waves: int) -> np.ndarray:
        out = np.zeros((n_waves, 10), np.uint64)
        self._chk(self.L.fi_debug_waves(self.h, out.ctypes.data, n_waves), "fi_debug_waves")
        return out

    def debug_epochs(self) -> list:
        out = np.zeros(16, np.uint32)
        self._chk(self.L.fi_debug_epochs(self.h, out.ctypes.data), "fi_debug_epochs")
        return out.tolist()

    def debug_dispatch_ms(self) -> list:
        ms = np.zeros(256, np.float32)
        n = C.c_uint32()
        self._chk(self.L.fi_debug_dispatch_ms(self.h, ms.ctypes.data, 256, C.byref(n)), "fi_debug_dispatch_ms")
        return [round(float(x), 3) for x in ms[:min(n.value, 256)]]

    def debug_dispatch_span_ms(self) -> list:
        """Device busy span of each dispatch since kernel_timer_reset (ms):
        first to last stamp of the waves that ran a trial."""
        ms = np.zeros(256, np.float32)
        n = C.c_uint32()
        self._chk(self.L.fi_debug_dispatch_span_ms(self.h, ms.ctypes.data, 256, C.byref(n)),
                  "fi_debug_dispatch_span_ms")
        return [round(float(x), 3) for x in ms[:min(n.value, 256)]]

    def debug_dispatch_kinds(self) -> list:
        """Kernel of each dispatch of debug_dispatch_ms: 0 64-lane, 1 solo, 2 solo-odd."""
        k = np.zeros(256, np.uint32)
        n = C.c_uint32()
        self._chk(self.L.fi_debug_dispatch_kinds(self.h, k.ctypes.data, 256, C.byref(n)), "fi_debug_dispatch_kinds")
        return k[:min(n.value, 256)].tolist()

    def debug_golden_trace(self):
        """(pre-decoded text as uint8[n,16], golden trace uint32[m], text_lo)"""
        npre, ntr, lo = C.c_uint64(), C.c_uint64(), C.c_uint64()
        self.L.fi_debug_golden_trace(self.h, None, 0, C.byref(npre), None, 0, C.byref(ntr), C.byref(lo))
        pre = np.zeros((npre.value, 16), np.uint8)
        tr = np.zeros(ntr.value, np.uint32)
        self.L.fi_debug_golden_trace(self.h, pre.ctypes.data, npre.value, C.byref(npre), tr.ctypes.data, ntr.value,
                                     C.byref(ntr), C.byref(lo))
        return pre, tr, lo.value

    def debug_translation(self) -> str:
        n = C.c_uint64()
        self.L.fi_debug_translation(self.h, None, 0, C.byref(n))
        buf = C.create_string_buffer(n.value + 1)
        self.L.fi_debug_translation(self.h, buf, n.value + 1, C.byref(n))
        return buf.value.decode()

    def last_kernel_ms(self) -> float:
        return self.L.fi_last_kernel_ms(self.h)

    def debug_stats(self) -> np.ndarray:
        out = np.zeros(64, np.uint64)
        self._chk(self.L.fi_debug_stats(self.h, out.ctypes.data), "fi_debug_stats")
        return out

    def config(self) -> dict:
        cfg = _Config()
        self._chk(self.L.fi_get_config(self.h, C.byref(cfg)), "fi_get_config")
        return {n: getattr(cfg, n) for n, _ in _Config._fields_}

    def kernel_timer_reset(self):
        self._chk(self.L.fi_kernel_timer_reset(self.h), "fi_kernel_timer_reset")

    def kernel_timer_read(self):
        ms, n = C.c_double(), C.c_uint32()
        self._chk(self.L.fi_kernel_timer_read(self.h, C.byref(ms), C.byref(n)), "fi_kernel_timer_read")
        return ms.value, n.value

    def debug_decode(self, raws: np.ndarray) -> np.ndarray:
        raws = np.ascontiguousarray(raws, np.uint32)
        dt = np.dtype([("raw", "<u4"), ("op", "u1"), ("rd", "u1"), ("rs1", "u1"), ("rs2", "u1"), ("imm", "<i4"),
                       ("len", "u1"), ("flags", "u1"), ("aux", "<u2")])
        out = np.zeros(len(raws), dt)
        self._chk(self.L.fi_debug_decode(self.h, raws.ctypes.data, len(raws), out.ctypes.data), "fi_debug_decode")
        return out

    def debug_loop_outcome(self, loops: np.ndarray) -> np.ndarray:
        """fi_debug_loop_outcome: loop_outcome (and the body's capped proof)
        on DEBUG_LOOP_DT records -> DEBUG_LOOP_OUT_DT."""
        loops = np.ascontiguousarray(loops, DEBUG_LOOP_DT)
        out = np.zeros(len(loops), DEBUG_LOOP_OUT_DT)
        self._chk(self.L.fi_debug_loop_outcome(self.h, loops.ctypes.data, len(loops), out.ctypes.data),
                  "fi_debug_loop_outcome")
        return out


def inst_group(raw: int) -> str:
    """gem5 instruction group of an `escape/inst` outcome's raw word (its
    `detail`): the opcode groups of src/arch/riscv/isa/decoder.isa that the
    engine decodes exactly but does not execute."""
    raw &= 0xFFFFFFFF
    if raw & 3 != 3:
        return "compressed"
    opc, f3 = (raw >> 2) & 31, (raw >> 12) & 7
    if opc == 0x15 or (opc in (0x01, 0x09) and f3 in (0, 5, 6, 7)):
        return "vector"                          # OP-V; LOAD-FP / STORE-FP vector widths
    if opc in (0x01, 0x09, 0x10, 0x11, 0x12, 0x13, 0x14):
        return "fp"
    if opc == 0x1e:
        return "m5op"
    if opc == 0x0b:
        return "amo"
    if opc == 0x1c:
        return "system" if f3 == 0 else "hypervisor" if f3 == 4 else "csr"
    if opc == 0x03:
        return "cbo"
    if opc in (0x04, 0x0c):
        return "crypto"
    return "other"


def escape_breakdown(out: np.ndarray) -> dict:
    """Escape outcomes by sub-code and, for escape/inst, by gem5 instruction
    group ("inst:vector", ...); escape/syscall by number ("syscall:78")."""
    esc = out[out["cls"] == 5]
    res: dict[str, int] = {}
    for sub, det in zip(esc["sub"].tolist(), esc["detail"].tolist()):
        name = ESCAPE_NAMES.get(sub, str(sub))
        if sub in (1, 6):
            name += ":" + inst_group(det)
        elif sub == 2:
            name += f":{det}"
        res[name] = res.get(name, 0) + 1
    return dict(sorted(res.items()))


def shard_range(trials: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous trial-id block of `rank`: [r*T/G, (r+1)*T/G).
    Sites are counter-based on (seed, trial id), so any sharding runs the same
    trials."""
    lo = trials * rank // world
    hi = trials * (rank + 1) // world
    return lo, hi - lo


def allreduce_histogram(hist, device=None, group=None):
    """Sum an outcome histogram (HIST_DT record) over all ranks: the campaign's
    only exchange.  RCCL over xGMI when `device` is a GPU and the process group
    is "nccl"; any torch.distributed backend works (gloo in CPU tests)."""
    import torch
    import torch.distributed as dist
    words = np.frombuffer(np.asarray(hist, HIST_DT).tobytes(), np.int64).copy()
    t = torch.from_numpy(words)
    if device is not None:
        t = t.to(device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return np.frombuffer(t.cpu().numpy().tobytes(), HIST_DT)[0].copy()


def bits_mask(spec) -> int:
    """`bits` parameter -> mask of eligible lowest flipped bit positions: an int
    mask, or a string of positions and ranges ("0-31,63"); None / "" = all."""
    if spec is None or spec == "":
        return 2**64 - 1
    if isinstance(spec, int):
        return spec & (2**64 - 1)
    m = 0
    for part in str(spec).split(","):
        part = part.strip()
        if not part:
            continue
        lo, _, hi = part.partition("-")
        lo, hi = int(lo, 0), int(hi or lo, 0)
        if not 0 <= lo <= hi <= 63:
            raise ValueError(f"bad bit range {part!r}")
        for b in range(lo, hi + 1):
            m |= 1 << b
    return m


class FaultCampaign:
    """Mirror of the gem5 `FaultCampaign` SimObject (src/gem5ext/FaultCampaign.py).

    Params (same names/meaning as the SimObject): workload (binary path), cmd
    (argv, cmd[0] defaults to workload), env, trials, seed, structures, bits,
    burst, protect_mask, protect_opclasses, num_gpus, max_insts_factor, output;
    executable (gem5's Process.executable: what /proc/self/exe resolves to;
    default the workload path, as gem5's se configs set it), input
    (Process.input: "cin" = the host's stdin, reads of fd 0 escape; else a
    file, opened relative to the working directory, that fd 0 reads);
    checkpoint (a gem5 SE checkpoint directory to start from),
    shadow_fu_model (SHREWD FU contention for result faults, off by default),
    priority_to_shadow and issue_params (the O3 issue model's parameters);
    cpu_type ("atomic": sites at a committed-instruction count, the default;
    "timing": sites at a tick of a TimingSimpleCPU run on the reference run
    script's NoCache + SingleChannelDDR3_1600 board -- simple_binary_run.py's
    CPUTypes.TIMING -- mapped to the instruction in flight) and timing_params.
    """

    def __init__(self, workload: str, cmd: Sequence[str] | None = None, env: Sequence[str] | None = None,
                 trials: int = 1000, seed: int = 0x5EED0001, structures=("int_reg",), burst: int = 1,
                 protect_mask: int = 0, num_gpus: int = 1, max_insts_factor: float = 2.0, output: str = "",
                 device: int = 0, private_pages: int = 16, protect_opclasses=(), bits=None,
                 shadow_fu_model: bool = False, priority_to_shadow: bool = False, issue_params: dict | None = None,
                 checkpoint: str = "", executable: str | None = None, input: str = "cin",
                 cpu_type: str = "atomic", timing_params: TimingParams | None = None):
        self.workload, self.cmd, self.env = workload, list(cmd or [workload]), list(env or [])
        self.trials, self.seed, self.structures, self.burst = trials, seed, structures, burst
        self.protect_mask, self.num_gpus, self.output = protect_mask, num_gpus, output
        self.max_insts_factor = max_insts_factor
        self.engine = Engine(device=device, private_pages=private_pages,
                             hang_factor_x16=max(1, int(round(max_insts_factor * 16))))
        self.checkpoint = checkpoint
        with open(workload, "rb") as f:
            if checkpoint:
                self.engine.load_checkpoint(checkpoint, f.read())
            else:
                self.engine.load_elf(f.read(), self.cmd, self.env)
        # gem5 answers /proc/self/exe with realpath(Process.executable or cmd[0])
        # (process.cc:124, syscall_emul.hh:1089-1111); the se configs set
        # executable to the workload path.  A path that does not resolve on
        # this host is left unset (that call then escapes as host).
        self.executable = workload if executable is None else executable
        exe = self.executable or self.cmd[0]
        if os.path.exists(exe):
            self.engine.set_exe_path(os.path.realpath(exe))
        # Process.input (Process.py:44; FDArray, fd_array.cc:50-75): the stdio
        # names map to the host's stdin, anything else is opened as a file
        self.input = input
        if input not in ("cin", "stdin"):
            if input == "":
                raise ValueError("input='': gem5 polls fd -1 and retries read(0) forever")
            with open(input, "rb") as f:
                self.engine.set_stdin(f.read())
        self.cpu_type = cpu_type.lower().removesuffix("simplecpu")
        if self.cpu_type not in ("atomic", "timing"):
            raise ValueError(f"cpu_type {cpu_type!r}: 'atomic' or 'timing'")
        self.engine.set_cpu_model(self.cpu_type, timing_params)
        # trials start at once; the translated kernels join when their build lands
        self.golden = self.engine.golden_run(wait_translation=False)
        if self.cpu_type == "timing" and self.engine.tick_info()["status"]:
            raise EngineError(f"cpu_type='timing': {self.engine.tick_info()['status']}")
        self.engine.set_campaign(seed, structures, burst)
        self.bits = bits_mask(bits)
        self.engine.set_bits(self.bits)
        self.engine.set_protect(protect_mask)
        self.protect_opclasses = opclass_mask(protect_opclasses)
        self.engine.set_protect_opclasses(self.protect_opclasses)
        self.shadow_fu_model = shadow_fu_model
        if shadow_fu_model:
            self.engine.set_issue_model({**(issue_params or {}), "priority_to_shadow": int(priority_to_shadow)})
        self._hist = None
        self.outcomes = None

    # PyBindMethod("setProtectMask") analogue of setEnableShrewd (BaseO3CPU.py:69-72)
    def setProtectMask(self, mask: int):
        self.protect_mask = mask
        self.engine.set_protect(mask)

    # PyBindMethod("setProtectOpClasses"): the op-class replication set
    def setProtectOpClasses(self, opclasses):
        self.protect_opclasses = opclass_mask(opclasses)
        self.engine.set_protect_opclasses(self.protect_opclasses)

    def run(self, first_trial: int = 0, n: int | None = None):
        """Run the campaign.  Under torch.distributed with num_gpus > 1 (one
        process per GPU), this rank runs its contiguous shard of the trial ids
        and the outcome histogram is all-reduced; per-trial outcomes stay per
        rank (written to `output` with a `.rankR` suffix)."""
        n = self.trials if n is None else n
        rank, world = 0, 1
        if self.num_gpus > 1:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                rank, world = dist.get_rank(), dist.get_world_size()
        lo, cnt = shard_range(n, world, rank)
        self.first = first_trial + lo
        if self.cpu_type == "timing":
            self.outcomes, self._hist = self.engine.run_tick_trials(self.first, cnt)
        else:
            self.outcomes, self._hist = self.engine.run_trials(self.first, cnt)
        if world > 1:
            import torch
            import torch.distributed as dist
            # RCCL reduces device tensors; other backends (gloo) host ones
            dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else None
            self._hist = allreduce_histogram(self._hist, dev)
        if self.output:
            np.save(self.output if world == 1 else f"{self.output}.rank{rank}", self.outcomes)
        return self.outcomes

    def histogram(self):
        return self._hist

    def summary(self) -> dict:
        h = self._hist
        cls = h["counts"].sum(axis=(0, 1))
        return {"trials": int(h["trials"]), **{CLASS_NAMES[i]: int(cls[i]) for i in range(6)},
                "crash_sub": {CRASH_NAMES.get(i, str(i)): int(h["crash_sub"][i]) for i in range(16)
                              if h["crash_sub"][i]},
                "escape_sub": {ESCAPE_NAMES.get(i, str(i)): int(h["escape_sub"][i]) for i in range(8)
                               if h["escape_sub"][i]},
                "guest_insts": int(h["guest_insts"])}


def softfp(op: int, fmt: int, rm: int, a, b=None, c=None, device: bool = False):
    """The engine's IEEE arithmetic port (csrc/hip/fi_softfp.h) over operand
    vectors, run on the host or on the device -> (result bits, flags)."""
    a = np.ascontiguousarray(a, np.uint64)
    b = np.ascontiguousarray(a if b is None else b, np.uint64)
    c = np.ascontiguousarray(a if c is None else c, np.uint64)
    out = np.zeros(len(a), np.uint64)
    fl = np.zeros(len(a), np.uint32)
    st = lib().fi_debug_softfp(op, fmt, rm, a.ctypes.data, b.ctypes.data, c.ctypes.data, len(a), out.ctypes.data,
                               fl.ctypes.data, 1 if device else 0)
    if st != FI_OK:
        raise EngineError(f"fi_debug_softfp failed ({st})")
    return out, fl


def crypto(fn: int, a, b=None, device: bool = False):
    """The engine's scalar-crypto port (csrc/hip/fi_crypto.h) over operand
    vectors, on the host or on the device -> results (function numbers as in
    fi_crypto.h, RNUM / BS in bits 8+)."""
    a = np.ascontiguousarray(a, np.uint64)
    b = np.ascontiguousarray(a if b is None else b, np.uint64)
    out = np.zeros(len(a), np.uint64)
    st = lib().fi_debug_crypto(fn, a.ctypes.data, b.ctypes.data, len(a), out.ctypes.data, 1 if device else 0)
    if st != FI_OK:
        raise EngineError(f"fi_debug_crypto failed ({st})")
    return out
