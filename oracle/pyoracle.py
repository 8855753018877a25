"""ctypes binding of the oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product (shrewd_amd/) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "librv64se.so")

OUTCOME_DT = np.dtype([("cls", "u1"), ("sub", "u1"), ("exit_code", "u1"), ("flags", "u1"),
                       ("detail", "<u4"), ("ninst", "<u8")])
SITE_DT = np.dtype([("inst", "<u8"), ("mask", "<u8"), ("addr", "<u8"), ("target", "<u4"), ("trial", "<u4")])


class Golden(C.Structure):
    _fields_ = [("ninst", C.c_uint64), ("ncycles", C.c_uint64), ("exit_code", C.c_uint32), ("cls", C.c_uint32),
                ("stdout_len", C.c_uint64), ("stderr_len", C.c_uint64),
                ("fetch_bytes", C.c_uint64), ("data_bytes", C.c_uint64)]


class Probe(C.Structure):
    _fields_ = [("rd_value", C.c_uint64), ("npc", C.c_uint64), ("fault", C.c_int32), ("rd", C.c_int32),
                ("len", C.c_uint32), ("op", C.c_uint32)]


class IssueParams(C.Structure):
    _fields_ = [("issue_width", C.c_uint32), ("dispatch_width", C.c_uint32), ("commit_width", C.c_uint32),
                ("iq_entries", C.c_uint32), ("rob_entries", C.c_uint32), ("load_latency", C.c_uint32),
                ("priority_to_shadow", C.c_uint32), ("fu_count", C.c_uint32 * 6)]


class IssueStats(C.Structure):
    _fields_ = [("ops", C.c_uint64), ("cycles", C.c_uint64), ("shadow_available", C.c_uint64),
                ("shadow_not_available", C.c_uint64), ("shadow_same_fu", C.c_uint64),
                ("shadow_not_same_fu", C.c_uint64), ("class_available", C.c_uint64 * 12),
                ("class_not_available", C.c_uint64 * 12)]


ISSUE_OP_DT = np.dtype([("src", "<u8"), ("dst", "<u8"), ("opclass", "u1"), ("kind", "u1"), ("pad", "u1", (6,))])
# tick-domain injection (timing_se.h; layouts == include/fi_engine.h fi_timing_*)
TIMING_OP_DT = np.dtype([("fetch", "<u8", (2,)), ("addr", "<u8", (2,)), ("size", "<u2", (2,)), ("nfetch", "u1"),
                         ("nfrag", "u1"), ("kind", "u1"), ("cmd", "u1"), ("pad", "u1", (8,))])
TIMING_TICKS_DT = np.dtype([("fetch_send", "<u8", (2,)), ("fetch_done", "<u8", (2,)), ("exec", "<u8"),
                            ("done", "<u8")])
TICK_SITE_DT = np.dtype([("tick", "<u8"), ("mask", "<u8"), ("target", "<u4"), ("trial", "<u4")])


class TimingParams(C.Structure):
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


def timing_params(**kw) -> TimingParams:
    """The reference board's timing parameters (timing_se.c), with overrides."""
    p = TimingParams()
    lib().or_timing_default_params(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, int(v))
    return p


def timing_model(ops: np.ndarray, params: TimingParams | None = None):
    """or_timing_model -> (ticks TIMING_TICKS_DT[n], TimingStats)"""
    ops = np.ascontiguousarray(ops, TIMING_OP_DT)
    out = np.zeros(len(ops), TIMING_TICKS_DT)
    st = TimingStats()
    if lib().or_timing_model(ops.ctypes.data, len(ops), C.byref(params or timing_params()), out.ctypes.data,
                             C.byref(st)) != 0:
        raise RuntimeError("or_timing_model: rejected")
    return out, st
FU_NAMES = ("IntALU", "IntMultDiv", "FP_ALU", "FP_MultDiv", "RdWrPort", "IprPort")


def issue_params(**kw) -> IssueParams:
    """The reference's O3 defaults (o3/BaseO3CPU.py:127-194, FuncUnitConfig.py)
    plus a 2-cycle load; overrides by field name or FU name."""
    p = IssueParams(8, 8, 8, 64, 192, 2, 0)
    for i, c in enumerate((6, 2, 4, 2, 4, 1)):
        p.fu_count[i] = c
    for k, v in kw.items():
        if k in FU_NAMES:
            p.fu_count[FU_NAMES.index(k)] = int(v)
        elif k == "fu_count":
            for i, c in enumerate(v):
                p.fu_count[i] = int(c)
        else:
            setattr(p, k, int(v))
    return p


def issue_model(ops: np.ndarray, params: IssueParams | None = None):
    """or_issue_model -> (shadow uint8[n], IssueStats)"""
    ops = np.ascontiguousarray(ops, ISSUE_OP_DT)
    out = np.zeros(len(ops), np.uint8)
    st = IssueStats()
    if lib().or_issue_model(ops.ctypes.data, len(ops), C.byref(params or issue_params()), out.ctypes.data,
                            C.byref(st)) != 0:
        raise RuntimeError("or_issue_model: bad parameters")
    return out, st


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.or_create_checkpoint.restype = C.c_void_p
        L.or_create_checkpoint.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t]
        L.or_write_checkpoint.argtypes = [C.c_void_p, C.c_uint64, C.c_char_p]
        L.or_create.restype = C.c_void_p
        L.or_create.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p]
        L.or_destroy.argtypes = [C.c_void_p]
        L.or_error.restype = C.c_char_p
        L.or_error.argtypes = [C.c_void_p]
        L.or_golden.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(Golden)]
        L.or_golden_stdout.restype = C.c_uint64
        L.or_golden_stdout.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64]
        L.or_golden_stderr.restype = C.c_uint64
        L.or_golden_stderr.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64]
        L.or_sample.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint64,
                                C.c_void_p]
        L.or_run_trials.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p, C.c_int]
        L.or_run_one_capture.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p,
                                         C.c_char_p, C.c_uint64, C.POINTER(C.c_uint64)]
        L.or_probe.argtypes = [C.c_uint32, C.c_uint64, C.c_void_p, C.POINTER(Probe)]
        L.or_mnemonic.restype = C.c_char_p
        L.or_mnemonic.argtypes = [C.c_uint32]
        L.or_sys_class.argtypes = [C.c_int]
        L.or_set_protect_opclasses.argtypes = [C.c_void_p, C.c_uint64]
        L.or_set_clock.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64]
        L.or_set_exe_path.argtypes = [C.c_void_p, C.c_char_p]
        L.or_set_stdin.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64]
        L.or_issue_model.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(IssueParams), C.c_void_p,
                                     C.POINTER(IssueStats)]
        L.or_set_issue_model.argtypes = [C.c_void_p, C.POINTER(IssueParams)]
        L.or_golden_ops.restype = C.c_uint64
        L.or_golden_ops.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
        L.or_shadow_map.restype = C.c_uint64
        L.or_shadow_map.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(IssueStats)]
        L.or_rvk.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
        L.or_timing_default_params.argtypes = [C.c_void_p]
        L.or_timing_model.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_tick_setup.argtypes = [C.c_void_p, C.c_void_p]
        L.or_tick_golden_ticks.restype = C.c_uint64
        L.or_tick_golden_ticks.argtypes = [C.c_void_p]
        L.or_tick_trace.restype = C.c_uint64
        L.or_tick_trace.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
        L.or_tick_sample.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32,
                                     C.c_uint64, C.c_void_p]
        L.or_run_tick_trials.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p,
                                         C.c_int]
        L.or_sf_ref.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                C.c_void_p, C.c_void_p]
        _lib = L
    return _lib


class Oracle:
    def __init__(self, elf: bytes, argv0: str, checkpoint: str | None = None):
        """A campaign from process start (cmd = [argv0]) or, with checkpoint,
        from a gem5 SE checkpoint directory."""
        self.L = lib()
        if checkpoint is not None:
            self.h = self.L.or_create_checkpoint(checkpoint.encode(), elf, len(elf))
        else:
            self.h = self.L.or_create(elf, len(elf), argv0.encode())
        err = self.L.or_error(self.h).decode()
        if err:
            raise RuntimeError(err)
        self.golden = None

    def close(self):
        if self.h:
            self.L.or_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def write_checkpoint(self, ninst: int, directory: str):
        """The golden run's state at numInst == ninst as a gem5 SE checkpoint."""
        if self.L.or_write_checkpoint(self.h, ninst, directory.encode()) != 0:
            raise RuntimeError(self.L.or_error(self.h).decode())

    def set_protect_opclasses(self, mask: int):
        """SHREWD replication set: bit k = gem5 OpClass enum value k."""
        self.L.or_set_protect_opclasses(self.h, mask)

    def set_issue_model(self, params: IssueParams | dict | None = None, **kw):
        """SHREWD FU contention for result faults; None and no keywords: off."""
        if params is None and not kw:
            self.L.or_set_issue_model(self.h, None)
            return
        p = params if isinstance(params, IssueParams) else issue_params(**{**(params or {}), **kw})
        if self.L.or_set_issue_model(self.h, C.byref(p)) != 0:
            raise RuntimeError(self.L.or_error(self.h).decode())

    def golden_ops(self) -> np.ndarray:
        """The golden trace as ISSUE_OP_DT records (register reads / writes)."""
        n = self.L.or_golden_ops(self.h, None, 0)
        out = np.zeros(n, ISSUE_OP_DT)
        self.L.or_golden_ops(self.h, out.ctypes.data, n)
        return out

    def shadow_map(self):
        n = self.L.or_shadow_map(self.h, None, 0, None)
        out = np.zeros(n, np.uint8)
        st = IssueStats()
        self.L.or_shadow_map(self.h, out.ctypes.data, n, C.byref(st))
        return out, st

    def run_golden(self, max_inst=1 << 32) -> Golden:
        g = Golden()
        if self.L.or_golden(self.h, max_inst, C.byref(g)) != 0:
            raise RuntimeError(self.L.or_error(self.h).decode())
        self.golden = g
        return g

    def golden_stdout(self) -> bytes:
        n = self.L.or_golden_stdout(self.h, None, 0)
        buf = C.create_string_buffer(max(n, 1))
        self.L.or_golden_stdout(self.h, buf, n)
        return buf.raw[:n]

    def golden_stderr(self) -> bytes:
        n = self.L.or_golden_stderr(self.h, None, 0)
        buf = C.create_string_buffer(max(n, 1))
        self.L.or_golden_stderr(self.h, buf, n)
        return buf.raw[:n]

    def sample(self, seed, first, n, structures, burst=1, bits=2**64 - 1) -> np.ndarray:
        sites = np.zeros(n, SITE_DT)
        if self.L.or_sample(self.h, seed, first, n, structures, burst, bits & (2**64 - 1), sites.ctypes.data) != 0:
            raise RuntimeError(self.L.or_error(self.h).decode())
        return sites

    def run_trials(self, sites: np.ndarray, protect_mask=0, hang_x16=0, threads=None) -> np.ndarray:
        sites = np.ascontiguousarray(sites, SITE_DT)
        out = np.zeros(len(sites), OUTCOME_DT)
        threads = threads or os.cpu_count() or 1
        if self.L.or_run_trials(self.h, sites.ctypes.data, len(sites), protect_mask, hang_x16,
                                out.ctypes.data, threads) != 0:
            raise RuntimeError(self.L.or_error(self.h).decode())
        return out

    def set_exe_path(self, path: str):
        """What readlinkat("/proc/self/exe") answers (realpath of the executable)."""
        self.L.or_set_exe_path(self.h, path.encode())

    def set_stdin(self, data: bytes | None):
        """Process.input: the bytes of the input file (None = "cin", host stdin)."""
        if self.L.or_set_stdin(self.h, data, 0 if data is None else len(data)) != 0:
            raise MemoryError("or_set_stdin")

    def set_clock(self, period_ticks=500, random_seed=5489):
        self.L.or_set_clock(self.h, period_ticks, random_seed)

    # ---- tick-domain injection under TimingSimpleCPU (rv64se.h)
    def tick_setup(self, params: TimingParams | None = None) -> int:
        """Record the golden run's requests and run the timing model; returns
        the golden run's length in ticks."""
        if self.L.or_tick_setup(self.h, C.byref(params) if params is not None else None) != 0:
            raise RuntimeError(self.L.or_error(self.h).decode())
        return int(self.L.or_tick_golden_ticks(self.h))

    def tick_trace(self):
        """(ops TIMING_OP_DT, ticks TIMING_TICKS_DT) of the golden run's attempts."""
        n = self.L.or_tick_trace(self.h, None, None, 0)
        ops = np.zeros(n, TIMING_OP_DT)
        ticks = np.zeros(n, TIMING_TICKS_DT)
        self.L.or_tick_trace(self.h, ops.ctypes.data, ticks.ctypes.data, n)
        return ops, ticks

    def tick_sample(self, seed, first, n, structures, burst=1, bits=2**64 - 1) -> np.ndarray:
        out = np.zeros(n, TICK_SITE_DT)
        if self.L.or_tick_sample(self.h, seed, first, n, structures, burst, bits & (2**64 - 1),
                                 out.ctypes.data) != 0:
            raise RuntimeError(self.L.or_error(self.h).decode())
        return out

    def run_tick_trials(self, sites: np.ndarray, hang_x16=0, threads=None, truth=False):
        """-> outcomes (the contract's escapes reported, not run), or
        (outcomes, literal outcomes of every trial) with truth=True"""
        sites = np.ascontiguousarray(sites, TICK_SITE_DT)
        out = np.zeros(len(sites), OUTCOME_DT)
        tr = np.zeros(len(sites), OUTCOME_DT) if truth else None
        threads = threads or os.cpu_count() or 1
        if self.L.or_run_tick_trials(self.h, sites.ctypes.data, len(sites), hang_x16, out.ctypes.data,
                                     tr.ctypes.data if truth else None, threads) != 0:
            raise RuntimeError(self.L.or_error(self.h).decode())
        return (out, tr) if truth else out

    def run_one(self, site=None, protect_mask=0, hang_x16=0):
        out = np.zeros(1, OUTCOME_DT)
        buf = C.create_string_buffer(1 << 16)
        n = C.c_uint64()
        sp = None
        if site is not None:
            s = np.ascontiguousarray(np.array([site], SITE_DT))
            sp = s.ctypes.data
        self.L.or_run_one_capture(self.h, sp, protect_mask, hang_x16, out.ctypes.data, buf, 1 << 16, C.byref(n))
        return out[0], buf.raw[:min(n.value, 1 << 16)]


def probe(inst: int, pc: int, regs) -> Probe:
    r = (C.c_uint64 * 32)(*[int(x) & (2**64 - 1) for x in regs])
    p = Probe()
    lib().or_probe(inst & 0xFFFFFFFF, pc, r, C.byref(p))
    return p


def mnemonic(inst: int) -> str:
    return lib().or_mnemonic(inst & 0xFFFFFFFF).decode()


def sys_class(num: int) -> int:
    return lib().or_sys_class(num)


def has_softfloat() -> bool:
    """The reference SoftFloat (oracle/_ref) is linked: F/D/Zfh arithmetic executes."""
    return bool(lib().or_has_softfloat())


def sf_ref(op: int, fmt: int, rm: int, a, b=None, c=None):
    """The reference SoftFloat over operand vectors -> (result bits, flags)."""
    a = np.ascontiguousarray(a, np.uint64)
    b = np.ascontiguousarray(a if b is None else b, np.uint64)
    c = np.ascontiguousarray(a if c is None else c, np.uint64)
    out = np.zeros(len(a), np.uint64)
    fl = np.zeros(len(a), np.uint32)
    lib().or_sf_ref(op, fmt, rm, a.ctypes.data, b.ctypes.data, c.ctypes.data, len(a), out.ctypes.data, fl.ctypes.data)
    return out, fl


def has_rvk() -> bool:
    """The reference's scalar-crypto helpers (oracle/_ref) are linked: Zkn/Zks execute."""
    return bool(lib().or_has_rvk())


def rvk_ref(fn: int, a, b=None):
    """The reference's rvk.hh over operand vectors (fi_crypto.h function numbers)."""
    a = np.ascontiguousarray(a, np.uint64)
    b = np.ascontiguousarray(a if b is None else b, np.uint64)
    out = np.zeros(len(a), np.uint64)
    lib().or_rvk(fn, a.ctypes.data, b.ctypes.data, len(a), out.ctypes.data)
    return out
