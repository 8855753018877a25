"""The load-time translator's loop proofs on the CPU (fi_translate.cpp; no GPU:
fi_debug_translate runs on the host).  Inputs: crc32's pre-decoded text and
golden block trace, as the engine dumps them (tools/gpu/dump_golden.py ->
tests/golden/tx_inputs_{crc32,intmix}.npz, the engine's own output, not
reference data).  The device side of the same proofs is tested against the oracle in
tests/test_gpu_parity.py (test_counted_loop_hang_proofs,
test_runoff_loop_proofs)."""
import ctypes as C
import os
import re

import numpy as np

from conftest import ROOT


def _translate(env=None, name="crc32"):
    from shrewd_amd.fi import lib
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        L = lib()
        L.fi_debug_translate.restype = C.c_int
        z = np.load(os.path.join(ROOT, "tests", "golden", f"tx_inputs_{name}.npz"))
        pre, tr = np.ascontiguousarray(z["pre"]), np.ascontiguousarray(z["trace"])
        n = C.c_uint64()
        L.fi_debug_translate(pre.ctypes.data, len(pre), int(z["text_lo"]), tr.ctypes.data, len(tr), None, 0, C.byref(n))
        buf = C.create_string_buffer(n.value + 1)
        L.fi_debug_translate(pre.ctypes.data, len(pre), int(z["text_lo"]), tr.ctypes.data, len(tr), buf, n.value + 1,
                             C.byref(n))
        return buf.value.decode()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_crc32_loop_proofs():
    body = _translate()
    # the table's inner bit loop (addi t6, t6, -1; bnez t6): a counted loop of
    # three blocks, no memory access -- a hang proof without loads, at every
    # block of the cycle (tested on dispatch entries)
    hang = re.findall(r"TXHANG\(X31, -1, 5u\).*?TXLOOP\((\d+)u, 5u, 0u\)", body)
    assert len(hang) == 3 and all(int(c) & 0xFF == 31 for c in hang)
    assert "goto SR_" not in body
    # the crc loop (lbu t1, 0(a0) ... addi a0, a0, 1; bne a0, a1): a run-off
    # block against a1, a counter load at a0 and a table load at s2 + [0, 1020]
    m = re.search(r"TXHANG\(X10 - X11, 1, 10u\).*?TXLOOP\((\d+)u, 10u, 2u\); TXLD\(0, (\d+)u, (-?\d+), (\d+)u\); "
                  r"TXLD\(1, (\d+)u, (-?\d+), (\d+)u\);", body)
    assert m, "crc loop has no run-off proof"
    cnt, d0, o0, s0, d1, o1, s1 = (int(x) for x in m.groups())
    assert cnt == 10 | 11 << 8 | 1 << 16
    assert (d0 & 0xFF, (d0 >> 8) & 15, (d0 >> 12) & 15, d0 >> 16, o0, s0) == (10, 0, 1, 0, 0, 0)   # lbu at a0
    assert (d1 & 0xFF, (d1 >> 8) & 15, (d1 >> 12) & 15, d1 >> 16, o1, s1) == (18, 1, 4, 5, 0, 1020)   # lwu at s2+
    # the buffer fill: sw t0, 0(t2) walks with t2 (+4 per pass), a store at
    # another induction register (kind 4, the step in the span field)
    m = re.search(r"TXHANG\(X9, -1, 10u\).*?TXLOOP\((\d+)u, 10u, 1u\); TXLD\(0, (\d+)u, (-?\d+), (\d+)u\);", body)
    assert m, "buffer fill has no run-off proof"
    d, o, st = int(m.group(2)), int(m.group(3)), int(m.group(4))
    assert (d & 0xFF, (d >> 8) & 15, (d >> 12) & 15, o, st) == (7, 4, 4, 0, 4)


def test_clean_body_shape():
    """The clean body is generated in one shape (the A/B variants of round 4
    are gone): the budget counts down, the cold hints are on, and the
    translator reads no variant switch from the environment."""
    base = _translate()
    clean = base.split("/*@TX_SPLIT@*/")[-1]
    assert "#define SADD(n_) (brem -= (n_))" in clean and "#define SCOLD(x)" in clean
    assert "SCOLD(" in clean and "SPRIV(x) __builtin_expect" not in clean
    assert _translate({"SHREWD_FI_TXV": "47"}) == base


def test_crc32_loop_estimates():
    """The counted loops the translator exports for the solo order's work-left
    estimate (fi_types.h LoopEst, fi_kernels.hip solo_work_left): the loops
    its hang proofs recognise -- crc32's buffer fill (s1 counts down), table
    inner bit loop (t6 counts down) and crc loop (a0 runs up to a1) -- each
    with its instructions per pass and a text span around its blocks."""
    from shrewd_amd.fi import lib
    L = lib()
    L.fi_debug_loop_est.restype = C.c_int
    L.fi_debug_loop_est.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                    C.POINTER(C.c_uint64)]
    z = np.load(os.path.join(ROOT, "tests", "golden", "tx_inputs_crc32.npz"))
    pre, tr = np.ascontiguousarray(z["pre"]), np.ascontiguousarray(z["trace"])
    dt = np.dtype([("lo", "<u4"), ("hi", "<u4"), ("reg", "u1"), ("treg", "u1"), ("step", "i1"), ("pad", "u1"),
                   ("m", "<u4")])
    n = C.c_uint64()
    assert L.fi_debug_loop_est(pre.ctypes.data, len(pre), int(z["text_lo"]), tr.ctypes.data, len(tr), None, 0,
                               C.byref(n)) == 0
    out = np.zeros(n.value, dt)
    L.fi_debug_loop_est(pre.ctypes.data, len(pre), int(z["text_lo"]), tr.ctypes.data, len(tr), out.ctypes.data,
                        n.value, C.byref(n))
    loops = {(int(r["reg"]), int(r["treg"]), int(r["step"]), int(r["m"])): (int(r["lo"]), int(r["hi"])) for r in out}
    assert (10, 11, 1, 10) in loops     # crc_loop: lbu .. addi a0, a0, 1; bne a0, a1
    assert (31, 0, -1, 5) in loops      # tbl_inner: addi t6, t6, -1; bnez t6 (shortest pass: 5)
    # the buffer fill (gen: sw t0, 0(t2); addi t2, t2, 4; addi s1, s1, -1;
    # bnez s1): its store walks with the pointer t2, an induction register of
    # its own (round 6: run-off proofs with stores)
    assert (9, 0, -1, 10) in loops and len(loops) == 3
    lo, hi = loops[(10, 11, 1, 10)]
    assert lo == 0x16C and hi == 0x16C + 0x22   # the crc loop's one block (pc 0x1016c, 34 bytes)


def test_clean_body_temporaries_at_function_scope():
    """The clean body declares no block-scope temporaries (a goto out of such
    a block leaves through clang's lifetime cleanup switch: DESIGN.md 4h);
    solo_tx_clean_run declares them (TX_TEMPS)."""
    clean = _translate().split("/*@TX_SPLIT@*/")[-1]
    for decl in ("uint8_t *p_;", "bool pv_;", "uint64_t v_;", "const uint64_t ea_", "const uint64_t e_ ",
                 "const uint64_t t_ ", "const uint64_t off_"):
        assert decl not in clean, decl
    assert "ea_ = X10 + " in clean
    src = open(os.path.join(ROOT, "shrewd_amd", "csrc", "hip", "fi_trial.hip")).read()
    fn = src[src.index("void solo_tx_clean_run("):src.index("/*@TX_SOLO_CLEAN@*/")]
    assert "TX_TEMPS();" in fn


def test_intmix_region_proof():
    """intmix's main loop (loop: ... call popcnt ... sd t3, 0(t2) ... skip:
    addi s2, s2, 1; bltu s2, s3, loop) is a region proof (round 6,
    fi_translate.cpp): it runs while s2 < s3, s2 grows by one per pass, the
    pass calls a leaf (popcnt, its own counted inner loop) and reads / writes
    the acc table at s1 + [0, 4088] and pctab at s0 + [0, 255] -- bounded
    accesses at registers the region never writes (kinds 1 and 5).  The
    shortest pass (callee included) is 30 instructions; the test sits at the
    loop's own blocks only (the callee's are shared with its other callers)."""
    body = _translate(name="intmix")
    clean = body.split("/*@TX_SPLIT@*/")[-1]
    tests = re.findall(r"case (\d+): if \(TXHANGU\(X18, X19, 1, 30u\)\).*?TXLOOP\((\d+)u, 30u, 3u\); "
                       r"TXLD\(0, (\d+)u, 0, 4088u\); TXLD\(1, (\d+)u, 0, 4088u\); TXLD\(2, (\d+)u, 0, 255u\);", clean)
    assert len(tests) == 4, tests
    for _, lp, d0, d1, d2 in tests:
        assert int(lp) == 18 | 19 << 8 | 1 << 16 | 1 << 24
        assert [(int(d) & 0xFF, (int(d) >> 8) & 15, (int(d) >> 12) & 15) for d in (d0, d1, d2)] == [(9, 1, 8), (9, 5, 8), (8, 1, 1)]
    assert "TXHANGU" not in body.split("/*@TX_SPLIT@*/")[1]   # the full solo body has no proofs
