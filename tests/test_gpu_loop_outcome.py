"""loop_outcome on the device (fi_trial.hip), the re-check the solo kernel runs
whenever a translated body claims a run-off loop cannot leave before the hang
cap.  The body proves against the instructions left capped at 2^32 - 1
(SoloTxIO::hleft); loop_outcome re-decides against the 64-bit count, so a
loop that leaves after 2^32 + k instructions must come back undecided, not a
hang (gem5: the trial runs on and exits, `BaseCPU::scheduleInstStop`,
cpu/base.cc:764-770, never fires).  Records are synthetic (fi_debug_loop):
no trial has to run billions of instructions to reach those paths.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PAGE_TOP = 0x7FFFFFFFFFFFF000   # the stack's top page (kStackTopVpn): in every page set
BEYOND = 0x8000000000000000     # above kStackBase: unmapped, not in a VMA, not stack growth


def cnt(counter, cmp, step):
    return counter | (cmp << 8) | ((step & 0xFF) << 16)


def ld(reg, kind, size, pos, off=0, span=0):
    return (reg | (kind << 8) | (size << 12) | (pos << 16), off & 0xFFFFFFFF, span)


def loop(regs, left, counter, cmp, step, m, loads=()):
    from shrewd_amd.fi import DEBUG_LOOP_DT
    r = np.zeros(1, DEBUG_LOOP_DT)[0]
    for k, v in regs.items():
        r["regs"][k] = v & (2**64 - 1)
    r["left"], r["lp_cnt"], r["lp_m"], r["lp_n"] = left, cnt(counter, cmp, step), m, len(loads)
    for j, t in enumerate(loads):
        r["lp_ld"][j] = t
    return r


def test_loop_outcome_64bit_left(engine_factory):
    from shrewd_amd.fi import DEBUG_LOOP_DT
    e = engine_factory("hello")
    m = 4
    cases = [
        # 0: leaves after (2^30 + 999) * 4 = 2^32 + 3996 instructions, left 2^33:
        #    the capped body proof fires, the 64-bit re-check says undecided
        (loop({5: 2**30 + 1000}, 2**33, 5, 0, -1, m), 0, 1),
        # 1: the same loop with 2^31 + 5 passes: a hang both ways
        (loop({5: 2**31 + 5}, 2**33, 5, 0, -1, m), 1, 1),
        # 2: a loop that leaves after 2^32 + 4 instructions with left exactly
        #    2^32 + 8: still undecided (the cap is not reached)
        (loop({5: 2**30 + 2}, 2**32 + 8, 5, 0, -1, m), 0, 1),
        # 3: left 2^32 + 3, the loop's last pass at 2^32 + 4: a hang
        (loop({5: 2**30 + 2}, 2**32 + 3, 5, 0, -1, m), 1, 1),
        # 4: a counter compared with x6, distance not a multiple of the step: never leaves
        (loop({5: 3, 6: 0}, 2**40, 5, 6, -2, m), 1, 1),
        # 5: a counter load walking up off the stack's top page: the page fault
        #    512 iterations on, at the first address above kStackBase
        (loop({5: PAGE_TOP, 6: PAGE_TOP + 8 * 2**40}, 2**33, 5, 6, 8, m, [ld(5, 0, 8, 2)]), 2, 1),
        # 6: the same walk downward below the stack: fixupFault would grow the
        #    stack there (mem_state.cc:387-447) -- undecided
        (loop({5: PAGE_TOP, 6: PAGE_TOP - 8 * 2**40}, 2**33, 5, 6, -8, m, [ld(5, 0, 8, 2)]), 0, 1),
        # 7: a bounded (table) load whose range is outside the page set: undecided
        (loop({5: 2**31 + 5, 9: 0x1000}, 2**33, 5, 0, -1, m, [ld(9, 1, 4, 1, 0, 64)]), 0, 1),
        # 8: a counter load that could straddle a line (unaligned): undecided
        (loop({5: PAGE_TOP + 4, 6: PAGE_TOP + 8 * 2**40}, 2**33, 5, 6, 8, m, [ld(5, 0, 8, 0)]), 0, 1),
        # 9: a short loop (100 passes): neither proof fires
        (loop({5: 100}, 2**33, 5, 0, -1, m), 0, 0),
    ]
    recs = np.array([c[0] for c in cases], DEBUG_LOOP_DT)
    out = e.debug_loop_outcome(recs)
    for i, (_, verdict, body) in enumerate(cases):
        assert (int(out["verdict"][i]), int(out["body_proof"][i])) == (verdict, body), (i, out[i])
    # the fault: 512 iterations of 4 instructions, the load third in the block
    assert int(out["k"][5]) == 512 * m + 2 and int(out["fva"][5]) == BEYOND
    # no record with a 64-bit loop shorter than `left` is a hang, whatever the capped proof says
    rng = np.random.default_rng(3)
    many = []
    for _ in range(4000):
        mm = int(rng.integers(1, 64))
        passes = int(rng.integers(2**32 // mm - 4, 2**34 // mm))
        left = int(rng.integers(2**32 - 16, 2**35))
        many.append(loop({5: passes}, left, 5, 0, -1, mm))
    many = np.array(many, DEBUG_LOOP_DT)
    o = e.debug_loop_outcome(many)
    passes = many["regs"][:, 5].astype(np.uint64)
    mm = many["lp_m"].astype(np.uint64)
    left = many["left"].astype(np.uint64)
    hang = (passes - 1) >= (left + mm - 1) // mm
    assert ((o["verdict"] == 1) == hang).all()
    assert (o["verdict"][~hang] == 0).all()
    assert (o["body_proof"].astype(bool) & ~hang).sum() > 100   # the capped proof alone would have been wrong
