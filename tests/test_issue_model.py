"""SHREWD functional-unit contention: the O3 issue model that
decides, per golden instruction, whether its shadow copy found a unit.

CPU tests.  Known answers are derived by hand from the reference's
FUPool::getUnit / InstructionQueue::scheduleReadyInsts / requestShadow
(src/cpu/o3/fu_pool.cc:155-301, inst_queue.cc:830-1181) and the default pool
(FuncUnitConfig.py: 6 IntALU, 2 IntMultDiv, 4 FP_ALU, 2 FP_MultDiv, 4 RdWrPort).
The product's host implementation (fi_issue_model_run in libshrewd_fi.so,
no device needed) and the oracle's independent restatement
(oracle/rv64se.c:or_issue_model) must agree bit for bit on random traces.
"""
import numpy as np
import pytest

from conftest import workload_elf

INTALU, INTMULT, INTDIV, FADD, FMULT, FDIV, FSQRT = 1, 2, 3, 4, 7, 9, 11
MEMREAD, MEMWRITE = 52, 53
PLAIN, LOAD, STORE, SERIAL = 0, 1, 2, 3


def ops_of(rows):
    from oracle.pyoracle import ISSUE_OP_DT
    a = np.zeros(len(rows), ISSUE_OP_DT)
    for i, (cls, src, dst, kind) in enumerate(rows):
        a[i]["opclass"], a[i]["kind"] = cls, kind
        a[i]["src"] = sum(1 << r for r in src)
        a[i]["dst"] = sum(1 << r for r in dst)
    return a


def both(ops, **kw):
    """(shadow, stats) from the oracle and from the product library, asserted equal."""
    from oracle import pyoracle
    from shrewd_amd import fi
    a, sa = pyoracle.issue_model(ops, pyoracle.issue_params(**kw))
    b, sb = fi.issue_model_run(ops, fi.issue_params(**kw))
    bad = np.flatnonzero(a != b)
    assert not len(bad), f"{len(bad)} ops differ, first at {bad[:5].tolist()}"
    for name, _ in pyoracle.IssueStats._fields_:
        va, vb = getattr(sa, name), getattr(sb, name)
        if not isinstance(va, int):
            va, vb = list(va), list(vb)
        assert va == vb, f"stats.{name}: oracle {va} vs product {vb}"
    return a, sa


def test_defaults_match_reference_o3():
    from shrewd_amd import fi
    p = fi.issue_params()
    assert (p.issue_width, p.dispatch_width, p.commit_width, p.iq_entries, p.rob_entries) == (8, 8, 8, 64, 192)
    assert list(p.fu_count) == [6, 2, 4, 2, 4, 1] and p.priority_to_shadow == 0


def test_deferred_shadows_take_leftover_units():
    """8 independent IntAlu ops, deferred mode.  Cycle 1: six primaries take the
    six IntALUs, the 7th finds none (IntAlu skipped for the cycle).  Then the
    shadows: IntALU busy -> FloatAdd (FP_ALU) for 4 of them; the last two find
    neither FloatAdd nor FloatCmp (the same FP_ALU units) -> no shadow.  Cycle
    2: ops 6 and 7 issue and get IntALU shadows."""
    sh, st = both(ops_of([(INTALU, [], [5 + i], PLAIN) for i in range(8)]))
    assert sh.tolist() == [1, 1, 1, 1, 0, 0, 1, 1]
    assert (st.shadow_available, st.shadow_not_available) == (6, 2)
    assert (st.shadow_same_fu, st.shadow_not_same_fu) == (2, 4)
    assert (st.class_available[INTALU], st.class_not_available[INTALU]) == (6, 2)
    assert st.cycles == 3


def test_priority_shadows_take_units_from_younger_primaries():
    """Same ops, priorityToShadow: each issue takes two IntALUs (primary +
    shadow), so 3 ops per cycle issue, every one with a shadow."""
    sh, st = both(ops_of([(INTALU, [], [5 + i], PLAIN) for i in range(8)]), priority_to_shadow=1)
    assert sh.tolist() == [1] * 8
    assert (st.shadow_available, st.shadow_not_available, st.shadow_same_fu) == (8, 0, 8)
    assert st.cycles == 4


def test_unpipelined_divide_shadow_on_float_divider():
    """IntDiv (20 cycles, unpipelined): two divides fill both IntMultDiv units;
    their deferred shadows go to the two FP_MultDiv units (FloatDiv).  The
    third divide waits until cycle 21 and then shadows on the free
    IntMultDiv."""
    sh, st = both(ops_of([(INTDIV, [], [5 + i], PLAIN) for i in range(3)]))
    assert sh.tolist() == [1, 1, 1]
    assert (st.shadow_same_fu, st.shadow_not_same_fu) == (1, 2)
    assert st.cycles == 41   # issue 1 and 21, done 21 and 41


def test_memory_and_no_opclass():
    """MemRead/MemWrite: NoShadowFU (no shadow, not counted).  No_OpClass:
    getUnit(No_OpClass, is_shadow) returns NoCapableFU, which requestShadow
    takes as a shadow (has_shadow = true, counted as available, same FU)."""
    sh, st = both(ops_of([(MEMREAD, [2], [5], LOAD), (MEMWRITE, [2, 5], [], STORE), (0, [], [], PLAIN)]))
    assert sh.tolist() == [0, 0, 1]
    assert (st.shadow_available, st.shadow_not_available, st.shadow_same_fu) == (1, 0, 1)


def test_dependences_serialise_issue():
    """A dependent chain issues one op per cycle: every shadow finds an IntALU."""
    sh, st = both(ops_of([(INTALU, [5], [5], PLAIN)] * 12))
    assert sh.tolist() == [1] * 12 and st.cycles == 13


def test_fewer_alus_starve_shadows():
    """With 2 IntALUs and no FP_ALU, deferred shadows of a 2-wide group find
    nothing; with priority they take the second ALU and halve the issue rate."""
    ops = ops_of([(INTALU, [], [5 + i % 8], PLAIN) for i in range(16)])
    sh, _ = both(ops, IntALU=2, FP_ALU=0)
    assert sh.sum() == 0
    sh, st = both(ops, IntALU=2, FP_ALU=0, priority_to_shadow=1)
    assert sh.sum() == 16 and st.cycles == 17


@pytest.mark.parametrize("seed", range(12))
def test_product_matches_oracle_on_random_traces(seed):
    """Random op mixes (all scalar classes, loads, stores, ecalls, random
    register dataflow) under random widths, queue sizes, pools and modes."""
    rng = np.random.default_rng(seed)
    classes = [0, INTALU, INTALU, INTALU, INTMULT, INTDIV, FADD, 5, 6, FMULT, 8, FDIV, 10, FSQRT, MEMREAD, MEMWRITE,
               54, 55]
    n = 3000
    rows = []
    for _ in range(n):
        c = int(rng.choice(classes))
        kind = LOAD if c in (MEMREAD, 54) else STORE if c in (MEMWRITE, 55) else PLAIN
        if rng.random() < 0.01:
            c, kind = 0, SERIAL
        src = [int(r) for r in rng.integers(1, 33, rng.integers(0, 3))]
        dst = [] if kind == STORE else [int(rng.integers(1, 33))]
        rows.append((c, src, dst, kind))
    ops = ops_of(rows)
    kw = dict(issue_width=int(rng.integers(1, 9)), dispatch_width=int(rng.integers(1, 9)),
              commit_width=int(rng.integers(1, 9)), iq_entries=int(rng.integers(4, 65)),
              rob_entries=int(rng.integers(8, 193)), load_latency=int(rng.integers(1, 6)),
              priority_to_shadow=int(seed % 2),
              fu_count=[int(rng.integers(1, 7)), int(rng.integers(1, 3)), int(rng.integers(0, 5)),
                        int(rng.integers(1, 3)), int(rng.integers(1, 5)), 1])
    sh, st = both(ops, **kw)
    assert st.ops == n and st.cycles >= n // kw["issue_width"]


def test_oracle_trace_of_a_workload():
    """The oracle's golden trace through the model: one entry per committed
    instruction; crc32's IntAlu-dense loop leaves some shadows unissued in
    deferred mode, none with the FU pool doubled."""
    from oracle.pyoracle import Oracle
    o = Oracle(workload_elf("crc32"), "crc32")
    g = o.run_golden()
    o.set_issue_model({})
    sh, st = o.shadow_map()
    assert len(sh) == g.ninst and st.ops >= g.ninst
    assert 0 < st.shadow_not_available and st.class_not_available[INTALU] > 0
    assert st.cycles < g.ninst       # superscalar: IPC > 1
    o.set_issue_model({"IntALU": 12, "FP_ALU": 8})
    sh2, st2 = o.shadow_map()
    assert st2.shadow_not_available == 0 and sh2.sum() >= sh.sum()
    o.close()


def test_oracle_result_faults_under_contention():
    """Result faults on crc32 with IntAlu protected: with the model on, a
    trial is detected only where the target's shadow issued; every other
    protected-target trial runs on as without protection."""
    from oracle.pyoracle import Oracle
    from shrewd_amd.fi import T_RESULT
    o = Oracle(workload_elf("crc32"), "crc32")
    o.run_golden()
    sites = o.sample(0x5EED0007, 0, 3000, 1 << T_RESULT)
    base = o.run_trials(sites, threads=8)
    o.set_protect_opclasses(1 << INTALU)
    always = o.run_trials(sites, threads=8)
    o.set_issue_model({})
    sh, _ = o.shadow_map()
    model = o.run_trials(sites, threads=8)
    det_always = always["cls"] == 4
    det_model = model["cls"] == 4
    assert det_model.sum() < det_always.sum()
    assert not (det_model & ~det_always).any()                  # the model only removes detections
    covered = sh[sites["inst"]] == 1
    assert np.array_equal(det_model, det_always & covered)
    # trials whose shadow did not issue behave exactly as unprotected ones
    lost = det_always & ~covered
    assert lost.any() and np.array_equal(model[lost], base[lost])
    o.set_issue_model(None)
    assert np.array_equal(o.run_trials(sites, threads=8), always)
    o.close()
