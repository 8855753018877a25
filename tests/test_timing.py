"""Tick-domain injection under TimingSimpleCPU, CPU side.

Two restatements of the reference board's timing (TimingSimpleCPU on a NoCache
SystemXBar with SingleChannelDDR3_1600 at 3 GHz, the SE run script's
CPUTypes.TIMING configuration): the product's fi_timing_model_run
(shrewd_amd/csrc/fi_timing.cpp, host code in the engine library) and the
oracle's or_timing_model (oracle/timing_se.c).  They must give the same tick
for every event of every request list; hand-derived ticks pin the latency
chain.  The oracle's tick-domain trials (a flip applied inside the attempt in
flight, rv64se.c tk_*) are checked against its own numInst trials where the
two must agree.  Against a live gem5: parity unpinned (no SCons here).
"""
import numpy as np
import pytest

from conftest import workload_elf

REGS_PC = ((1 << 32) - 2) | (1 << 32)
T_PC, T_RESULT = 32, 34


def rand_ops(rng, n, span):
    from shrewd_amd.fi import TIMING_OP_DT
    ops = np.zeros(n, TIMING_OP_DT)
    for i in range(n):
        o = ops[i]
        pc = int(rng.integers(0, span)) * 4
        if rng.random() < 0.15:
            o["nfetch"] = 2
            o["fetch"] = (pc, pc + 4)
        else:
            o["nfetch"] = 1
            o["fetch"][0] = pc
        r = rng.random()
        if i == n - 1:
            o["kind"] = 2
        elif r < 0.05:
            o["kind"] = 1
        elif r < 0.55:
            a = int(rng.integers(0, span * 4))
            sz = int(rng.choice([1, 2, 4, 8, 64]))
            if sz == 64:
                a &= ~63
            o["cmd"] = int(rng.choice([0, 0, 1, 1, 2, 3, 4]))
            if a // 64 != (a + sz - 1) // 64:
                s0 = (a // 64 + 1) * 64 - a
                o["nfrag"] = 2
                o["addr"] = (a, a + s0)
                o["size"] = (s0, sz - s0)
            else:
                o["nfrag"] = 1
                o["addr"][0] = a
                o["size"][0] = sz
    return ops


@pytest.mark.parametrize("variant", ["board", "refresh", "small_queues", "narrow_xbar"])
def test_timing_models_agree_on_random_requests(oracle_mod, variant):
    """Product and oracle restatements: every tick of every attempt equal, over
    random request lists (straddles, split accesses, faults, every command)
    and stressed parameters (frequent refresh; 8-entry write / 4-entry read
    queues; an 8-byte crossbar so writes occupy the layer for cycles)."""
    from shrewd_amd.fi import timing_model_run, timing_params
    kw = {"board": {}, "refresh": {"tREFI": 400000, "tRFC": 100000},
          "small_queues": {"write_buffer": 8, "read_buffer": 4}, "narrow_xbar": {"xbar_width": 8}}[variant]
    rng = np.random.default_rng(["board", "refresh", "small_queues", "narrow_xbar"].index(variant) + 11)
    seen = {}
    for it in range(40):
        span = int(rng.choice([64, 4096, 1 << 16, 1 << 22]))
        ops = rand_ops(rng, int(rng.integers(2, 2500)), span)
        pt, ps = timing_model_run(ops, timing_params(**kw))
        ot, os_ = oracle_mod.timing_model(ops, oracle_mod.timing_params(**kw))
        assert (pt == ot).all(), (variant, it, int(np.nonzero(pt != ot)[0][0]))
        assert ps.as_dict() == {n: getattr(os_, n) for n, _ in os_._fields_}
        for k, v in ps.as_dict().items():
            seen[k] = seen.get(k, 0) + v
    # the paths these lists reach
    assert seen["write_queue_hits"] and seen["activates"] and seen["writes"]
    if variant == "refresh":
        assert seen["refreshes"] > 100
    if variant in ("board", "narrow_xbar"):
        assert seen["xbar_retries"]


def test_timing_hand_derived_ticks():
    """The latency chain, derived by hand from the reference code (1 tick = 1 ps,
    CPU / crossbar clock 333 ticks):
      fetch 0 sent at 0; crossbar header = 0 (edge) + (3 + 4) x 333 + 333
        (snoop filter) = 2664; DRAM: row closed -> ACT at 0, RD at max(tRCD
        13750, nextBurstAt = tRP + tRCD = 27500) = 27500, ready 27500 + tCL
        13750 + tBURST 5000 = 46250; response 46250 + 10 + 10 ns + 2664 =
        68914; crossbar: next edge 68931 + 2 x 333 -> 69597 = completeIfetch.
      fetch 1 (row hit) sent at 69597: RD at 69597, ready 88347, response
        111011, edge 111222 + 666 -> 111888.
      load 0x2000 (bank 1: ACT at 111888, RD at 125638), ready 144388,
        response 167052, edge 167166 + 666 -> 167832.
      store 0x2000 at 210123: accepted at once, response 210123 + 10 ns +
        2664 + 333 (one 64-byte beat) = 223120, edge 223443 + 666 -> 224109."""
    from shrewd_amd.fi import TIMING_OP_DT, timing_model_run
    ops = np.zeros(4, TIMING_OP_DT)
    ops["nfetch"] = 1
    ops["fetch"][:, 0] = [0x0, 0x4, 0x8, 0xc]
    ops[1]["nfrag"], ops[1]["addr"][0], ops[1]["size"][0], ops[1]["cmd"] = 1, 0x2000, 8, 0
    ops[2]["nfrag"], ops[2]["addr"][0], ops[2]["size"][0], ops[2]["cmd"] = 1, 0x2000, 8, 1
    ops[3]["kind"] = 2
    t, st = timing_model_run(ops)
    assert t["exec"][0] == 69597
    assert t["fetch_send"][1][0] == 69597 and t["exec"][1] == 111888 and t["done"][1] == 167832
    assert t["exec"][2] == 210123 and t["done"][2] == 224109
    assert t["fetch_send"][3][0] == 224109 and st.ticks == t["exec"][3]


def test_timing_model_rejects_malformed_lists():
    from shrewd_amd.fi import TIMING_OP_DT, EngineError, timing_model_run
    ops = np.zeros(2, TIMING_OP_DT)
    ops["nfetch"] = 1
    with pytest.raises(EngineError):   # no FI_TOP_END at the end
        timing_model_run(ops)
    ops[1]["kind"] = 2
    ops[0]["nfrag"], ops[0]["addr"][0], ops[0]["size"][0] = 1, 60, 8   # a fragment across a burst
    with pytest.raises(EngineError):
        timing_model_run(ops)


@pytest.mark.parametrize("name", ["hello", "crc32", "qsort"])
def test_golden_requests_time_the_same(oracle_mod, name):
    """The oracle's golden request list (recorded by its own interpreter, frames
    in SE allocation order) timed by both models: equal ticks; the attempts
    are the AtomicSimpleCPU ticks less the second fetches."""
    from shrewd_amd.fi import timing_model_run
    o = oracle_mod.Oracle(workload_elf(name), name)
    g = o.run_golden()
    T = o.tick_setup()
    ops, ticks = o.tick_trace()
    assert len(ops) + int((ops["nfetch"] == 2).sum()) == g.ncycles
    assert ops["kind"][-1] == 2 and T == ticks["exec"][-1]
    pt, _ = timing_model_run(ops)
    assert (pt == ticks).all()
    # monotone: every attempt starts when the previous one completes
    assert (ticks["fetch_send"][1:, 0] == ticks["done"][:-1]).all()
    o.close()


def _tick_setup(oracle_mod, name):
    o = oracle_mod.Oracle(workload_elf(name), name)
    o.run_golden()
    o.tick_setup()
    return o


def test_literal_tick_flips_match_numinst_injection(oracle_mod):
    """The oracle's literal tick injection against its own numInst injection,
    where gem5's mechanics make them one machine: a register flipped while an
    instruction is fetched (no ecall / retry before it) = the numInst flip at
    that instruction; flipped while a load's data is outstanding = the numInst
    flip after it, or nothing if the load writes that register."""
    o = _tick_setup(oracle_mod, "crc32")
    ops, ticks = o.tick_trace()
    rng = np.random.default_rng(7)
    commit = np.nonzero(ops["kind"] == 0)[0]
    n_before = np.cumsum(np.concatenate([[0], (ops["kind"][:-1] == 0).astype(np.int64)]))
    sites, num = [], []
    for j in rng.choice(commit[1:-1], 300, replace=False):
        r = int(rng.integers(1, 32))
        b = int(rng.integers(0, 64))
        start = int(ticks["done"][j - 1]) + 1
        if ops["kind"][j - 1] != 0:
            continue
        sites.append((start, 1 << b, r, len(sites)))
        num.append((int(n_before[j]), 1 << b, 0, r, len(num)))
    ts = np.array(sites, oracle_mod.TICK_SITE_DT)
    ns = np.array(num, oracle_mod.SITE_DT)
    a = o.run_tick_trials(ts, threads=8)
    b = o.run_trials(ns, threads=8)
    assert (a == b).all()
    o.close()


def test_literal_data_phase_flips(oracle_mod):
    """Flips while a load's data access is outstanding: the destination is
    overwritten by the completion (the golden outcome); another register acts
    from the next instruction on."""
    o = _tick_setup(oracle_mod, "qsort")
    ops, ticks = o.tick_trace()
    g = o.golden
    gops = o.golden_ops()          # one per committed instruction and ecall
    assert len(gops) == len(ops)   # (qsort takes no page-fault retries)
    n_before = np.cumsum(np.concatenate([[0], (ops["kind"][:-1] == 0).astype(np.int64)]))
    loads = np.nonzero((ops["kind"] == 0) & (ops["nfrag"] > 0) & (ops["cmd"] == 0))[0]
    dst_sites, use_sites, num = [], [], []
    for j in loads[::max(1, len(loads) // 400)]:
        d = int(gops["dst"][j]) & 0xFFFFFFFE
        s = int(gops["src"][j + 1]) & 0xFFFFFFFE & ~d
        if bin(d).count("1") != 1 or not s:
            continue
        rd, rs = d.bit_length() - 1, s.bit_length() - 1
        t = int(ticks["done"][j])
        dst_sites.append((t, 1 << 40, rd, len(dst_sites)))
        use_sites.append((t, 1 << 40, rs, len(use_sites)))
        num.append((int(n_before[j]) + 1, 1 << 40, 0, rs, len(num)))
    assert len(num) > 200
    lit_d = o.run_tick_trials(np.array(dst_sites, oracle_mod.TICK_SITE_DT), threads=8)
    lit_u = o.run_tick_trials(np.array(use_sites, oracle_mod.TICK_SITE_DT), threads=8)
    ref_u = o.run_trials(np.array(num, oracle_mod.SITE_DT), threads=8)
    # the destination: the completion overwrote the flip -> the golden run
    assert ((lit_d["cls"] == 0) & (lit_d["ninst"] == g.ninst)).all()
    # a register the next instruction reads: the numInst flip after the load
    assert (lit_u == ref_u).all()
    assert (ref_u["cls"] != 0).sum() > 20
    o.close()


@pytest.mark.parametrize("name", ["crc32", "qsort"])
def test_tick_campaign_escapes_are_rare(oracle_mod, name):
    """Every FI_ESC_TIMING in a register + pc + result campaign names a
    contract reason, and they are a small share."""
    o = _tick_setup(oracle_mod, name)
    s = o.tick_sample(0x5EED0002, 0, 3000, REGS_PC | (1 << T_RESULT))
    out = o.run_tick_trials(s, threads=8)
    esc = (out["cls"] == 5) & (out["sub"] == 7)
    assert esc.mean() < 0.02
    assert set(out["exit_code"][esc].tolist()) <= set(range(1, 9))
    assert esc.any() and (out["cls"] == 1).any() and (out["cls"] == 0).any()
    o.close()


def test_tick_setup_refuses_clock_readers(oracle_mod):
    """A golden run that reads curTick prints another value under
    TimingSimpleCPU: the tick model refuses it."""
    from test_isa_vectors import clk_program_elf
    o = oracle_mod.Oracle(clk_program_elf(), "clk")
    o.run_golden()
    with pytest.raises(RuntimeError, match="curTick"):
        o.tick_setup()
    o.close()


def test_tick_sites_lie_inside_the_run(oracle_mod):
    o = _tick_setup(oracle_mod, "hello")
    T = oracle_mod.Oracle.tick_setup(o)
    bad = np.array([(T, 1, 5, 0)], oracle_mod.TICK_SITE_DT)
    with pytest.raises(RuntimeError, match="ends at"):
        o.run_tick_trials(bad)
    ok = o.run_tick_trials(np.array([(T - 1, 1, 5, 0)], oracle_mod.TICK_SITE_DT))
    assert ok["cls"][0] == 0
    o.close()
