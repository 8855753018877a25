"""GPU parity: the HIP engine against the oracle, through the C ABI.

Bar: bit-exact per-trial outcomes (class, sub-code, exit code, flags, detail,
committed-instruction count) on the same seeded sites.
"""
import os

import re

import numpy as np
import pytest

from conftest import ROOT, WORKLOADS, workload_elf

pytestmark = pytest.mark.gpu

REGS = (1 << 32) - 2
PC = 1 << 32
MEM = 1 << 33


def oracle_for(oracle_mod, name, argv0=None):
    o = oracle_mod.Oracle(workload_elf(name), argv0 or name)
    o.run_golden()
    return o


def compare(dev, ref, sites):
    bad = np.nonzero(dev != ref)[0]
    if len(bad):
        i = bad[0]
        raise AssertionError(f"{len(bad)} of {len(sites)} outcomes differ; first: site={sites[i]} "
                             f"gpu={dev[i]} oracle={ref[i]}")


def test_decode_parity_compressed(engine_factory, oracle_mod):
    e = engine_factory("hello")
    raws = np.arange(0x10000, dtype=np.uint32)
    raws = raws[(raws & 3) != 3]
    d = e.debug_decode(raws)
    names = [oracle_mod.mnemonic(int(r)) for r in raws]
    _check_decode(d, raws, names, oracle_mod)


def test_decode_parity_32bit(engine_factory, oracle_mod):
    e = engine_factory("hello")
    rng = np.random.default_rng(1)
    raws = (rng.integers(0, 2**32, 200000, dtype=np.uint64).astype(np.uint32) | 3)
    d = e.debug_decode(raws)
    names = [oracle_mod.mnemonic(int(r)) for r in raws]
    _check_decode(d, raws, names, oracle_mod)


def test_decode_parity_gem5_vectors(engine_factory, oracle_mod):
    """Device decoder against the oracle on every word of the gem5-decoder
    fixture (the oracle itself is checked against it in test_oracle.py)."""
    from test_oracle import load_decode_vectors
    raws = load_decode_vectors()[0]
    e = engine_factory("hello")
    d = e.debug_decode(raws)
    for i in range(len(raws)):
        p = oracle_mod.probe(int(raws[i]), 0x10000, [0] * 32)
        assert (d["op"][i], d["len"][i]) == (p.op, p.len), (hex(int(raws[i])), oracle_mod.mnemonic(int(raws[i])))
        if p.rd > 0:   # an FP destination is reported as 32 + f
            assert d["rd"][i] == p.rd % 32, hex(int(raws[i]))


def _check_decode(d, raws, names, oracle_mod):
    # device op ids share the oracle's op list order; compare through the
    # oracle probe (op id, rd, len) for every encoding
    for i in range(0, len(raws), max(1, len(raws) // 20000)):
        p = oracle_mod.probe(int(raws[i]), 0x10000, [0] * 32)
        assert d["op"][i] == p.op, (hex(int(raws[i])), names[i], int(d["op"][i]), p.op)
        assert d["len"][i] == p.len
        if p.rd > 0:   # an FP destination is reported as 32 + f
            assert d["rd"][i] == p.rd % 32, (hex(int(raws[i])), names[i])


@pytest.mark.parametrize("name", WORKLOADS)
def test_golden_run_matches_oracle(engine_factory, oracle_mod, name):
    e = engine_factory(name)
    o = oracle_for(oracle_mod, name)
    g, og = e.golden, o.golden
    assert (g.ninst, g.ncycles, g.exit_code) == (og.ninst, og.ncycles, og.exit_code)
    assert e.golden_stdout() == o.golden_stdout()


@pytest.mark.parametrize("name", ["crc32", "qsort"])
def test_sampler_matches_oracle(engine_factory, oracle_mod, name):
    e = engine_factory(name)
    o = oracle_for(oracle_mod, name)
    for structs, burst in ((REGS | PC, 1), (MEM, 1), (MEM, 4), (REGS | PC | MEM, 8)):
        e.set_campaign(0xABCDEF, structs, burst)
        dev = e.sample(1000, 3000)
        ref = o.sample(0xABCDEF, 1000, 3000, structs, burst)
        assert np.array_equal(dev, ref)
    # the `bits` parameter (eligible lowest flipped bits)
    from shrewd_amd.fi import bits_mask
    for spec, burst in (("0-7,40,63", 1), ("10-20", 2), (0x8000000000000001, 1)):
        e.set_campaign(0xABCDEF, REGS | PC | MEM, burst)
        e.set_bits(bits_mask(spec))
        dev = e.sample(0, 3000)
        ref = o.sample(0xABCDEF, 0, 3000, REGS | PC | MEM, burst, bits_mask(spec))
        assert np.array_equal(dev, ref), spec


@pytest.mark.parametrize("name,structs,burst,n", [
    ("hello", REGS | PC, 1, 1000),        # C1: 1k regfile flips
    ("crc32", REGS | PC, 1, 6000),        # C2 (sampled)
    ("qsort", REGS | PC, 1, 6000),        # C2 (sampled)
    ("crc32", MEM, 1, 3000),              # C4 memory words
    ("qsort", MEM, 4, 3000),              # C4 bursts
    ("qsort", REGS | PC | MEM, 8, 2000),
    ("intmix", REGS | PC, 1, 5000),       # C3 kernel (sampled)
    ("fpamo", REGS | PC | MEM, 1, 4000),  # F/D data movement + AMOs (the golden run has FP state)
    ("fpamo", REGS | PC, 3, 2000),
])
def test_trials_bit_exact(engine_factory, oracle_mod, name, structs, burst, n):
    e = engine_factory(name)
    o = oracle_for(oracle_mod, name)
    e.set_campaign(0x5EED0001 + n, structs, burst)
    e.set_protect(0)
    sites = e.sample(0, n)
    dev, hist = e.run_sites(sites)
    ref = o.run_trials(sites, protect_mask=0)
    compare(dev, ref, sites)
    assert int(hist["trials"]) == n
    assert int(hist["counts"].sum()) == n


def test_rewritten_code_bit_exact(engine_factory, oracle_mod):
    """Trials whose stores land in the text (a flipped pointer in crc32's fill
    loop): pre-decoded and translated code stay in use for every instruction
    whose bytes the lane did not rewrite; the rewritten ones decode from the
    lane's own pages."""
    e = engine_factory("crc32")
    o = oracle_for(oracle_mod, "crc32")
    e.set_campaign(0x5EED0003, REGS | PC, 1)
    sites = e.sample(0, 100_000)
    sites = sites[(sites["target"] == 7) | (sites["target"] == 8)][:4000]   # t2 / s0: the fill loop's pointers
    dev, _ = e.run_sites(sites)
    ref = o.run_trials(sites)
    compare(dev, ref, sites)


S_REGS = (1 << 8) | (1 << 9) | sum(1 << r for r in range(18, 28))     # s0-s11
T_REGS = (1 << 5) | (1 << 6) | (1 << 7) | sum(1 << r for r in range(28, 32))   # t0-t6


@pytest.mark.parametrize("mask", [0, (1 << 1) | (1 << 2) | (1 << 3) | (1 << 4),
                                  sum(1 << r for r in range(10, 18)), S_REGS, T_REGS,
                                  (1 << 32) - 2 | (1 << 32)])
def test_protect_mask_bit_exact(engine_factory, oracle_mod, mask):
    """C5: selective-replication sweep -- detected-by-replica classification."""
    e = engine_factory("crc32")
    o = oracle_for(oracle_mod, "crc32")
    e.set_campaign(99, REGS | PC, 1)
    e.set_protect(mask)
    sites = e.sample(0, 3000)
    dev, hist = e.run_sites(sites)
    ref = o.run_trials(sites, protect_mask=mask)
    e.set_protect(0)
    compare(dev, ref, sites)
    if mask:
        assert (dev["cls"] == 4).sum() > 0


RESULT = 1 << 34
OPC_INT = (1 << 1) | (1 << 2) | (1 << 3)        # IntAlu | IntMult | IntDiv (gem5 OpClass enum)


@pytest.mark.parametrize("name,opc,n", [
    ("hello", 0, 500), ("crc32", 0, 4000), ("crc32", OPC_INT, 4000), ("qsort", 1 << 1, 3000),
    ("intmix", (1 << 1) | (1 << 2), 600), ("fpamo", OPC_INT | (1 << 6) | (1 << 10), 2000),
])
def test_result_faults_bit_exact(engine_factory, oracle_mod, name, opc, n):
    """Result faults (structure 34) and SHREWD replication by OpClass: the
    first instruction committing at the inject time has its x[rd] value
    flipped, or is detected when its class is protected and has a shadow FU."""
    e = engine_factory(name)
    o = oracle_for(oracle_mod, name)
    e.set_campaign(0xFACE + n, RESULT | REGS, 1)
    e.set_protect_opclasses(opc)
    o.set_protect_opclasses(opc)
    sites = e.sample(0, n)
    dev, _ = e.run_sites(sites)
    ref = o.run_trials(sites)
    e.set_protect_opclasses(0)
    compare(dev, ref, sites)
    if opc and name != "hello":
        assert (dev["cls"] == 4).sum() > 0


@pytest.mark.parametrize("name", ["crc32", "qsort", "intmix", "fpamo"])
@pytest.mark.parametrize("prio", [0, 1])
def test_shadow_map_matches_oracle(engine_factory, oracle_mod, name, prio):
    """SHREWD FU contention: the engine's issue model over the device-recorded
    golden trace equals the oracle's over its own golden run, per committed
    instruction and in every counter."""
    e = engine_factory(name)
    o = oracle_for(oracle_mod, name)
    e.set_issue_model(priority_to_shadow=prio)
    o.set_issue_model(priority_to_shadow=prio)
    a, sa = e.shadow_map()
    b, sb = o.shadow_map()
    e.set_issue_model(None)
    assert len(a) == e.golden.ninst
    bad = np.flatnonzero(a != b)
    assert not len(bad), f"{len(bad)} instructions differ, first {bad[:5].tolist()}"
    for f, _ in oracle_mod.IssueStats._fields_:
        va, vb = getattr(sa, f), getattr(sb, f)
        assert (list(va) if not isinstance(va, int) else va) == (list(vb) if not isinstance(vb, int) else vb), f


@pytest.mark.parametrize("name,opc,n", [("crc32", OPC_INT, 6000), ("qsort", 1 << 1, 4000),
                                        ("intmix", OPC_INT, 3000)])
def test_result_faults_under_contention_bit_exact(engine_factory, oracle_mod, name, opc, n):
    """Result faults with the FU-contention model on (deferred shadows): a
    protected instruction is detected only if its shadow found a unit."""
    e = engine_factory(name)
    o = oracle_for(oracle_mod, name)
    e.set_campaign(0xC0DE + n, RESULT, 1)
    e.set_protect_opclasses(opc)
    o.set_protect_opclasses(opc)
    e.set_issue_model({})
    o.set_issue_model({})
    sites = e.sample(0, n)
    dev, _ = e.run_sites(sites)
    ref = o.run_trials(sites)
    sh, _ = e.shadow_map()
    e.set_issue_model(None)
    e.set_protect_opclasses(0)
    compare(dev, ref, sites)
    det = dev["cls"] == 4
    assert det.any() and not (det & (sh[sites["inst"]] == 0)).any()


@pytest.mark.parametrize("name", ["hello", "crc32", "qsort", "intmix", "fpamo"])
def test_golden_register_accesses_match_oracle(engine_factory, oracle_mod, name):
    """The integer registers every golden instruction and ecall reads and
    writes -- the inputs of register liveness, first-access forwarding and the
    issue model -- equal the oracle's, event by event."""
    e = engine_factory(name)
    o = oracle_for(oracle_mod, name)
    pre, tr, _ = e.debug_golden_trace()
    ops = o.golden_ops()
    assert len(tr) == len(ops) > 0
    rec = pre[tr & 0x7FFFFFFF]
    rd, rs1, rs2, fl = (rec[:, k].astype(np.uint64) for k in (5, 6, 7, 13))
    one = np.uint64(1)
    src = (np.where((fl & 4) != 0, one << rs1, 0) | np.where((fl & 8) != 0, one << rs2, 0)).astype(np.uint64)
    dst = np.where((fl & 16) != 0, one << rd, 0).astype(np.uint64)
    ecall = (tr & 0x80000000) != 0
    src[ecall], dst[ecall] = 0x3FC00, 1 << 10
    m = np.uint64(0xFFFFFFFE)
    bad = np.flatnonzero(((src & m) != (ops["src"] & m)) | ((dst & m) != (ops["dst"] & m)))
    assert not len(bad), f"{len(bad)} events differ, first {bad[:5].tolist()}"


@pytest.mark.parametrize("name", ["crc32", "qsort", "intmix"])
def test_first_access_forwarding(engine_factory, oracle_mod, name):
    """Register sites are injected at the golden run's next access of the
    register (dead ones end at injection): outcomes equal the oracle's and
    the unforwarded engine's."""
    e = engine_factory(name)
    f = engine_factory(name, flags=512)
    o = oracle_for(oracle_mod, name)
    for x in (e, f):
        x.set_campaign(0xF0A0, REGS, 1)
    sites = e.sample(0, 3000)
    dev, _ = e.run_sites(sites)
    dead = int(e.debug_stats()[27])
    ref, _ = f.run_sites(sites)
    assert int(f.debug_stats()[27]) == 0 and dead > 0
    compare(dev, ref, sites)
    compare(dev, o.run_trials(sites), sites)


def test_translation_skipped_without_hot_code(engine_factory):
    """Straight-line code run once (hello) is not translated: the static
    kernels run it, and the engine says why."""
    e = engine_factory("hello")
    assert e.translate_status().startswith("nothing to translate")
    assert e.golden.translated_blocks == 0


@pytest.mark.parametrize("name", ["crc32", "qsort", "intmix"])
def test_translated_path_active(engine_factory, name):
    """The load-time translated kernel (fi_trial_kernel_tx) is built and runs:
    a hipRTC failure would otherwise fall back to the static kernel silently."""
    e = engine_factory(name)
    assert e.translate_status() == "", e.translate_status()
    assert e.golden.translated_blocks > 0 and e.golden.translated_insts > 0
    e.set_campaign(0x7A11, REGS | PC, 1)
    e.run_trials(0, 2000)
    st = e.debug_stats()
    assert int(st[16]) > 0 and int(st[17]) > 0   # translated instructions, block entries


def test_dead_memory_faults_end_at_injection(engine_factory, oracle_mod):
    """A memory fault on bytes the golden run never reads again before writing
    them ends at injection as the golden run (the golden run's access index,
    fi_trial.hip:mem_dead); the outcomes still equal the oracle's full runs,
    and the shortcut is really taken."""
    e = engine_factory("crc32")
    o = oracle_for(oracle_mod, "crc32")
    e.set_campaign(0x5EED0D0D, MEM, 2)
    sites = e.sample(0, 4000)
    dev, _ = e.run_sites(sites)
    assert int(e.debug_stats()[26]) > 1000
    compare(dev, o.run_trials(sites), sites)


PATH_FLAGS = {
    "default": 0,
    "no_translate": 4,                      # FI_CFG_NO_TRANSLATE: interpreter only
    "from_start": 1 | 2 | 16384,            # FI_CFG_NO_SNAPSHOT_START | NO_EARLY_EXIT | NO_HANG_PROOF
    "no_epochs": 8,                         # FI_CFG_NO_EPOCHS
    "pack_runs": 16,                        # FI_CFG_PACK_RUNS
    "fixed_resume": 32,                     # FI_CFG_FIXED_RESUME
    "no_solo": 64,                          # FI_CFG_NO_SOLO: resumed epochs on the 64-lane kernel
    "solo_all": 128,                        # FI_CFG_SOLO_ALL: every epoch on the one-trial-per-wave kernel
    "solo_all_interp": 128 | 4,             # the solo build without translated blocks
    "simt": 256,                            # FI_CFG_SIMT: diverged lanes step together, per lane
    "no_forward": 512,                      # FI_CFG_NO_FORWARD: inject at the sampled time
    "no_sdc_exit": 1024,                    # FI_CFG_NO_SDC_EXIT: SDC trials run to their end
    "simt_no_solo_interp": 256 | 64 | 4,    # the step loop for every epoch, no translated blocks
    "no_odd_kernel": 4096,                  # FI_CFG_NO_ODD_KERNEL: odd-pc survivors on the solo kernel
    "no_redo": 2048,                        # FI_CFG_NO_REDO: no second pass for private-page exhaustion
    "no_loop_order": 65536,                 # FI_CFG_NO_LOOP_ORDER: solo order by the golden remainder only
}
_PATH_REF = {}


@pytest.mark.parametrize("name", ["crc32", "qsort", "intmix", "crcblk"])
@pytest.mark.parametrize("path", list(PATH_FLAGS))
def test_execution_paths_bit_exact(engine_factory, oracle_mod, name, path):
    """Every execution path of the engine (translated blocks, pre-decoded and
    general interpreter, snapshot start + early exit, epochs and the resume
    packings) gives the oracle's outcomes on the same sites."""
    n = 3000
    e = engine_factory(name, flags=PATH_FLAGS[path], max_trials_per_launch=n)
    if PATH_FLAGS[path] & 4:
        assert e.translate_status().startswith("disabled")
    e.set_campaign(0x5EED0BAD, REGS | PC | MEM, 1)
    e.set_protect(0)
    sites = e.sample(0, n)
    if name not in _PATH_REF:
        o = oracle_for(oracle_mod, name)
        _PATH_REF[name] = (sites, o.run_trials(sites, protect_mask=0))
    rsites, ref = _PATH_REF[name]
    assert np.array_equal(sites, rsites)
    dev, hist = e.run_sites(sites)
    compare(dev, ref, sites)
    assert int(hist["device_insts"]) <= int(hist["guest_insts"])
    if PATH_FLAGS[path] & 1:   # from process start, no early exit, no hang proofs: the device runs every instruction
        assert int(hist["device_insts"]) == int(hist["guest_insts"])


def test_counted_loop_hang_proofs(engine_factory, oracle_mod):
    """(And the run-off loop proofs: see below.)  crc32's t6 flips loop in the table's inner bit loop (a counted loop:
    addi t6, t6, -1; bnez t6) until the hang cap.  The clean translated body
    proves those hangs when it enters the loop (fi_translate.cpp): the records
    equal a run without the proofs (FI_CFG_NO_HANG_PROOF: every hang runs to
    the cap) and the oracle's, with fewer instructions executed."""
    from shrewd_amd.fi import CFG_NO_HANG_PROOF
    n = 20000
    on = engine_factory("crc32", max_trials_per_launch=n)
    off = engine_factory("crc32", flags=CFG_NO_HANG_PROOF, max_trials_per_launch=n)
    for e in (on, off):
        e.set_campaign(0x5EED0002, REGS | PC, 1)
        e.set_protect(0)
    a, ha = on.run_trials(0, n)
    proved, crashed = int(on.debug_stats()[56]), int(on.debug_stats()[57])
    b, hb = off.run_trials(0, n)
    assert int(off.debug_stats()[56]) == 0 and int(off.debug_stats()[57]) == 0
    assert np.array_equal(a, b)
    hang = np.nonzero(a["cls"] == 3)[0]
    assert len(hang) > 20 and proved > 0 and proved <= len(hang)
    assert (a["detail"][hang] == 0).all()
    # the crc loop's end-pointer (a1) flips run off the buffer: page-fault
    # crashes proved at the loop's entry (run-off loop proofs)
    crash = np.nonzero((a["cls"] == 2) & (a["sub"] == 3))[0]
    assert crashed > 20 and crashed <= len(crash)
    assert int(ha["device_insts"]) < int(hb["device_insts"])
    sel = np.concatenate([hang, crash])
    sites = on.sample(0, n)[sel]
    compare(a[sel], oracle_for(oracle_mod, "crc32").run_trials(sites), sites)


# tail trials of the 1M-trial north-star campaigns (seed 0x5EED0003, found by
# tools/gpu/launch_size.py): loops no translated block covers -- floating-point
# loads and arithmetic in rewritten code with silent stores (qsort 805936,
# 127484, 735672), a return into its own epilogue (373107), an RVV no-op in a
# data page (775944), a no-effect M5 op in rewritten code (953708), and
# `jal x4, 0` in a data page (intmix 990675, 682623)
DYN_LOOP_TRIALS = {"qsort": [805936, 127484, 735672, 373107, 775944, 953708], "intmix": [990675, 682623]}


@pytest.mark.parametrize("name", ["qsort", "intmix"])
def test_dynamic_loop_proofs(engine_factory, oracle_mod, name):
    """Dynamic loop proofs (fi_trial.hip LoopProbe / lp_prove):
    a trial looping in the interpreters is single-stepped through one pass of
    its loop and proved to repeat forever.  Every such trial is a hang whose
    record equals the oracle's (which runs it to the cap) and the engine's
    own without proofs (FI_CFG_NO_HANG_PROOF), and the proofs fired
    (stats[59]) with far fewer instructions executed."""
    from shrewd_amd.fi import CFG_NO_HANG_PROOF
    ids = DYN_LOOP_TRIALS[name]
    on = engine_factory(name, flags=128, max_trials_per_launch=4096)            # FI_CFG_SOLO_ALL
    off = engine_factory(name, flags=128 | CFG_NO_HANG_PROOF, max_trials_per_launch=4096)
    for e in (on, off):
        e.set_campaign(0x5EED0003, REGS | PC, 1)
        e.set_protect(0)
    sites = on.sample(0, max(ids) + 1)[ids]
    a, ha = on.run_sites(sites)
    proved = int(on.debug_stats()[59])
    b, hb = off.run_sites(sites)
    assert int(off.debug_stats()[59]) == 0
    assert np.array_equal(a, b)
    assert (a["cls"] == 3).all() and (a["detail"] == 0).all()
    assert proved >= len(ids) - 1
    assert int(ha["device_insts"]) * 5 < int(hb["device_insts"])
    compare(a, oracle_for(oracle_mod, name).run_trials(sites), sites)
    # and inside a normal campaign (the 64-lane epoch first): same records as without proofs
    n = 20000
    on2 = engine_factory(name, max_trials_per_launch=n)
    off2 = engine_factory(name, flags=CFG_NO_HANG_PROOF, max_trials_per_launch=n)
    for e in (on2, off2):
        e.set_campaign(0x5EED0003, REGS | PC, 1)
        e.set_protect(0)
    c, _ = on2.run_trials(0, n)
    d, _ = off2.run_trials(0, n)
    assert np.array_equal(c, d)


def test_runoff_loop_proofs(oracle_mod):
    """Run-off loops (fi_translate.cpp, fi_trial.hip loop_outcome): faults on
    the scan pointer / end of the runoff program's three scan loops.  Trials
    that walk off a .bss buffer or below the text end as page-fault crashes
    proved at the loop's entry (stats[57]); those that walk into heap pages
    the fault handler would map stay undecided (stats[58]) and run on.  Every
    record equals the oracle's, with the proofs on and off."""
    from shrewd_amd import Engine
    from shrewd_amd.fi import CFG_NO_HANG_PROOF
    import test_isa_vectors as kat
    elf = kat.runoff_program_elf()
    o = oracle_mod.Oracle(elf, "runoff")
    g = o.run_golden()
    sites = kat.runoff_sites(g.ninst, 3000)
    ref = o.run_trials(sites, protect_mask=0)
    got = []
    for flags in (0, CFG_NO_HANG_PROOF):
        e = Engine(flags=flags)
        e.load_elf(elf, ["runoff"])
        e.golden_run()
        dev, h = e.run_sites(sites)
        assert e.translate_status() == ""
        compare(dev, ref, sites)
        st = e.debug_stats()
        got.append((int(st[57]), int(st[58]), int(h["device_insts"])))
        e.close()
    (crash_on, und_on, ins_on), (crash_off, und_off, ins_off) = got
    assert crash_on > 10 and und_on > 0 and crash_off == 0 and und_off == 0
    assert ins_on < ins_off


def test_storeoff_loop_proofs(oracle_mod):
    """Run-off loops that store at their counter (round 6: fi_translate.cpp
    kind 2, fi_trial.hip loop_outcome): store walks off a .bss buffer end as
    page-fault crashes proved at the loop's entry (stats[57]); walks that
    could reach the code range or go into heap pages the fault handler maps
    stay undecided (stats[58]) and run on.  Every record equals the oracle's
    (reference semantics: mem_state.cc:387-447, sim/faults.cc:95-105), with
    the proofs on and off."""
    from shrewd_amd import Engine
    from shrewd_amd.fi import CFG_NO_HANG_PROOF
    import test_isa_vectors as kat
    elf = kat.storeoff_program_elf()
    o = oracle_mod.Oracle(elf, "storeoff")
    g = o.run_golden()
    sites = kat.storeoff_sites(g.ninst, 3000)
    ref = o.run_trials(sites, protect_mask=0)
    got = []
    for flags in (0, CFG_NO_HANG_PROOF):
        e = Engine(flags=flags)
        e.load_elf(elf, ["storeoff"])
        e.golden_run()
        dev, h = e.run_sites(sites)
        assert e.translate_status() == ""
        if flags == 0:   # proofs for counter stores (kind 2) and induction-pointer stores / loads (4 / 3)
            kinds = {(int(d) >> 8) & 15 for d in re.findall(r"TXLD\(\d+, (\d+)u", e.debug_translation())}
            assert {0, 2, 3, 4} <= kinds, kinds
        compare(dev, ref, sites)
        st = e.debug_stats()
        got.append((int(st[57]), int(st[58]), int(h["device_insts"])))
        e.close()
    (crash_on, und_on, ins_on), (crash_off, und_off, ins_off) = got
    assert crash_on > 10 and und_on > 0 and crash_off == 0 and und_off == 0
    assert ins_on < ins_off


def test_region_loop_proofs(engine_factory, oracle_mod):
    """intmix's loop bound s3 flipped high: the main loop (a call and table
    stores per pass) runs to the hang cap.  The region proof (fi_translate.cpp,
    fi_trial.hip loop_outcome: bounded accesses, kinds 1 / 5) ends those
    trials as hangs at their next dispatch entry into the loop (stats[56]);
    every record equals the oracle's, with the proofs on and off."""
    from oracle.pyoracle import SITE_DT
    from shrewd_amd.fi import CFG_NO_HANG_PROOF
    o = oracle_for(oracle_mod, "intmix")
    g = o.run_golden()
    r = np.random.default_rng(21)
    n = 256
    s = np.zeros(n, SITE_DT)
    s["inst"] = r.integers(1000, g.ninst - 1000, n)
    s["mask"] = np.uint64(1) << r.integers(0, 64, n).astype(np.uint64)
    s["target"] = 19
    s["trial"] = np.arange(n)
    ref = o.run_trials(s, protect_mask=0)
    got = []
    for flags in (0, CFG_NO_HANG_PROOF):
        e = engine_factory("intmix", flags=flags)
        dev, h = e.run_sites(s)
        compare(dev, ref, s)
        got.append((int(e.debug_stats()[56]), int(h["device_insts"])))
    (hang_on, ins_on), (hang_off, ins_off) = got
    assert (ref["cls"] == 3).sum() > 50
    assert hang_on > 20 and hang_off == 0 and ins_on < ins_off // 2, got


def test_run_trials_equals_run_sites(engine_factory):
    e = engine_factory("crc32")
    e.set_campaign(4242, REGS | PC, 1)
    out1, h1 = e.run_trials(100, 5000)
    sites = e.sample(100, 5000)
    out2, h2 = e.run_sites(sites)
    assert np.array_equal(out1, out2)
    assert np.array_equal(h1["counts"], h2["counts"])


def test_chunking_invariance(engine_factory):
    """Launch size must not change any outcome (shard invariance).  Chunks
    are pipelined with no host wait between them (fi_engine.cpp run_chunks):
    a chunk's second pass (resource escapes: crc32 with P = 1 and no
    overflow pool) runs after the next chunk's first,
    from its own sites buffer -- the outcomes, the histogram and its totals
    equal a one-launch run's, on the host path and the device path."""
    small = engine_factory("qsort", max_trials_per_launch=1000)
    big = engine_factory("qsort")
    for e in (small, big):
        e.set_campaign(77, REGS | PC | MEM, 2)
    a, ha = small.run_trials(0, 5000)
    b, hb = big.run_trials(0, 5000)
    assert np.array_equal(a, b)
    assert np.array_equal(ha["counts"], hb["counts"])
    from shrewd_amd.fi import CFG_NO_OVERFLOW
    redo = [engine_factory("crc32", max_trials_per_launch=m, private_pages=1, flags=CFG_NO_OVERFLOW)
            for m in (1000, 3000)]
    outs = []
    for e in redo:
        e.set_campaign(77, REGS | PC | MEM, 2)
        o, h = e.run_trials(0, 3000)
        assert int(e.debug_stats()[30]) > 0, "no resource escape to redo"
        outs.append((o, h))
    assert np.array_equal(outs[0][0], outs[1][0])
    for f in ("counts", "crash_sub", "escape_sub", "trials", "guest_insts"):
        assert np.array_equal(outs[0][1][f], outs[1][1][f]), f
    ref = engine_factory("crc32")
    ref.set_campaign(77, REGS | PC | MEM, 2)
    assert np.array_equal(outs[0][0], ref.run_trials(0, 3000)[0])
    assert int(outs[0][1]["trials"]) == 3000 and int(outs[0][1]["guest_insts"]) == int(outs[0][0]["ninst"].sum())
    # the device path (bench.py's): chunked outcomes land in place
    import torch
    from shrewd_amd import HIST_DT
    d_out = torch.zeros(3000 * a.dtype.itemsize, dtype=torch.uint8, device="cuda")
    d_hist = torch.zeros(HIST_DT.itemsize, dtype=torch.uint8, device="cuda")
    redo[0].run_trials_device(0, 3000, d_out.data_ptr(), d_hist.data_ptr())
    redo[0].sync()
    dev = np.frombuffer(d_out.cpu().numpy().tobytes(), dtype=a.dtype)
    hd = np.frombuffer(d_hist.cpu().numpy().tobytes(), dtype=HIST_DT)[0]
    assert np.array_equal(dev, outs[0][0])
    for f in ("counts", "crash_sub", "escape_sub", "trials", "guest_insts"):
        assert np.array_equal(hd[f], outs[0][1][f]), f


def test_argv_shapes_stack(engine_factory, oracle_mod):
    """argv[0] length moves sp (argsInit); golden + trials still agree."""
    e = engine_factory("crc32", argv0="/some/much/longer/path/to/crc32")
    o = oracle_for(oracle_mod, "crc32", "/some/much/longer/path/to/crc32")
    e.set_campaign(5, REGS | PC | MEM, 1)
    sites = e.sample(0, 2000)
    dev, _ = e.run_sites(sites)
    compare(dev, o.run_trials(sites), sites)


def test_full_size_properties(engine_factory):
    """C2 at full size (100k trials): size-independent properties."""
    e = engine_factory("crc32")
    e.set_campaign(0x5EED0002, REGS | PC, 1)
    out, h = e.run_trials(0, 100_000)
    g = e.golden
    assert int(h["trials"]) == 100_000
    assert int(h["guest_insts"]) == int(out["ninst"].sum())
    cls = np.bincount(out["cls"], minlength=6)
    assert cls[0] > 50_000 and cls[2] > 0
    masked = out[out["cls"] == 0]
    assert (masked["exit_code"] == g.exit_code).all()
    # flips of x0..: the PC-flip crash share is large, register flips mostly masked
    out2, _ = e.run_trials(0, 100_000)
    assert np.array_equal(out, out2)   # deterministic


def test_native_driver_matches_engine(engine_factory, tmp_path):
    """src/campaign (the FaultCampaign SimObject's core) over the C ABI gives the
    same per-trial outcomes and histogram as the Python binding, with one
    engine and with two engines on device 0 (--devices 0,0: the in-process
    multi-device path, one host thread per engine, histograms summed on the
    host); its JSON summary names every class and sub-code as the Python
    mirror's summary() does."""
    import json
    import subprocess
    from shrewd_amd import HIST_DT, OUTCOME_DT
    from shrewd_amd import build as b
    from shrewd_amd.fi import CLASS_NAMES, CRASH_NAMES, ESCAPE_NAMES
    exe = b.build_cli()
    n, seed = 3000, 0x5EED0003
    e = engine_factory("crc32")
    e.set_campaign(seed, (1 << 34) - 2, 1)
    e.set_protect(0)
    ref, rh = e.run_trials(0, n)
    for devices in ("0", "0,0"):
        prefix = str(tmp_path / f"camp{devices.count(',')}")
        r = subprocess.run([exe, "--workload", os.path.join(ROOT, "workloads", "crc32.elf"), "--cmd", "crc32",
                            "--trials", str(n), "--seed", hex(seed), "--structures", "int_reg,pc,mem",
                            "--devices", devices, "--output", prefix], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        out = np.fromfile(prefix + ".outcomes.bin", OUTCOME_DT)
        hist = np.fromfile(prefix + ".hist.bin", HIST_DT)[0]
        assert out.tobytes() == ref.tobytes()
        assert hist["counts"].tobytes() == rh["counts"].tobytes()
        js = json.loads(r.stdout)
        assert js["num_gpus"] == devices.count(",") + 1
        cls = rh["counts"].sum(axis=(0, 1))
        assert {c: js[c] for c in CLASS_NAMES} == {CLASS_NAMES[i]: int(cls[i]) for i in range(6)}
        assert js["crash_sub"] == {CRASH_NAMES[i]: int(rh["crash_sub"][i]) for i in range(16) if rh["crash_sub"][i]}
        assert js["escape_sub"] == {ESCAPE_NAMES[i]: int(rh["escape_sub"][i]) for i in range(8) if rh["escape_sub"][i]}


@pytest.mark.parametrize("prog", ["alu", "mem", "cmp", "rvc", "sys", "lrsc", "vm", "fp", "rnd", "xop", "sys2", "clk",
                                  "stdin", "vset", "vcfg"])
def test_known_answer_programs(oracle_mod, prog):
    """Known answers on the device (guest programs of tests/test_isa_vectors.py).

    alu: every M/shift/bit-manipulation/Zicond op on every vector pair.
    mem: sb/sh/sw/sd then all seven loads at misaligned, 64-byte-line-crossing
    and page-crossing offsets.
    cmp: slt/sltu/slti/sltiu and the six branches (data-dependent, so the
    translated code diverges and merges).
    rvc: the compressed (RVC + Zcb) register forms.
    sys: the modelled syscalls (get*id, write to stdout/stderr/bad fd,
    an ignored call, exit status & 0xff).
    lrsc: LR/SC reservations and lock records.
    vm: brk / mmap / munmap / set_tid_address / ioctl / getrlimit / prlimit64 /
    uname / writev / close (the SE memory map).
    fp: F/D/Zfh arithmetic in every rounding mode with fflags, the dynamic
    rounding mode and fcsr (answers from the reference SoftFloat).
    rnd: getrandom (gem5's mt19937_64 stream) and clock_gettime (curTick).
    clk: clock_gettime after a branch whose arms differ only in ticks.
    stdin: read / write / writev of fd 0 with Process.input a file.
    xop: scalar crypto, Zfa (fli / fround / fcvtmod.w.d), M5 pseudo-ops, the
    warn-only privileged no-ops and the cache-block ops.
    sys2: read, readlinkat (/proc/self/exe) and riscv_hwprobe.
    vset: vset* with illegal vtype requests from the start vector state.
    vcfg: vset* chains through legal vector configurations (AVL, VLMAX, the
    kept vl of x0, x0, uint32_t AVL truncation, vsetvl's vill bit).  The device golden run (general interpreter)
    must print exactly the reference-derived models; no-fault trials
    (pre-decoded and translated paths, from snapshots) must end masked with
    the oracle's records; faulted trials must match the oracle bit for bit."""
    from shrewd_amd import Engine
    import test_isa_vectors as kat
    elf, expected = {"alu": (kat.program_elf, kat.program_expected),
                     "mem": (kat.mem_program_elf, kat.mem_program_expected),
                     "cmp": (kat.cmp_program_elf, kat.cmp_program_expected),
                     "rvc": (kat.rvc_program_elf, kat.rvc_program_expected),
                     "sys": (kat.sys_program_elf, kat.sys_program_expected),
                     "lrsc": (kat.lrsc_program_elf, kat.lrsc_program_expected),
                     "vm": (kat.vm_program_elf, kat.vm_program_expected),
                     "fp": (kat.fp_program_elf, kat.fp_program_expected),
                     "rnd": (kat.rnd_program_elf, kat.rnd_program_expected),
                     "xop": (kat.xop_program_elf, kat.xop_program_expected),
                     "sys2": (kat.sys2_program_elf, kat.sys2_program_expected),
                     "clk": (kat.clk_program_elf, kat.clk_program_expected),
                     "stdin": (kat.stdin_program_elf, kat.stdin_program_expected),
                     "vset": (kat.vset_program_elf, kat.vset_program_expected),
                     "vcfg": (kat.vcfg_program_elf, kat.vcfg_program_expected)}[prog]
    if prog in ("fp", "xop") and not oracle_mod.has_softfloat():
        pytest.skip("oracle without the reference SoftFloat")
    if prog == "xop" and not oracle_mod.has_rvk():
        pytest.skip("oracle without the reference rvk.hh")
    stderr = {"sys": kat.SYS_STDERR, "vm": kat.VM_STDERR}.get(prog, b"")
    elf, expected = elf(), expected()
    e = Engine(private_pages=64)
    e.load_elf(elf, [prog])
    if prog == "sys2":
        e.set_exe_path(kat.SYS2_EXE)
    if prog == "stdin":
        e.set_stdin(kat.STDIN_DATA)
    g = e.golden_run()
    assert g.exit_code == (300 & 0xFF if prog == "sys" else 0)
    assert g.stderr_len == len(stderr)
    assert e.golden_stdout() == expected
    assert e.golden_stderr() == stderr
    o = oracle_mod.Oracle(elf, prog)
    if prog == "sys2":
        o.set_exe_path(kat.SYS2_EXE)
    if prog == "stdin":
        o.set_stdin(kat.STDIN_DATA)
    o.run_golden()
    assert o.golden_stderr() == e.golden_stderr()
    e.set_campaign(0x5EED00A1, REGS | PC, 1)
    e.set_protect(0)
    sites = e.sample(0, 3000)
    nofault = sites[:512].copy()
    nofault["inst"] = 1 << 40
    dev, _ = e.run_sites(nofault)
    compare(dev, o.run_trials(nofault, protect_mask=0), nofault)
    assert (dev["cls"] == 0).all()
    dev, _ = e.run_sites(sites)
    compare(dev, o.run_trials(sites, protect_mask=0), sites)


@pytest.mark.parametrize("prog", ["alu", "cmp", "rvc", "mem"])
def test_known_answer_programs_solo_interpreter(oracle_mod, prog):
    """The known-answer programs from process start through the solo
    pre-decoded interpreter only (FI_CFG_SOLO_ALL | NO_TRANSLATE |
    NO_SNAPSHOT_START | NO_EARLY_EXIT): every op of the alu program -- the
    M-extension edge pairs (x / 0, INT_MIN / -1, the W forms, mulh*) among
    them -- runs in the assembly inner loop (solo_fast_run), no-fault trials
    print the models and end masked, faulted trials match the oracle."""
    from shrewd_amd import Engine
    import test_isa_vectors as kat
    elf = {"alu": kat.program_elf, "cmp": kat.cmp_program_elf, "rvc": kat.rvc_program_elf,
           "mem": kat.mem_program_elf}[prog]()
    e = Engine(private_pages=64, flags=128 | 4 | 1 | 2)
    e.load_elf(elf, [prog])
    e.golden_run()
    o = oracle_mod.Oracle(elf, prog)
    o.run_golden()
    e.set_campaign(0x5EED00A5, REGS | PC, 1)
    e.set_protect(0)
    sites = e.sample(0, 1500)
    nofault = sites[:64].copy()
    nofault["inst"] = 1 << 40
    dev, h = e.run_sites(nofault)
    assert (dev["cls"] == 0).all()
    assert int(h["device_insts"]) == int(h["guest_insts"])
    compare(dev, o.run_trials(nofault, protect_mask=0), nofault)
    dev, _ = e.run_sites(sites)
    compare(dev, o.run_trials(sites, protect_mask=0), sites)
    st = e.debug_stats()
    assert int(st[54]) > 0, "the assembly inner loop did not run"
    e.close()


@pytest.mark.parametrize("flags", [0, 128 | 4 | 1 | 2])
def test_m5_simulator_control_ops(oracle_mod, flags):
    """The simulator-control M5 ops (test_isa_vectors.m5end_program_source):
    the device golden run ends at m5_fail with code 7 (sub m5_fail); faulted
    trials reach m5_quiesce (hang, sub m5_quiesce), an early m5_exit (sdc,
    sub m5_exit), a delayed exit (escape) and a changed fail code, bit for bit
    with the oracle -- default configuration (early exit from snapshots: a
    converged trial takes the golden run's end sub-code) and the solo
    interpreter from process start."""
    from shrewd_amd import Engine
    from shrewd_amd.fi import SITE_DT
    import test_isa_vectors as kat
    elf = kat.m5end_program_elf()
    e = Engine(private_pages=64, flags=flags)
    e.load_elf(elf, ["m5end"])
    g = e.golden_run()
    assert g.exit_code == kat.M5END_CODE & 0xFF and e.golden_stdout() == b"hi\n"
    o = oracle_mod.Oracle(elf, "m5end")
    o.run_golden()
    n = g.ninst
    L = [(i, 1 << b, reg) for reg in (5, 6, 7, 10, 11) for b in (0, 1, 9) for i in range(n)]
    sites = np.zeros(len(L), dtype=SITE_DT)
    for k, (i, mask, reg) in enumerate(L):
        sites[k] = (i, mask, 0, reg, k)
    dev, _ = e.run_sites(sites)
    compare(dev, o.run_trials(sites, protect_mask=0), sites)
    got = {(int(c), int(s)) for c, s in zip(dev["cls"], dev["sub"])}
    assert {(0, 2), (1, 1), (1, 2), (3, 2), (5, 1)} <= got, got
    e.set_campaign(0x5EED00A7, REGS | PC, 1)
    e.set_protect(0)
    sites = e.sample(0, 3000)
    dev, _ = e.run_sites(sites)
    compare(dev, o.run_trials(sites, protect_mask=0), sites)
    e.close()


@pytest.mark.parametrize("golden_m5", [False, True])
@pytest.mark.parametrize("flags", [0, 128 | 4 | 1 | 2])
def test_end_kind_decides_masked(oracle_mod, golden_m5, flags):
    """Same output and exit code by another end (exit syscall vs m5_exit,
    test_isa_vectors.endkind_program_source): SDC with the trial's own end
    sub-code, on the device as in the oracle."""
    from shrewd_amd import Engine
    import test_isa_vectors as kat
    elf = kat.endkind_program_elf(golden_m5)
    e = Engine(private_pages=64, flags=flags)
    e.load_elf(elf, ["endkind"])
    e.golden_run()
    o = oracle_mod.Oracle(elf, "endkind")
    o.run_golden()
    sites = kat.endkind_sites()
    dev, _ = e.run_sites(sites)
    compare(dev, o.run_trials(sites, protect_mask=0), sites)
    assert (dev["cls"] == 1).any() and (dev["cls"] == 0).any()
    e.close()


def test_clock_read_blocks_tick_blind_early_exit(oracle_mod):
    """Exact early exit when the golden suffix reads curTick: the clk program's
    branch-register faults take an arm with 16 extra non-counting ticks
    (ignored-syscall ecalls) and reconverge with the golden pc, registers,
    memory and numInst at every later snapshot -- but print a later time.
    The comparator must also require the golden tick count there
    (fi_trial.hip, DevCtx::clk_until): every such trial is SDC, as on the
    oracle, with early exit on (the golden run touches no FP/VM/LR-SC state,
    so snapshots and early exit stay enabled) and off."""
    from shrewd_amd import Engine
    import test_isa_vectors as kat
    elf = kat.clk_program_elf()
    o = oracle_mod.Oracle(elf, "clk")
    o.run_golden()
    sites = kat.clk_branch_sites(64)
    ref = o.run_trials(sites, protect_mask=0)
    assert (ref["cls"] == 1).all()
    for flags in (0, 2):   # default, FI_CFG_NO_EARLY_EXIT
        e = Engine(flags=flags, snapshot_interval=64)
        e.load_elf(elf, ["clk"])
        e.golden_run()
        dev, _ = e.run_sites(sites)
        if flags == 0:
            assert int(e.debug_stats()[11]) > 0, "early-exit comparisons did not run"
        compare(dev, ref, sites)
        e.close()


def test_stdin_file_classifies_fd0_trials(oracle_mod):
    """hello with bit 0 of a0 flipped before its write: write(0) touches the
    host's stdin, which only escapes while Process.input is "cin".  With an
    input file (fi_set_stdin) the write to the O_RDONLY fd 0 returns -EBADF
    and the trial is classified (SDC: nothing printed).  Outcomes equal the
    oracle's with the same input, also on C1's 1,000 sites (whose host
    escapes are write lengths of 2 GiB and more: a flipped a2 makes gem5's
    BufferArg allocate and zero that many host bytes, which a host may or may
    not survive); the engine refuses process settings after the golden run."""
    from shrewd_amd import Engine, EngineError, SITE_DT
    elf = workload_elf("hello")
    o = oracle_mod.Oracle(elf, "hello")
    o.set_stdin(b"some input\n")
    g = o.run_golden()
    fd0 = np.zeros(g.ninst + 1, SITE_DT)
    fd0["inst"] = np.arange(g.ninst + 1)
    fd0["mask"] = 1
    fd0["target"] = 10
    fd0["trial"] = np.arange(g.ninst + 1)
    cin = Engine()
    cin.load_elf(elf, ["hello"])
    cin.golden_run()
    cin.set_campaign(0x5EED0001, REGS, 1)
    c1 = cin.sample(0, 1000)
    a, _ = cin.run_sites(fd0)
    assert ((a["cls"] == 5) & (a["sub"] == 4)).sum() > 0
    a1, _ = cin.run_sites(c1)
    with pytest.raises(EngineError):
        cin.set_stdin(b"x")
    cin.close()
    e = Engine()
    e.load_elf(elf, ["hello"])
    e.set_stdin(b"some input\n")
    e.golden_run()
    b, _ = e.run_sites(fd0)
    assert not ((b["cls"] == 5) & (b["sub"] == 4)).any()
    compare(b, o.run_trials(fd0, protect_mask=0), fd0)
    b1, _ = e.run_sites(c1)
    compare(b1, o.run_trials(c1, protect_mask=0), c1)
    host = (b1["cls"] == 5) & (b1["sub"] == 4)
    assert (c1["target"][host] == 12).all() and (c1["mask"][host] >= 1 << 31).all()
    assert np.array_equal(a1, b1)
    e.close()


@pytest.mark.parametrize("name", ["crc32", "qsort"])
def test_background_translation_same_outcomes(engine_factory, oracle_mod, name):
    """The translated kernels build in the background (three code objects in
    parallel helper processes, no cache: FI_CFG_JIT_NO_CACHE): trials run at
    once on the static kernels and pick the build up at a chunk boundary.  Outcomes before, across and after the switch equal the
    waited engine's and the oracle's."""
    from shrewd_amd import Engine
    from shrewd_amd.fi import CFG_JIT_NO_CACHE
    n = 60000
    ref_e = engine_factory(name)
    ref_e.set_campaign(0x5EED0B6, REGS | PC, 1)
    ref_e.set_protect(0)
    ref, _ = ref_e.run_trials(0, n)
    e = Engine(flags=CFG_JIT_NO_CACHE)
    e.load_elf(workload_elf(name), [name])
    e.golden_run(wait_translation=False)
    assert e.translate_status() == "compiling"
    e.set_campaign(0x5EED0B6, REGS | PC, 1)
    e.set_protect(0)
    a, _ = e.run_trials(0, n)
    g = e.wait_translation()
    assert e.translate_status() == "" and g.translated_blocks > 0 and g.translate_us > 0
    b, _ = e.run_trials(0, n)
    assert np.array_equal(a, ref) and np.array_equal(b, ref)
    sites = e.sample(0, 2000)
    compare(a[:2000], oracle_for(oracle_mod, name).run_trials(sites, protect_mask=0), sites)
    e.close()


def test_sdc_early_exit(engine_factory, oracle_mod):
    """A trial whose output already differs but whose machine state equals a
    golden snapshot ends there as SDC (crcblk prints each block's CRC as it
    is computed): the same outcomes as running every SDC trial to its end and
    as the oracle, with fewer instructions executed on the device."""
    n = 20000
    on = engine_factory("crcblk", max_trials_per_launch=n)
    off = engine_factory("crcblk", flags=1024, max_trials_per_launch=n)
    for e in (on, off):
        e.set_campaign(0x5EED0C0B, REGS | PC, 1)
        e.set_protect(0)
    a, ha = on.run_trials(0, n)
    b, hb = off.run_trials(0, n)
    assert np.array_equal(a, b)
    assert (a["cls"] == 1).sum() > 100
    assert int(ha["device_insts"]) < int(hb["device_insts"])
    sites = on.sample(0, 3000)
    compare(a[:3000], oracle_for(oracle_mod, "crcblk").run_trials(sites, protect_mask=0), sites)


@pytest.mark.parametrize("name", ["qsort", "intmix"])
def test_resource_redo(engine_factory, oracle_mod, name):
    """Trials that run out of copy-on-write pages (FI_ESC_RESOURCE, an engine
    capacity limit) either take a block of overflow pages from the launch's
    pool and go on, or -- the pool spent, or off (FI_CFG_NO_OVERFLOW) -- run
    again with more pages before the histogram: with one private page per
    trial the outcomes equal the default engine's and the oracle's either
    way, while the same engine with neither escapes."""
    from shrewd_amd.fi import CFG_NO_OVERFLOW, CFG_NO_REDO
    n = 3000
    tight = engine_factory(name, private_pages=1, max_trials_per_launch=n)                    # overflow + redo
    redo = engine_factory(name, private_pages=1, flags=CFG_NO_OVERFLOW, max_trials_per_launch=n)
    ovf = engine_factory(name, private_pages=1, flags=CFG_NO_REDO, max_trials_per_launch=n)
    neither = engine_factory(name, private_pages=1, flags=CFG_NO_REDO | CFG_NO_OVERFLOW, max_trials_per_launch=n)
    for e in (tight, redo, ovf, neither):
        e.set_campaign(0x5EED0BED, REGS | PC | MEM, 1)
        e.set_protect(0)
    sites = tight.sample(0, n)
    b, hb = neither.run_sites(sites)
    esc = (b["cls"] == 5) & (b["sub"] == 5)
    assert esc.sum() > 0
    r, hr = redo.run_sites(sites)
    assert int(redo.debug_stats()[30]) == int(esc.sum()) and int(redo.debug_stats()[61]) == 0
    v, hv = ovf.run_sites(sites)
    blocks = int(ovf.debug_stats()[61])
    assert blocks > 0
    # the pool (64 blocks) runs dry at P = 1: the rest still escape without the redo pass
    assert int(((v["cls"] == 5) & (v["sub"] == 5)).sum()) == int(esc.sum()) - blocks
    a, ha = tight.run_sites(sites)
    assert int(tight.debug_stats()[30]) == int(esc.sum()) - int(tight.debug_stats()[61])
    for x, h in ((a, ha), (r, hr)):
        assert not ((x["cls"] == 5) & (x["sub"] == 5)).any()
        assert int(h["escape_sub"][5]) == 0 and int(h["trials"]) == n
    assert np.array_equal(a, r)
    ok = ~((v["cls"] == 5) & (v["sub"] == 5))
    assert np.array_equal(a[ok], v[ok])
    compare(a, oracle_for(oracle_mod, name).run_trials(sites, protect_mask=0), sites)
    assert np.array_equal(a[~esc], b[~esc])


@pytest.mark.parametrize("name", ["crc32", "qsort"])
def test_odd_pc_kernel(engine_factory, oracle_mod, name):
    """pc bit-0 flips leave the pc odd: their survivors run on the solo-odd
    kernel (translated odd-pc streams, second stream) -- the same outcomes as
    on the solo kernel and as the oracle."""
    e = engine_factory(name)
    off = engine_factory(name, flags=4096)   # FI_CFG_NO_ODD_KERNEL
    for x in (e, off):
        x.set_campaign(0x5EED0DD, REGS | PC, 1)
        x.set_protect(0)
    sites = e.sample(0, 400_000)
    sites = sites[(sites["target"] == 32) & (sites["mask"] == 1)][:600]
    assert len(sites) > 100
    e.kernel_timer_reset()
    a, _ = e.run_sites(sites)
    kinds = e.debug_dispatch_kinds()
    assert e.translate_status() == "" and 2 in kinds, kinds
    b, _ = off.run_sites(sites)
    assert 2 not in off.debug_dispatch_kinds()
    assert np.array_equal(a, b)
    compare(a, oracle_for(oracle_mod, name).run_trials(sites, protect_mask=0), sites)


def test_odd_stream_loop_proofs(engine_factory, oracle_mod):
    """pc bit-0 flips that land in a loop of odd-pc instructions run the
    translated odd-pc streams (solo-odd kernel), which the static proofs do
    not cover.  Past the golden run's length such a trial can only crash or
    hang: its translated calls return at the golden length and whenever a
    loop probe is due, and the probe proves the hang (qsort 80709 / 32646:
    a store loop whose values converge).  Records equal the engine's own
    without proofs and the oracle's (which runs them to the cap)."""
    from shrewd_amd.fi import CFG_NO_HANG_PROOF
    ids = [80709, 32646, 37937, 68608]
    on = engine_factory("qsort")
    off = engine_factory("qsort", flags=CFG_NO_HANG_PROOF)
    for e in (on, off):
        e.set_campaign(0x5EED0002, REGS | PC, 1)
        e.set_protect(0)
    sites = on.sample(0, max(ids) + 1)[ids]
    a, _ = on.run_sites(sites)
    assert int(on.debug_stats()[59]) >= 2
    b, _ = off.run_sites(sites)
    assert np.array_equal(a, b)
    assert (a["cls"][:2] == 3).all()
    compare(a, oracle_for(oracle_mod, "qsort").run_trials(sites, protect_mask=0), sites)


@pytest.mark.parametrize("name,seed,ids", [("qsort", 0x5EED0002, [11487, 46948]),
                                          ("intmix", 0x5EED0002, [64617, 53499, 34535]),
                                          ("qsort", 0x5EED0003, [631236, 934410, 140047, 644543, 802705])])
def test_rewritten_code_loops_bit_exact(engine_factory, oracle_mod, name, seed, ids):
    """The campaign tails: trials whose flipped base pointer stored into the
    text and that then loop through the rewritten code (intmix 64617: 1.33M
    instructions, 6 clean and 4 rewritten per iteration).  These trials leave
    the translated blocks at the rewritten instructions for the solo
    kernel's pre-decoded interpreter (which decodes the trial's own bytes)
    and come back at the next block leader; the test pins that path against
    the oracle.  qsort 631236 / 934410 (seed 3) keep rewriting code inside the
    assembly interpreter (its rewrite marking); 140047 / 802705 reach a vset*
    with vsew 6 (abort) and 644543 one with LMUL 1/16 (vl = 0, runs on)."""
    e = engine_factory(name)
    o = oracle_for(oracle_mod, name)
    e.set_campaign(seed, REGS | PC, 1)
    e.set_protect(0)
    sites = e.sample(0, max(ids) + 1)[ids]
    dev, _ = e.run_sites(sites)
    compare(dev, o.run_trials(sites, protect_mask=0), sites)
