"""gem5 SE checkpoint ingestion: campaigns that start from a
checkpoint instead of process start.

The checkpoints are written by the oracle in gem5's serialization format
(oracle/rv64se.c:or_write_checkpoint: m5.cpt INI sections + gzip memory
store).  A real gem5 checkpoint cannot be produced here (no gem5 build), so
the format is "parity unpinned" against gem5 itself; what is pinned is the
round trip: a campaign restored at numInst K behaves exactly like the
process-start campaign from K on.
"""
import numpy as np
import pytest

from conftest import workload_elf

REGS_PC = ((1 << 32) - 2) | (1 << 32)
MEM = 1 << 33


@pytest.fixture(scope="module")
def crc32_cpt(tmp_path_factory, oracle_mod):
    elf = workload_elf("crc32")
    o = oracle_mod.Oracle(elf, "crc32")
    g = o.run_golden()
    k = 20_000
    d = str(tmp_path_factory.mktemp("cpt") / "crc32_20000")
    o.write_checkpoint(k, d)
    return elf, d, k, o, g


def test_checkpoint_files(crc32_cpt):
    import gzip
    import os
    _, d, k, _, _ = crc32_cpt
    txt = open(os.path.join(d, "m5.cpt")).read()
    for sec in ("[system.cpu.xc.0]", "[system.cpu.workload]", "[system.cpu.workload.ptable]",
                "[system.cpu.workload.vmalist.Vma0]", "[system.physmem.store0]"):
        assert sec in txt
    regs = [l for l in txt.splitlines() if l.startswith("regs.integer=")][0]
    assert len(regs.split("=")[1].split()) == 33 * 8
    mem = gzip.open(os.path.join(d, "system.physmem.store0.pmem")).read()
    assert len(mem) % 4096 == 0 and len(mem) > 0


def test_restored_golden_is_the_suffix(crc32_cpt, oracle_mod):
    elf, d, k, o, g = crc32_cpt
    r = oracle_mod.Oracle(elf, "crc32", checkpoint=d)
    rg = r.run_golden()
    assert rg.ninst == g.ninst - k
    assert rg.exit_code == g.exit_code
    full = o.golden_stdout()
    assert full.endswith(r.golden_stdout())


def test_restored_trials_equal_shifted_process_start_trials(crc32_cpt, oracle_mod):
    """A trial restored at K and injected at t is the process-start trial
    injected at K + t: same class, sub-code, exit code, detail and flags;
    numInst shifted by K.  (Hangs only agree in class: the cap, 2 x golden
    numInst + 1000, follows each campaign's own golden run.)"""
    elf, d, k, o, g = crc32_cpt
    r = oracle_mod.Oracle(elf, "crc32", checkpoint=d)
    r.run_golden()
    sites = r.sample(0x5EED0C97, 0, 3000, REGS_PC)
    got = r.run_trials(sites, threads=8)
    shifted = sites.copy()
    shifted["inst"] += k
    ref = o.run_trials(shifted, threads=8)
    assert np.array_equal(got["cls"], ref["cls"])
    fin = got["cls"] != 3
    assert fin.sum() > 2500
    for f in ("sub", "exit_code", "flags", "detail"):
        assert np.array_equal(got[f][fin], ref[f][fin]), f
    assert np.array_equal(got["ninst"][fin] + k, ref["ninst"][fin])


def test_unsupported_checkpoint_is_refused(tmp_path, oracle_mod):
    elf = workload_elf("crc32")
    r = oracle_mod.Oracle.__new__(oracle_mod.Oracle)
    r.L = oracle_mod.lib()
    r.h = r.L.or_create_checkpoint(str(tmp_path).encode(), elf, len(elf))
    assert r.L.or_error(r.h).decode().startswith("cannot read")
    r.close()


@pytest.mark.gpu
def test_engine_from_checkpoint_matches_oracle(crc32_cpt, oracle_mod):
    """The engine restored from the same checkpoint: golden run and trials
    (register, pc and memory sites) bit-exact against the restored oracle."""
    from shrewd_amd import Engine
    elf, d, k, o, g = crc32_cpt
    r = oracle_mod.Oracle(elf, "crc32", checkpoint=d)
    rg = r.run_golden()
    e = Engine()
    e.load_checkpoint(d, elf)
    eg = e.golden_run()
    assert (eg.ninst, eg.ncycles, eg.exit_code) == (rg.ninst, rg.ncycles, rg.exit_code)
    assert e.golden_stdout() == r.golden_stdout()
    assert e.translate_status() == ""
    for structs, n in ((REGS_PC, 4000), (MEM, 2000)):
        e.set_campaign(0x5EEDC0DE, structs, 1)
        sites = e.sample(0, n)
        assert np.array_equal(sites, r.sample(0x5EEDC0DE, 0, n, structs))
        dev, _ = e.run_sites(sites)
        ref = r.run_trials(sites)
        bad = np.flatnonzero(dev != ref)
        assert not len(bad), f"{len(bad)} differ, first {sites[bad[0]]} {dev[bad[0]]} {ref[bad[0]]}"
    e.close()


@pytest.mark.gpu
def test_native_driver_from_checkpoint_matches_oracle(crc32_cpt, oracle_mod, tmp_path):
    """The native driver (the FaultCampaign SimObject's core) with --checkpoint:
    per-trial outcomes bit-exact against the oracle restored from the same
    directory."""
    import os
    import subprocess
    from conftest import ROOT
    from shrewd_amd import OUTCOME_DT
    from shrewd_amd import build as b
    elf, d, k, o, g = crc32_cpt
    exe = b.build_cli()
    n, seed = 2000, 0x5EEDC0DF
    prefix = str(tmp_path / "cpt_camp")
    r = subprocess.run([exe, "--workload", os.path.join(ROOT, "workloads", "crc32.elf"), "--cmd", "crc32",
                        "--trials", str(n), "--seed", hex(seed), "--structures", "int_reg,pc",
                        "--checkpoint", d, "--output", prefix], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = np.fromfile(prefix + ".outcomes.bin", OUTCOME_DT)
    ro = oracle_mod.Oracle(elf, "crc32", checkpoint=d)
    ro.run_golden()
    ref = ro.run_trials(ro.sample(seed, 0, n, REGS_PC))
    bad = np.flatnonzero(out != ref)
    assert not len(bad), f"{len(bad)} differ, first {bad[0]}: {out[bad[0]]} {ref[bad[0]]}"


# ------------------------------------------------------------ checkpoint breadth
# FP registers + fcsr (regs.floating_point, the ISA's miscRegFile), heap/mmap
# VMAs ([<process>.vmalist]) and curTick ([Globals]), each pinned by the same
# round trip: restored at K, the campaign is the process-start one from K on.
def _kat(name):
    import test_isa_vectors as kat
    return {"vm": kat.vm_program_elf, "rnd": kat.rnd_program_elf, "fp": kat.fp_program_elf}[name]()


def _cpt_case(oracle_mod, tmp_path, elf, argv0, frac):
    o = oracle_mod.Oracle(elf, argv0)
    g = o.run_golden()
    k = max(1, int(g.ninst * frac))
    d = str(tmp_path / f"{argv0}_{k}")
    o.write_checkpoint(k, d)
    r = oracle_mod.Oracle(elf, argv0, checkpoint=d)
    rg = r.run_golden()
    assert rg.ninst == g.ninst - k and rg.exit_code == g.exit_code
    assert o.golden_stdout().endswith(r.golden_stdout())
    return o, r, g, k, d


def _shifted_equal(o, r, k, structs, n, seed):
    sites = r.sample(seed, 0, n, structs)
    got = r.run_trials(sites, threads=8)
    shifted = sites.copy()
    shifted["inst"] += k
    ref = o.run_trials(shifted, threads=8)
    assert np.array_equal(got["cls"], ref["cls"])
    fin = got["cls"] != 3
    for f in ("sub", "exit_code", "flags", "detail"):
        assert np.array_equal(got[f][fin], ref[f][fin]), f
    assert np.array_equal(got["ninst"][fin] + k, ref["ninst"][fin])
    return got


def test_checkpoint_fp_state_round_trip(oracle_mod, tmp_path):
    """fpamo checkpointed after its FP registers and fflags hold values."""
    import os
    elf = workload_elf("fpamo")
    o, r, g, k, d = _cpt_case(oracle_mod, tmp_path, elf, "fpamo", 0.6)
    txt = open(os.path.join(d, "m5.cpt")).read()
    fregs = [l for l in txt.splitlines() if l.startswith("regs.floating_point=")][0].split("=")[1].split()
    assert any(int(b) for b in fregs), "the checkpoint should hold FP state"
    misc = [l for l in txt.splitlines() if l.startswith("miscRegFile=")][0].split("=")[1].split()
    assert len(misc) == 193
    _shifted_equal(o, r, k, REGS_PC, 2000, 0x5EEDF9)


def test_checkpoint_vma_list_round_trip(oracle_mod, tmp_path):
    """The vm program checkpointed after its brk / mmap calls: a VMA list
    beyond the stack VMA and a lowered mmap end."""
    import os
    import re
    o, r, g, k, d = _cpt_case(oracle_mod, tmp_path, _kat("vm"), "vm", 0.7)
    txt = open(os.path.join(d, "m5.cpt")).read()
    nv = int(re.search(r"\[system\.cpu\.workload\.vmalist\]\nsize=(\d+)", txt).group(1))
    assert nv > 1
    assert "mmapEnd=4611686018427387904" not in txt
    _shifted_equal(o, r, k, REGS_PC | MEM, 2000, 0x5EEDF8)


def test_checkpoint_curtick_round_trip(oracle_mod, tmp_path):
    """The rnd program checkpointed between getrandom and its clock_gettime
    calls: the restored run reports the same times (curTick continues from the
    checkpoint's [Globals] curTick), so its output is the original's."""
    import test_isa_vectors as kat
    elf = kat.rnd_program_elf()
    o = oracle_mod.Oracle(elf, "rnd")
    g = o.run_golden()
    k = 10   # after the getrandom ecall, before the first clock_gettime
    d = str(tmp_path / "rnd_cpt")
    o.write_checkpoint(k, d)
    assert "curTick=0\n" not in open(d + "/m5.cpt").read()
    r = oracle_mod.Oracle(elf, "rnd", checkpoint=d)
    rg = r.run_golden()
    assert rg.ninst == g.ninst - k
    assert r.golden_stdout() == o.golden_stdout()
    kat.rnd_check(r.golden_stdout())


def test_checkpoint_vector_state_refused(oracle_mod, tmp_path, crc32_cpt):
    import shutil
    elf, d, k, o, g = crc32_cpt
    d2 = str(tmp_path / "vec")
    shutil.copytree(d, d2)
    txt = open(d2 + "/m5.cpt").read().replace("_vtype=9223372036854775808", "_vtype=24")
    open(d2 + "/m5.cpt", "w").write(txt)
    r = oracle_mod.Oracle.__new__(oracle_mod.Oracle)
    r.L = oracle_mod.lib()
    r.h = r.L.or_create_checkpoint(d2.encode(), elf, len(elf))
    assert "vector" in r.L.or_error(r.h).decode()
    r.close()


def test_miscreg_indices_fixture():
    """The checkpoint readers' miscRegFile positions (oracle/rv64se.c
    CPT_MISC_*, shrewd_amd/csrc/fi_checkpoint.cpp kMisc*) against the
    reference enum (tests/golden/riscv_miscreg.json)."""
    import json
    import os
    import re
    from conftest import ROOT
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "riscv_miscreg.json")))
    src = open(os.path.join(ROOT, "oracle", "rv64se.c")).read()
    m = re.search(r"CPT_MISC_FFLAGS = (\d+), CPT_MISC_FRM = (\d+), CPT_NUM_MISC = (\d+)", src)
    assert tuple(map(int, m.groups())) == (fx["MISCREG_FFLAGS"], fx["MISCREG_FRM"], fx["NUM_PHYS_MISCREGS"])
    cpp = open(os.path.join(ROOT, "shrewd_amd", "csrc", "fi_checkpoint.cpp")).read()
    m = re.search(r"kMiscFflags = (\d+), kMiscFrm = (\d+)", cpp)
    assert tuple(map(int, m.groups())) == (fx["MISCREG_FFLAGS"], fx["MISCREG_FRM"])


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["fp", "vm", "rnd"])
def test_engine_from_wide_checkpoint_matches_oracle(oracle_mod, tmp_path, case):
    """The engine restored from checkpoints holding FP state (fpamo), a VMA
    list (vm) and a nonzero curTick (rnd): golden run and trials bit-exact
    against the restored oracle."""
    from shrewd_amd import Engine
    elf, argv0, frac = {"fp": (workload_elf("fpamo"), "fpamo", 0.6), "vm": (_kat("vm"), "vm", 0.7),
                        "rnd": (_kat("rnd"), "rnd", None)}[case]
    o = oracle_mod.Oracle(elf, argv0)
    g = o.run_golden()
    k = 10 if frac is None else max(1, int(g.ninst * frac))
    d = str(tmp_path / f"{case}_cpt")
    o.write_checkpoint(k, d)
    r = oracle_mod.Oracle(elf, argv0, checkpoint=d)
    rg = r.run_golden()
    e = Engine(private_pages=64)
    e.load_checkpoint(d, elf)
    eg = e.golden_run()
    assert (eg.ninst, eg.ncycles, eg.exit_code) == (rg.ninst, rg.ncycles, rg.exit_code)
    assert e.golden_stdout() == r.golden_stdout()
    for structs, n in ((REGS_PC, 2000), (MEM, 1000)):
        e.set_campaign(0x5EEDC0DF, structs, 1)
        sites = e.sample(0, n)
        assert np.array_equal(sites, r.sample(0x5EEDC0DF, 0, n, structs))
        dev, _ = e.run_sites(sites)
        ref = r.run_trials(sites)
        bad = np.flatnonzero(dev != ref)
        assert not len(bad), f"{len(bad)} differ, first {sites[bad[0]]} {dev[bad[0]]} {ref[bad[0]]}"
    e.close()
