"""GPU parity of tick-domain injection (cpu_type="timing").

The engine rebuilds the golden run's requests from its device trace, times
them with its own restatement of the reference board (fi_timing.cpp), maps
each tick site to the numInst site it equals (or a contract escape) and runs
those on the device.  The oracle runs every tick trial literally: the flip
applied to the attempt in flight (rv64se.c tk_*).  Bar: the golden request
lists and ticks identical, the sampled tick sites identical, and per-trial
outcomes bit-exact.  Against a live gem5 TimingSimpleCPU: parity unpinned.
"""
import numpy as np
import pytest

from conftest import np_histogram, workload_elf

pytestmark = pytest.mark.gpu

REGS = (1 << 32) - 2
PC = 1 << 32
RESULT = 1 << 34
SEED = 0x5EED7101


@pytest.fixture(scope="module")
def tick_pair(oracle_mod):
    from shrewd_amd import Engine, build_library
    build_library()
    cache = {}

    def make(name):
        if name not in cache:
            e = Engine()
            e.load_elf(workload_elf(name), [name])
            e.set_cpu_model("timing")
            e.golden_run()
            o = oracle_mod.Oracle(workload_elf(name), name)
            o.run_golden()
            o.tick_setup()
            cache[name] = (e, o)
        return cache[name]

    yield make
    for e, o in cache.values():
        e.close()
        o.close()


def _compare(dev, ref, sites):
    bad = np.nonzero(dev != ref)[0]
    if len(bad):
        i = bad[0]
        raise AssertionError(f"{len(bad)} of {len(sites)} outcomes differ; first: site={sites[i]} "
                             f"gpu={dev[i]} oracle={ref[i]}")


@pytest.mark.parametrize("name", ["hello", "crc32", "qsort", "intmix"])
def test_golden_tick_trace_matches_oracle(tick_pair, name):
    """The requests rebuilt from the device's golden trace (frames in SE
    allocation order, page-fault retries, second fetches) and their ticks =
    the oracle's, recorded by its own interpreter."""
    e, o = tick_pair(name)
    info = e.tick_info()
    assert info["status"] == ""
    ops, ticks = e.tick_trace()
    oops, oticks = o.tick_trace()
    assert len(ops) == len(oops) == info["attempts"]
    for f in ("fetch", "addr", "size", "nfetch", "nfrag", "kind", "cmd"):
        bad = np.nonzero((ops[f] != oops[f]).reshape(len(ops), -1).any(axis=1))[0]
        assert not len(bad), (f, int(bad[0]), ops[bad[0]], oops[bad[0]])
    assert (ticks == oticks).all()
    assert info["golden_ticks"] == int(oticks["exec"][-1])


@pytest.mark.parametrize("name", ["crc32", "qsort"])
def test_tick_sampler_matches_oracle(tick_pair, name):
    e, o = tick_pair(name)
    for structs, burst in ((REGS | PC, 1), (REGS | PC | RESULT, 1), (REGS, 4)):
        e.set_campaign(SEED, structs, burst)
        e.set_bits(2**64 - 1)
        a = e.sample_tick_sites(1000, 5000)
        b = o.tick_sample(SEED, 1000, 5000, structs, burst)
        assert (a == b).all()


@pytest.mark.parametrize("name,structs", [("crc32", REGS | PC | RESULT), ("qsort", REGS | PC | RESULT),
                                          ("hello", REGS | PC), ("intmix", REGS | PC)])
def test_tick_trials_match_oracle(tick_pair, name, structs):
    """Sampled tick campaigns: device outcomes (mapped numInst sites, golden
    copies, contract escapes) = the oracle's literal trials, per trial."""
    e, o = tick_pair(name)
    e.set_campaign(SEED, structs, 1)
    e.set_bits(2**64 - 1)
    n = 6000
    dev, hist = e.run_tick_trials(0, n)
    ts = o.tick_sample(SEED, 0, n, structs)
    ref = o.run_tick_trials(ts, threads=16)
    _compare(dev, ref, ts)
    assert hist["trials"] == n
    # the histogram files each trial under its tick site's target / lowest bit
    h = np_histogram(np.array([(0, int(s["mask"]), 0, int(s["target"]), 0) for s in ts],
                              dtype=[("inst", "<u8"), ("mask", "<u8"), ("addr", "<u8"), ("target", "<u4"),
                                     ("trial", "<u4")]), ref)
    assert (hist["counts"] == h["counts"]).all()
    assert (hist["escape_sub"] == h["escape_sub"]).all()
    assert hist["guest_insts"] == h["guest_insts"]


def _boundary_sites(o, rng, n):
    """Tick sites on the edges of attempts (first / last tick of each phase),
    every target kind, across the run."""
    ops, ticks = o.tick_trace()
    end = int(ticks["exec"][-1])   # sites lie in [0, golden ticks)
    out = []
    for j in rng.integers(0, len(ops), n):
        T = ticks[j]
        cand = [int(T["fetch_send"][0]), int(T["fetch_send"][0]) + 1, int(T["exec"]), int(T["exec"]) + 1,
                int(T["done"])]
        if ops["nfetch"][j] == 2:
            cand += [int(T["fetch_done"][0]), int(T["fetch_done"][0]) + 1]
        t = int(rng.choice(cand))
        tgt = int(rng.choice([32, 32, 34, int(rng.integers(1, 32))]))
        b = int(rng.integers(0, 64)) if tgt != 32 else int(rng.choice([1, 2, 3, 5, 12, 20, 40]))
        out.append((min(t, end - 1), 1 << b, tgt, len(out)))
    return np.array(out, dtype=[("tick", "<u8"), ("mask", "<u8"), ("target", "<u4"), ("trial", "<u4")])


@pytest.mark.parametrize("name", ["crc32", "qsort", "hello"])
def test_tick_boundary_sites_match_oracle(tick_pair, name):
    """Explicit tick sites at the phase edges the contract splits on (pc flips
    on straddles, data-phase flips, ecall attempts), device vs oracle."""
    e, o = tick_pair(name)
    ts = _boundary_sites(o, np.random.default_rng(5), 6000)
    dev, _ = e.run_tick_sites(ts)
    ref = o.run_tick_trials(ts, threads=16)
    _compare(dev, ref, ts)
    esc = (ref["cls"] == 5) & (ref["sub"] == 7)
    assert esc.any() and (~esc).sum() > 0.5 * len(ts)


def test_tick_map_dispositions(tick_pair):
    """fi_map_tick_sites: golden-equal and escape trials never reach the device;
    their host outcomes are the oracle's."""
    e, o = tick_pair("crc32")
    ts = _boundary_sites(o, np.random.default_rng(9), 3000)
    # flips of a load's destination while its data is outstanding: golden-equal
    ops, ticks = o.tick_trace()
    gops = o.golden_ops()
    loads = np.nonzero((ops["kind"] == 0) & (ops["nfrag"] > 0) & (ops["cmd"] == 0))[0]
    extra = [(int(ticks["done"][j]), 1 << 7, (int(gops["dst"][j]) & 0xFFFFFFFE).bit_length() - 1, 0)
             for j in loads[::max(1, len(loads) // 200)] if bin(int(gops["dst"][j]) & 0xFFFFFFFE).count("1") == 1]
    ts = np.concatenate([ts, np.array(extra, ts.dtype)])
    ts["trial"] = np.arange(len(ts))
    sites, disp, ho = e.map_tick_sites(ts)
    ref = o.run_tick_trials(ts, threads=16)
    assert set(np.unique(disp).tolist()) <= {0, 1, 2}
    assert (disp == 2).any() and (disp == 1).any()
    assert (ho[disp == 2] == ref[disp == 2]).all()
    assert (ho[disp == 1] == ref[disp == 1]).all()


def test_fault_campaign_timing(tmp_path, oracle_mod):
    """The SimObject mirror with cpu_type='timing' runs the tick campaign."""
    from shrewd_amd import FaultCampaign
    path = tmp_path / "crc32.elf"
    path.write_bytes(workload_elf("crc32"))
    fc = FaultCampaign(str(path), cmd=["crc32"], trials=3000, seed=SEED, structures=("int_reg", "pc"),
                       cpu_type="TimingSimpleCPU")
    out = fc.run()
    o = oracle_mod.Oracle(workload_elf("crc32"), "crc32")
    o.run_golden()
    o.tick_setup()
    ref = o.run_tick_trials(o.tick_sample(SEED, 0, 3000, REGS | PC), threads=16)
    assert (out == ref).all()
    assert fc.summary()["trials"] == 3000
    o.close()


def test_timing_refuses_clock_reader(tmp_path):
    """A golden run that reads curTick has another output under TimingSimpleCPU:
    cpu_type='timing' refuses it (the atomic campaign is unaffected)."""
    from shrewd_amd import FaultCampaign
    from shrewd_amd.fi import EngineError
    from test_isa_vectors import clk_program_elf
    path = tmp_path / "clk.elf"
    path.write_bytes(clk_program_elf())
    with pytest.raises(EngineError, match="curTick"):
        FaultCampaign(str(path), cmd=["clk"], trials=10, cpu_type="timing")
    FaultCampaign(str(path), cmd=["clk"], trials=10, cpu_type="atomic").run()


def test_native_cli_timing(tick_pair, tmp_path):
    """fi_campaign --cpu-type timing (one engine and two on device 0): the
    engine's tick campaign, outcome for outcome."""
    import os
    import subprocess
    from conftest import ROOT
    from shrewd_amd import HIST_DT, OUTCOME_DT
    from shrewd_amd import build as b
    exe = b.build_cli()
    e, _ = tick_pair("crc32")
    n = 4000
    e.set_campaign(SEED, REGS | PC, 1)
    e.set_bits(2**64 - 1)
    ref, rh = e.run_tick_trials(0, n)
    for devices in ("0", "0,0"):
        prefix = str(tmp_path / f"t{devices.count(',')}")
        r = subprocess.run([exe, "--workload", os.path.join(ROOT, "workloads", "crc32.elf"), "--cmd", "crc32",
                            "--trials", str(n), "--seed", hex(SEED), "--structures", "int_reg,pc",
                            "--cpu-type", "timing", "--devices", devices, "--output", prefix],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        out = np.fromfile(prefix + ".outcomes.bin", OUTCOME_DT)
        hist = np.fromfile(prefix + ".hist.bin", HIST_DT)[0]
        assert out.tobytes() == ref.tobytes()
        assert hist["counts"].tobytes() == rh["counts"].tobytes()
