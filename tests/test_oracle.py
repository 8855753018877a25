"""CPU tests of the oracle (test infrastructure): workloads, sampler, syscall table."""
import json
import os
import struct
import zlib

import numpy as np
import pytest

from conftest import ROOT, workload_elf

M64 = 2**64


def ref_crc32():
    x, buf = 0x12345678, b""
    for _ in range(1024):
        x ^= (x << 13) & 0xFFFFFFFF
        x ^= x >> 17
        x ^= (x << 5) & 0xFFFFFFFF
        buf += struct.pack("<I", x)
    return b"%08x\n" % zlib.crc32(buf)


def ref_crcblk():
    x, buf = 0x12345678, b""
    for _ in range(1024):
        x ^= (x << 13) & 0xFFFFFFFF
        x ^= x >> 17
        x ^= (x << 5) & 0xFFFFFFFF
        buf += struct.pack("<I", x)
    return b"".join(b"%08x\n" % zlib.crc32(buf[k:k + 512]) for k in range(0, 4096, 512))


def ref_qsort():
    x, a = 1, []
    for _ in range(1024):
        x = (x * 1103515245 + 12345) & 0x7FFFFFFF
        a.append(x)
    h = 0
    for v in sorted(a):
        h = (h * 31 + v) % M64
    return b"%016x\n" % h


def ref_intmix():
    acc, h, acc2 = [0] * 512, 0x2545F4914F6CDD1D, 0
    for i in range(10000):
        h ^= i
        h = (h * 0x9E3779B97F4A7C15) % M64
        h ^= h >> 29
        c = bin(h).count("1")
        k = (h >> 7) % 251
        acc[k & 511] = (acc[k & 511] + c + k) % M64
        if h & 3 == 0:
            acc2 = (acc2 * 3 + h // 7) % M64
    t = acc2
    for v in acc:
        t = ((t << 5) | (t >> 59)) % M64
        t ^= v
    return b"%016x\n" % t


def _fclass(ui, eb, fb):
    """RISC-V fclass bit (the ISA manual's table), from the raw encoding"""
    e, f, s = (ui >> fb) & ((1 << eb) - 1), ui & ((1 << fb) - 1), (ui >> (eb + fb)) & 1
    emax = (1 << eb) - 1
    if e == emax:
        if f == 0:
            return 1 << (0 if s else 7)
        return 1 << (9 if (f >> (fb - 1)) & 1 else 8)
    if e == 0:
        return 1 << ((3 if s else 4) if f == 0 else (2 if s else 5))
    return 1 << (1 if s else 6)


def ref_fpamo():
    """workloads/fpamo.s: F/D/Zfh moves + AMOs folded into an FNV-style hash"""
    h = 0x1234567

    def mix(v):
        nonlocal h
        h = ((h ^ (v % M64)) * 0x100000001B3) % M64

    sx = lambda v, n: (v & ((1 << n) - 1)) - ((v >> (n - 1) & 1) << n)  # noqa: E731
    box32 = lambda v: 0xFFFFFFFF00000000 | (v & 0xFFFFFFFF)  # noqa: E731
    unbox32 = lambda v: v & 0xFFFFFFFF if v >> 32 == 0xFFFFFFFF else 0x7FC00000  # noqa: E731
    S = 1 << 63
    dvals = [0x3ff0000000000000, 0xbff8000000000000, 0x7ff0000000000000, 0x1,
             0x7ff4000000000000, 0x8000000000000000, 0x7ff8000000000000, 0xffefffffffffffff]
    f1 = 0
    for d in dvals:
        f1 = d
        mix(_fclass(d, 11, 52))
        f2 = (d & ~S) | (~d & S)
        mix(f2)
        f3 = (d & ~S) | ((d ^ f2) & S)
        mix(f3)
        x = unbox32(d)
        mix(sx(box32(x) & 0xFFFFFFFF, 32))
    fvals = [0x3f800000, 0xff800000, 0x7fa00000, 0x80000001]
    for v in fvals:
        f5 = box32(v)
        mix(_fclass(v, 8, 23))
        mix(sx(v & 0x7FFFFFFF, 32))
        a0 = sx(v, 32) % M64
        mix(a0)
        mix(box32(a0))
    f5 = box32(fvals[-1])
    f8 = 0xFFFFFFFFFFFF0000 | 0x3c00
    mix(_fclass(0x3c00, 5, 10))
    mix(0x3c00)
    mix(0xFFFFFFFFFFFF0000 | 0xbc00)
    mem = bytearray(struct.pack("<QQQQQ", 0x0123456789abcdef, 0xfedcba9876543210, 0x0000000500000005, 0, 0))

    def amo(off, size, fn):
        old = int.from_bytes(mem[off:off + size], "little")
        new = fn(old) % (1 << (8 * size))
        mem[off:off + size] = new.to_bytes(size, "little")
        return sx(old, 32) % M64 if size == 4 else old

    s32 = lambda v: sx(v, 32)  # noqa: E731
    s64 = lambda v: sx(v, 64)  # noqa: E731
    mix(amo(0, 4, lambda m: m + 0x11))
    b = -5 % M64
    mix(amo(0, 4, lambda m: b if s32(b) < s32(m) else m))
    mix(amo(0, 4, lambda m: max(b & 0xFFFFFFFF, m)))
    b = 0x0f0f
    mix(amo(8, 8, lambda m: m ^ b))
    mix(amo(8, 8, lambda m: m | b))
    mix(amo(8, 8, lambda m: m & b))
    mix(amo(8, 8, lambda m: 7))
    b = -9 % M64
    mix(amo(8, 8, lambda m: b if s64(b) > s64(m) else m))
    mix(amo(8, 8, lambda m: min(b, m)))
    mix(amo(8, 8, lambda m: b if s64(b) < s64(m) else m))
    b = 3
    mix(amo(17, 4, lambda m: m + b))
    amo(17, 4, lambda m: b)
    mix(amo(17, 4, lambda m: b if s32(b) > s32(m) else m))
    mix(amo(17, 4, lambda m: min(b, m)))
    mix(amo(17, 4, lambda m: m | b))
    mix(amo(17, 4, lambda m: m & b))
    mix(amo(17, 4, lambda m: m ^ b))
    for off in (0, 8, 16):
        mix(int.from_bytes(mem[off:off + 8], "little"))
    mem[24:32] = f1.to_bytes(8, "little")
    mem[32:36] = (f5 & 0xFFFFFFFF).to_bytes(4, "little")
    mem[36:38] = (f8 & 0xFFFF).to_bytes(2, "little")
    mix(int.from_bytes(mem[24:32], "little"))
    mix(int.from_bytes(mem[32:40], "little"))
    mix(0xFFFFFFFFFFFF0000 | int.from_bytes(mem[36:38], "little"))
    return b"%016x\n" % h


EXPECTED = {"hello": b"Hello world!\n", "crc32": ref_crc32(), "qsort": ref_qsort(), "intmix": ref_intmix(),
            "fpamo": ref_fpamo(), "crcblk": ref_crcblk()}


@pytest.mark.parametrize("name", list(EXPECTED))
def test_golden_outputs(oracle_mod, name):
    o = oracle_mod.Oracle(workload_elf(name), name)
    g = o.run_golden()
    assert g.exit_code == 0
    assert o.golden_stdout() == EXPECTED[name]
    assert g.ncycles >= g.ninst > 0


def test_assembler_is_reproducible():
    from tools.rvasm.rvasm import assemble
    for name in EXPECTED:
        with open(os.path.join(ROOT, "workloads", f"{name}.s")) as f:
            assert assemble(f.read()) == workload_elf(name), f"{name}.elf is stale: re-run tools/rvasm"


def test_hello_counts(oracle_mod):
    # hello = li,auipc,addi,li,li,(ecall) li,li,(ecall): 7 committed instructions;
    # ecalls are not counted (atomic.cc:687-689) but take a tick each.
    o = oracle_mod.Oracle(workload_elf("hello"), "hello")
    g = o.run_golden()
    assert g.ninst == 7


def test_sampler_deterministic_and_sharded(oracle_mod):
    o = oracle_mod.Oracle(workload_elf("crc32"), "crc32")
    g = o.run_golden()
    s_all = o.sample(7, 0, 1000, ((1 << 32) - 2) | (1 << 32) | (1 << 33), 1)
    s_a = o.sample(7, 0, 400, ((1 << 32) - 2) | (1 << 32) | (1 << 33), 1)
    s_b = o.sample(7, 400, 600, ((1 << 32) - 2) | (1 << 32) | (1 << 33), 1)
    assert np.array_equal(s_all, np.concatenate([s_a, s_b]))
    assert (s_all["inst"] < g.ninst).all()
    assert set(np.unique(s_all["target"])) <= set(range(1, 34))
    assert (np.bitwise_count(s_all["mask"]) == 1).all()
    mem = s_all[s_all["target"] == 33]
    assert len(mem) > 0 and (mem["addr"] % 8 == 0).all()


def test_sampler_burst(oracle_mod):
    o = oracle_mod.Oracle(workload_elf("qsort"), "qsort")
    o.run_golden()
    for k in (2, 4, 8, 64):
        s = o.sample(1, 0, 300, 1 << 33, k)
        assert (np.bitwise_count(s["mask"]) == k).all()


def test_syscall_table_fixture(oracle_mod):
    """The compact classification in oracle+device matches the table derived
    from src/arch/riscv/linux/se_workload.cc (tools/oracle/gen_syscall_table.py)."""
    with open(os.path.join(ROOT, "tests", "golden", "syscalls_rv64.json")) as f:
        tab = {int(k): v for k, v in json.load(f).items()}
    modelled = {29, 57, 63, 64, 66, 78, 93, 94, 96, 113, 160, 163, 172, 173, 174, 175, 176, 177, 178, 214, 215, 222,
                258, 261, 278, 1058}
    for num in range(-5, 2100):
        got = oracle_mod.sys_class(num)
        if num not in tab:
            exp = 0
        elif num in modelled:
            exp = 4
        elif tab[num][1] == "unimpl":
            exp = 1
        elif tab[num][1] == "ignore":
            exp = 2
        else:
            exp = 3
        assert got == exp, (num, tab.get(num))


def test_oracle_trials_smoke(oracle_mod):
    o = oracle_mod.Oracle(workload_elf("crc32"), "crc32")
    g = o.run_golden()
    sites = o.sample(0x5EED0002, 0, 500, ((1 << 32) - 2) | (1 << 32), 1)
    out = o.run_trials(sites, threads=4)
    assert len(out) == 500
    cls = np.bincount(out["cls"], minlength=6)
    assert cls[0] > 300            # most register flips are masked
    assert cls[2] > 0              # PC flips crash
    masked = out[out["cls"] == 0]
    # output-masked trials usually retire exactly the golden count (a few take
    # a different path to the same output)
    assert (masked["ninst"] == g.ninst).mean() > 0.95
    assert (masked["exit_code"] == 0).all()


def test_unapplied_memory_site(oracle_mod):
    o = oracle_mod.Oracle(workload_elf("crc32"), "crc32")
    o.run_golden()
    site = np.zeros(1, oracle_mod.SITE_DT)[0]
    site["inst"], site["mask"], site["addr"], site["target"] = 10, 1, 0x100000000, 33
    res, out = o.run_one(site)
    assert res["cls"] == 0 and res["flags"] == 3


def load_decode_vectors():
    """tests/golden/decode_rv64.npz: instruction words and the class gem5's own
    decoder (decoder.isa through the reference isa_parser) gives each; made by
    tools/oracle/gen_decode_vectors.py."""
    z = np.load(os.path.join(ROOT, "tests", "golden", "decode_rv64.npz"))
    return z["raw"], z["leaf"], z["cls"], z["fmt"], z["mnem"]


def test_decode_matches_gem5_decoder(oracle_mod):
    raw, leaf, cls, fmt, mnem = load_decode_vectors()
    assert len(raw) > 250_000 and len(cls) > 800
    seen = {}
    for r, lf in zip(raw.tolist(), leaf.tolist()):
        seen.setdefault(lf, set()).add(oracle_mod.mnemonic(r))
    executed = set()
    for lf, names in seen.items():
        # every gem5 class maps to exactly one oracle op ...
        assert len(names) == 1, (cls[lf], names)
        name = names.pop()
        if cls[lf] == "Unknown":
            assert name == "unknown"
        elif name.startswith("escape:"):
            # ... a class the engine does not execute ends the trial as an escape
            assert name != "escape:UNKNOWN"
        elif name.startswith("vector:"):
            # ... an RVV class carries its action before any vset*
            # (gen_vector_actions.py): whole-register moves need vector state (vset*
            # execute from the start state: their own mnemonics, below)
            act = int(name.split(":")[1])
            assert 2 <= act <= 6
            assert str(fmt[lf]) != "VConfOp", cls[lf]
            if str(fmt[lf]) in ("VlWholeOp", "VsWholeOp", "VMvWholeFormat"):
                assert act == 6, cls[lf]
            if "Float" in str(fmt[lf]):   # no vill check before the SEW = 8 decode, no non-split float op at SEW 8
                assert act in (2, 5), cls[lf]
        else:
            # ... and an executed class carries gem5's own mnemonic
            assert name == str(mnem[lf]), (cls[lf], name)
            executed.add(name)
    assert {"c_addi4spn", "addi", "ld", "sd", "jalr", "mulhsu", "sh3add_uw", "czero_nez",
            "csrrw", "csrrci", "ecall", "fence_i", "prefetch_w"} <= executed


# ---------------------------------------------------------------- SHREWD op classes
INTALU, INTMULT, INTDIV, MEMREAD, MEMWRITE = 1, 2, 3, 52, 53
RESULT = 34


def test_opclass_fixture_matches_table():
    """gem5_opclass_table.h (device + oracle) carries exactly the OpClass the
    reference's generated constructors name (tests/golden/opclass_rv64.json)."""
    import re
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "opclass_rv64.json")))
    enum, ops = fx["enum"], fx["ops"]
    assert enum[:4] == ["No_OpClass", "IntAlu", "IntMult", "IntDiv"] and enum[MEMREAD] == "MemRead"
    hdr = open(os.path.join(ROOT, "shrewd_amd", "csrc", "gem5_opclass_table.h")).read()
    rows = dict((n, int(c)) for n, c in re.findall(r"X\((\w+), (\d+)\)", hdr))
    assert rows == {n: enum.index(c) for n, c in ops.items()}
    for n, c in {"add": "IntAlu", "c_addi": "IntAlu", "beq": "IntAlu", "jal": "IntAlu", "mul": "IntMult",
                 "mulhu": "IntMult", "div_": "IntDiv", "remuw": "IntDiv", "lw": "MemRead", "c_ldsp": "MemRead",
                 "sd": "MemWrite", "amoadd_w": "MemRead", "fmv_x_d": "FloatCvt", "ecall": "No_OpClass"}.items():
        assert ops[n] == c, n


def _result_site(oracle_mod, inst, mask):
    s = np.zeros(1, oracle_mod.SITE_DT)[0]
    s["inst"], s["mask"], s["target"] = inst, mask, RESULT
    return s


def test_result_fault_known_answers(oracle_mod):
    """hello: 0 li a0,1 | 1-2 la a1 | 3 li a2,13 | 4 li a7,64 | ecall | 5 li a0,0 | 6 li a7,94 | ecall."""
    o = oracle_mod.Oracle(workload_elf("hello"), "hello")
    o.run_golden()
    res, out = o.run_one(_result_site(oracle_mod, 3, 1))          # count 13 -> 12: the newline is lost
    assert res["cls"] == 1 and out == b"Hello world!" and res["flags"] == 1
    res, out = o.run_one(_result_site(oracle_mod, 5, 1))          # armed at the ecall, lands on li a0,0
    assert res["cls"] == 1 and res["exit_code"] == 1 and out == b"Hello world!\n"
    o.set_protect_opclasses(1 << INTALU)                           # the shadow ALU disagrees at commit
    res, _ = o.run_one(_result_site(oracle_mod, 3, 1))
    assert res["cls"] == 4 and res["ninst"] == 4
    o.set_protect_opclasses((1 << MEMREAD) | (1 << MEMWRITE) | (1 << INTMULT))   # no shadow for li
    res, _ = o.run_one(_result_site(oracle_mod, 3, 1))
    assert res["cls"] == 1


def test_result_fault_replication_properties(oracle_mod):
    """Protecting classes only turns outcomes into detected-by-replica; the
    classes FUPool::getUnit gives no shadow (MemRead/MemWrite) change nothing."""
    o = oracle_mod.Oracle(workload_elf("crc32"), "crc32")
    o.run_golden()
    sites = o.sample(7, 0, 3000, 1 << RESULT, 1)
    assert (sites["target"] == RESULT).all()
    base = o.run_trials(sites)
    assert (base["cls"] != 4).all() and ((base["flags"] & 2) != 0).any()   # stores/branches: nothing to flip
    o.set_protect_opclasses((1 << MEMREAD) | (1 << MEMWRITE))
    assert np.array_equal(o.run_trials(sites), base)
    o.set_protect_opclasses((1 << INTALU) | (1 << INTMULT) | (1 << INTDIV))
    prot = o.run_trials(sites)
    same = prot == base
    assert ((prot["cls"] == 4) | same).all() and (prot["cls"] == 4).sum() > 0
    assert (base["cls"][prot["cls"] == 4] != 4).all()


def test_sampler_bits_mask(oracle_mod):
    """`bits` restricts the lowest flipped bit to the eligible positions; the
    full mask is the plain draw (same sites as without it)."""
    from shrewd_amd.fi import bits_mask
    o = oracle_mod.Oracle(workload_elf("crc32"), "crc32")
    o.run_golden()
    regs = ((1 << 32) - 2)
    plain = o.sample(7, 0, 4000, regs, 1)
    assert plain.tobytes() == o.sample(7, 0, 4000, regs, 1, bits_mask("0-63")).tobytes()
    m = bits_mask("0-7,40,63")
    s = o.sample(7, 0, 4000, regs, 1, m)
    low = np.array([int(x).bit_length() - 1 for x in s["mask"]])
    assert set(low.tolist()) == {0, 1, 2, 3, 4, 5, 6, 7, 40, 63}
    assert (s["inst"] == plain["inst"]).all() and (s["target"] == plain["target"]).all()
    s4 = o.sample(7, 0, 4000, regs, 4, bits_mask("58-63"))   # a 4-bit burst starts at 58..60
    lows = {int(x & -x).bit_length() - 1 for x in s4["mask"]}
    assert lows == {58, 59, 60}
    assert bits_mask(0xF0) == 0xF0 and bits_mask(None) == 2**64 - 1


def test_device_modelled_syscalls_equal_oracle():
    """The device's modelled-syscall set (fi_trial.hip sys_class, first switch)
    is the oracle's (rv64se.c sys_modelled): a call the oracle models must not
    escape on the device."""
    import re
    from conftest import ROOT
    dev = open(os.path.join(ROOT, "shrewd_amd", "csrc", "hip", "fi_trial.hip")).read()
    ora = open(os.path.join(ROOT, "oracle", "rv64se.c")).read()
    d = dev[dev.index("__device__ int sys_class(int num)"):]
    d = d[:d.index("return 4;")]
    o = ora[ora.index("static int sys_modelled(int num)"):]
    o = o[:o.index("return 1;")]
    cases = lambda t: {int(x) for x in re.findall(r"case (\d+):", t)}
    assert cases(d) == cases(o) and 63 in cases(d)
    assert "num >= 172 && num <= 178" in dev[dev.index("__device__ int sys_class(int num)"):][:600]
