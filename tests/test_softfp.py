"""The engine's IEEE arithmetic port (shrewd_amd/csrc/hip/fi_softfp.h) pinned
against the reference's own SoftFloat (gem5 ext/softfloat, RISC-V
specialization, compiled into oracle/_ref by oracle/softfloat_ref.mk): every
operation gem5's F/D/Zfh instructions call, in binary16/32/64, in all five
rounding modes, on edge operands (zeros, subnormal extremes, min normal, max
finite, infinities, quiet and signalling NaNs, values around 1 and around the
rounding boundaries) crossed with each other and on random operands with
clustered exponents; result bits and exception flags must both match.

The CPU tests run the host build of the port; the GPU test runs the same
vectors through the device build (the code the trial kernel executes)."""
import numpy as np
import pytest

from oracle import pyoracle

OPS = {"add": 0, "sub": 1, "mul": 2, "div": 3, "sqrt": 4, "fma": 5, "eq": 6, "lt": 7, "le": 8, "ltq": 9, "leq": 10,
       "to_i32": 11, "to_u32": 12, "to_i64": 13, "to_u64": 14, "from_i32": 15, "from_u32": 16, "from_i64": 17,
       "from_u64": 18, "to_h": 19, "to_s": 20, "to_d": 21, "rint": 22, "rintx": 23}
FMTS = {"h": (0, 5, 10), "s": (1, 8, 23), "d": (2, 11, 52)}
ARITY = {"sqrt": 1, "fma": 3, "rint": 1, "rintx": 1}

pytestmark = pytest.mark.skipif(not pyoracle.has_softfloat(),
                                reason="oracle built without the reference SoftFloat (oracle/_ref)")


def edge_values(eb, mb):
    w = 1 + eb + mb
    sign = 1 << (w - 1)
    emax = (1 << eb) - 1
    bias = (1 << (eb - 1)) - 1
    frac = (1 << mb) - 1
    v = [0, 1, 2, frac >> 1, frac, 1 << mb, (1 << mb) | 1, ((emax - 1) << mb) | frac, (emax - 1) << mb,
         emax << mb, (emax << mb) | 1, (emax << mb) | (1 << (mb - 1)), (emax << mb) | frac,
         bias << mb, (bias << mb) | 1, ((bias - 1) << mb) | frac, (bias + 1) << mb, ((bias + 1) << mb) | frac,
         (bias + mb) << mb, ((bias + mb) << mb) | frac, (bias + mb + 1) << mb, ((bias + 31) << mb),
         ((bias + 32) << mb) | frac, (bias + 63) << mb, (bias + 64) << mb, ((bias - mb) << mb) | 3,
         (1 << mb) - 3, ((bias >> 1) << mb) | 5]
    v = [x for x in v if x < (1 << (w - 1))]
    return np.array(sorted(set(v + [x | sign for x in v])), np.uint64)


def random_values(rng, n, eb, mb):
    w = 1 + eb + mb
    emax = (1 << eb) - 1
    bias = (1 << (eb - 1)) - 1
    s = rng.integers(0, 2, n, dtype=np.uint64) << np.uint64(w - 1)
    # exponents: uniform, clustered around the bias, and near both ends
    pick = rng.integers(0, 4, n)
    e = np.where(pick == 0, rng.integers(0, emax + 1, n),
                 np.where(pick == 1, bias + rng.integers(-mb - 3, mb + 4, n),
                          np.where(pick == 2, rng.integers(0, mb + 3, n), emax - rng.integers(0, 4, n))))
    e = np.clip(e, 0, emax).astype(np.uint64)
    m = rng.integers(0, 1 << mb, n, dtype=np.uint64)
    # some mantissas with long runs of ones / zeros (rounding boundaries)
    runs = rng.integers(0, 3, n)
    m = np.where(runs == 0, m, np.where(runs == 1, m | np.uint64((1 << mb) - 1) >> rng.integers(0, mb, n).astype(np.uint64),
                                        m & ~(np.uint64((1 << mb) - 1) >> rng.integers(0, mb, n).astype(np.uint64))))
    return s | (e << np.uint64(mb)) | (m & np.uint64((1 << mb) - 1))


def int_values(rng, n):
    edge = np.array([0, 1, 2, 3, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFF, 0x100000000, 0x7FFFFFFFFFFFFFFF,
                     0x8000000000000000, 0xFFFFFFFFFFFFFFFF, 0xFFFFFFFF80000000, 0x1FFFFFFFFFFFFF, 0x20000000000001,
                     0xFFFFFF, 0x1000001, 0x7FF, 0x801, 0xFFFFFFFFFFFFFFFE], np.uint64)
    r = rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True)
    sh = rng.integers(0, 64, n).astype(np.uint64)
    return np.concatenate([edge, r >> sh, r])


def operands(name, fmt, rng, n_rand):
    _, eb, mb = FMTS[fmt]
    if name.startswith("from_"):
        a = int_values(rng, n_rand)
        return a, a, a
    ed = edge_values(eb, mb)
    ar = ARITY.get(name, 2)
    if ar == 1 or name.startswith("to_"):
        a = np.concatenate([ed, random_values(rng, n_rand, eb, mb)])
        return a, a, a
    ea, eb2 = np.meshgrid(ed, ed)
    a = np.concatenate([ea.ravel(), random_values(rng, n_rand, eb, mb)])
    b = np.concatenate([eb2.ravel(), random_values(rng, n_rand, eb, mb)])
    if ar == 3:
        c = np.concatenate([np.resize(ed, ea.size), random_values(rng, n_rand, eb, mb)])
        # exact-cancellation cases: c = -(a * b) for small products
        k = min(2000, len(a))
        prod, _ = pyoracle.sf_ref(OPS["mul"], FMTS[fmt][0], 0, a[:k], b[:k])
        c[:k // 2] = prod[:k // 2] ^ np.uint64(1 << (eb + mb))
        return a, b, c
    return a, b, a


def check(name, fmt, rm, device=False, n_rand=20000, seed=0):
    from shrewd_amd.fi import softfp
    rng = np.random.default_rng(seed + 131 * OPS[name] + 7 * FMTS[fmt][0] + rm)
    a, b, c = operands(name, fmt, rng, n_rand)
    ref, rfl = pyoracle.sf_ref(OPS[name], FMTS[fmt][0], rm, a, b, c)
    got, gfl = softfp(OPS[name], FMTS[fmt][0], rm, a, b, c, device=device)
    bad = np.nonzero((ref != got) | (rfl != gfl))[0]
    if len(bad):
        i = bad[0]
        raise AssertionError(f"{name}.{fmt} rm={rm}: {len(bad)}/{len(a)} differ, first: a={int(a[i]):#x} "
                             f"b={int(b[i]):#x} c={int(c[i]):#x} ref={int(ref[i]):#x}/{int(rfl[i]):#x} "
                             f"port={int(got[i]):#x}/{int(gfl[i]):#x}")
    return len(a)


@pytest.mark.parametrize("fmt", list(FMTS))
@pytest.mark.parametrize("name", [k for k in OPS if not k.startswith("to_") or k in ("to_i32", "to_u32", "to_i64",
                                                                                       "to_u64")])
def test_port_matches_reference(name, fmt):
    for rm in range(5):
        check(name, fmt, rm)


@pytest.mark.parametrize("src", list(FMTS))
@pytest.mark.parametrize("dst", ["to_h", "to_s", "to_d"])
def test_conversions_match_reference(src, dst):
    if dst == "to_" + src:
        pytest.skip("same format")
    for rm in range(5):
        check(dst, src, rm)


@pytest.mark.gpu
def test_device_port_matches_reference():
    """The device build of the port (what the trial kernel runs) on the same vectors."""
    n = 0
    for fmt in FMTS:
        for name in OPS:
            if name in ("to_h", "to_s", "to_d") and name == "to_" + fmt:
                continue
            for rm in range(5):
                n += check(name, fmt, rm, device=True, n_rand=4000)
    assert n > 100000
