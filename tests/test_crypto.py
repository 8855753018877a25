"""The engine's scalar-crypto port (shrewd_amd/csrc/hip/fi_crypto.h) pinned
against the reference's own helpers (src/arch/riscv/rvk.hh, compiled into
oracle/_ref by oracle/rvk_ref.mk): every Zkn/Zks/Zbkb/Zbkx function gem5's
RV64 decoder reaches, every RNUM / BS variant, on edge operands (zero, all
ones, sign boundaries, single bits) and random operands.

The CPU test runs the host build of the port; the GPU test runs the same
vectors through the device build (the code the trial kernel executes)."""
import numpy as np
import pytest

from oracle import pyoracle

pytestmark = pytest.mark.skipif(not pyoracle.has_rvk(),
                                reason="oracle built without the reference's rvk.hh (oracle/_ref)")

# fi_crypto.h numbering; RNUM (aes64ks1i) and BS (sm4ed / sm4ks) in bits 8+
FUNCS = [*range(0, 11), *[11 | (r << 8) for r in range(16)], 12, *[13 | (bs << 8) for bs in range(4)],
         *[14 | (bs << 8) for bs in range(4)], *range(15, 22)]


def operands(seed=7, n=4096):
    rng = np.random.default_rng(seed)
    edge = [0, 1, 0x7F, 0x80, 0xFF, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFF, 0x100000000, 0x7FFFFFFFFFFFFFFF,
            0x8000000000000000, 0xFFFFFFFFFFFFFFFF, 0x0123456789ABCDEF, 0xFEDCBA9876543210]
    edge += [1 << k for k in range(64)]
    e = np.array(edge, np.uint64)
    a = np.concatenate([np.repeat(e, len(e)), rng.integers(0, 2**64, n, dtype=np.uint64)])
    b = np.concatenate([np.tile(e, len(e)), rng.integers(0, 2**64, n, dtype=np.uint64)])
    return a, b


def _check(device):
    from shrewd_amd.fi import crypto
    a, b = operands()
    for fn in FUNCS:
        ref = pyoracle.rvk_ref(fn, a, b)
        got = crypto(fn, a, b, device=device)
        bad = np.nonzero(ref != got)[0]
        assert len(bad) == 0, (f"fn {fn & 0xFF} sub {fn >> 8}: {len(bad)} mismatches, first a={int(a[bad[0]]):#x} "
                               f"b={int(b[bad[0]]):#x} ref={int(ref[bad[0]]):#x} got={int(got[bad[0]]):#x}")


def test_crypto_port_matches_reference_host():
    _check(device=False)


@pytest.mark.gpu
def test_crypto_port_matches_reference_device():
    _check(device=True)
