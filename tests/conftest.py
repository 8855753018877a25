import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

WORKLOADS = ["hello", "crc32", "qsort", "intmix", "fpamo", "crcblk"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) -- runs through the C ABI")
    config.addinivalue_line("markers", "slow: long-running")


def workload_elf(name: str) -> bytes:
    with open(os.path.join(ROOT, "workloads", f"{name}.elf"), "rb") as f:
        return f.read()


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import pyoracle
    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def engine_factory():
    """Builds the HIP library (if stale) and returns a factory of loaded engines."""
    import torch  # noqa: F401  (device visibility check goes through HIP itself)
    from shrewd_amd import Engine, build_library
    build_library()

    cache = {}

    def make(name, argv0=None, **kw):
        key = (name, argv0, tuple(sorted(kw.items())))
        if key not in cache:
            e = Engine(**kw)
            e.load_elf(workload_elf(name), [argv0 or name])
            e.golden_run()
            cache[key] = e
        return cache[key]

    yield make
    for e in cache.values():
        e.close()


def np_histogram(sites, outcomes):
    """Host restatement of fi_hist_kernel (test-side checker only)."""
    import numpy as np
    from shrewd_amd.fi import HIST_DT, N_STRUCT
    h = np.zeros(1, HIST_DT)[0]
    t = np.where(sites["target"] < N_STRUCT, sites["target"], 0).astype(np.int64)
    m = sites["mask"].astype(np.uint64)
    bit = np.zeros(len(m), np.int64)
    nz = m != 0
    low = m[nz] & (~m[nz] + np.uint64(1))
    bit[nz] = np.log2(low.astype(np.float64)).round().astype(np.int64)
    cls = np.where(outcomes["cls"] < 6, outcomes["cls"], 5).astype(np.int64)
    np.add.at(h["counts"], (t, bit, cls), 1)
    np.add.at(h["crash_sub"], (outcomes["sub"][cls == 2] & 15).astype(np.int64), 1)
    np.add.at(h["escape_sub"], (outcomes["sub"][cls == 5] & 7).astype(np.int64), 1)
    h["trials"] = len(sites)
    h["guest_insts"] = int(outcomes["ninst"].astype(np.uint64).sum())
    return h
