import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

WORKLOADS = ["hello", "crc32", "qsort", "intmix"]


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
