"""CPU checks of the product library: builds for gfx950, loads, exports the ABI."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def header_functions():
    names = []
    for h in ("fi_engine.h", "fi_debug.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        names += re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(fi_\w+)\s*\(", txt, flags=re.M)
    return sorted(set(names))


def test_library_builds_and_exports_every_declared_symbol():
    from shrewd_amd import build_library
    path = build_library()
    assert os.path.exists(path)
    lib = ctypes.CDLL(path)
    fns = header_functions()
    assert "fi_run_trials" in fns and "fi_golden_run" in fns and len(fns) >= 15
    for f in fns:
        assert hasattr(lib, f), f"{f} declared in include/ but not exported"


def test_code_object_targets_gfx950():
    from shrewd_amd import build_library
    data = open(build_library(), "rb").read()
    assert b"gfx950" in data


def test_engine_refuses_without_device(monkeypatch):
    """No GPU here: the product must fail loudly rather than fall back to CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from shrewd_amd import Engine, EngineError
    with pytest.raises(EngineError):
        Engine()


def test_structures_mask():
    from shrewd_amd import structures_mask
    assert structures_mask(["int_reg"]) == ((1 << 32) - 2)
    assert structures_mask(["pc", "mem"]) == (1 << 32) | (1 << 33)
    assert structures_mask(["a0", "sp", "x5"]) == (1 << 10) | (1 << 2) | (1 << 5)


def test_native_driver_refuses_without_device():
    """The C++ campaign driver (src/campaign) builds, links the engine and, with
    no GPU visible, fails loudly instead of computing anything on the CPU."""
    import subprocess
    import torch
    from shrewd_amd import build as b
    if torch.cuda.is_available():
        pytest.skip("GPU visible")
    exe = b.build_cli()
    r = subprocess.run([exe, "--workload", os.path.join(ROOT, "workloads", "hello.elf"), "--trials", "8"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "no HIP device" in r.stderr


def test_structures_mask_names():
    from shrewd_amd import structures_mask
    assert structures_mask(["int_reg", "pc"]) == 0x1FFFFFFFE
    assert structures_mask(["a0", "x5", "mem"]) == (1 << 10) | (1 << 5) | (1 << 33)


def test_native_driver_names_every_subcode():
    """Every crash / escape sub-code of include/fi_engine.h has the Python
    mirror's name in src/campaign/campaign.cc (its JSON keys)."""
    from shrewd_amd.fi import CRASH_NAMES, ESCAPE_NAMES
    src = open(os.path.join(ROOT, "src", "campaign", "campaign.cc")).read()
    for name in list(CRASH_NAMES.values()) + list(ESCAPE_NAMES.values()):
        assert f'"{name}"' in src, name
