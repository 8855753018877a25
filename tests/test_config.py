"""configs/fi_campaign.py, the drop-in config script: its
arguments reach the FaultCampaign SimObject's params under gem5.opt and the
ctypes mirror otherwise -- Process.input / Process.executable included
(src/sim/Process.py:44,69; src/gem5ext/FaultCampaign.py:33-37)."""
import importlib.util
import json
import os
import subprocess
import sys
import types

import numpy as np
import pytest

from conftest import ROOT, workload_elf

CFG = os.path.join(ROOT, "configs", "fi_campaign.py")


def _load_config():
    spec = importlib.util.spec_from_file_location("fi_campaign_cfg", CFG)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


ARGS = ["--workload", "w.elf", "--cmd", "w,x", "--input", "in.txt", "--executable", "/opt/w", "--trials", "7",
        "--seed", "0x1234", "--structures", "int_reg,pc", "--protect-mask", "0x6", "--max-insts-factor", "3",
        "--cpu-type", "timing"]


def test_arguments_reach_the_simobject(monkeypatch):
    """Under gem5.opt: every argument becomes a FaultCampaign param."""
    cfg = _load_config()
    seen = {}

    class FakeCampaign:
        def __init__(self, **kw):
            seen.update(kw)

        def run(self):
            seen["ran"] = True

        def summaryJson(self):
            return "{}"

        def histogram(self):
            return []

    class FakeRoot:
        def __init__(self, full_system, campaign):
            self.campaign = campaign

    m5 = types.ModuleType("m5")
    m5.instantiate = lambda: None
    objs = types.ModuleType("m5.objects")
    objs.FaultCampaign, objs.Root = FakeCampaign, FakeRoot
    m5.objects = objs
    monkeypatch.setitem(sys.modules, "m5", m5)
    monkeypatch.setitem(sys.modules, "m5.objects", objs)
    cfg.run_gem5(cfg.parse(ARGS))
    assert seen["ran"]
    assert seen["input"] == "in.txt" and seen["executable"] == "/opt/w"
    assert seen["workload"] == "w.elf" and seen["cmd"] == ["w", "x"] and seen["trials"] == 7
    assert seen["seed"] == 0x1234 and seen["structures"] == ["int_reg", "pc"] and seen["protect_mask"] == 6
    assert seen["max_insts_factor"] == 3.0 and seen["cpu_type"] == "timing"
    # defaults: the host's stdin, the workload path, numInst sites
    seen.clear()
    cfg.run_gem5(cfg.parse(["--workload", "w.elf"]))
    assert seen["input"] == "cin" and seen["executable"] == "" and seen["cpu_type"] == "atomic"


def test_arguments_reach_the_ctypes_mirror(monkeypatch):
    """Without gem5: the same arguments reach shrewd_amd.FaultCampaign."""
    cfg = _load_config()
    import shrewd_amd
    seen = {}

    class FakeCampaign:
        def __init__(self, workload, **kw):
            seen.update(kw, workload=workload)

        def run(self, first_trial=0):
            seen["first_trial"] = first_trial

        def summary(self):
            return {"trials": 7}

    monkeypatch.setattr(shrewd_amd, "FaultCampaign", FakeCampaign)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    cfg.run_ctypes(cfg.parse(ARGS))
    assert seen["input"] == "in.txt" and seen["executable"] == "/opt/w"
    assert seen["workload"] == "w.elf" and seen["cmd"] == ["w", "x"] and seen["trials"] == 7
    assert seen["cpu_type"] == "timing"
    seen.clear()
    cfg.run_ctypes(cfg.parse(["--workload", "w.elf"]))
    assert seen["input"] == "cin" and seen["executable"] is None and seen["cpu_type"] == "atomic"


@pytest.mark.gpu
def test_config_script_with_input_file(tmp_path, oracle_mod):
    """The script end to end on the GPU with an input file: hello's fd-0
    trials are classified (no host escapes: write(0) on the O_RDONLY input
    returns -EBADF) and the histogram equals the ctypes FaultCampaign's with
    the same input; the oracle agrees on the sampled sites."""
    elf = tmp_path / "hello.elf"
    elf.write_bytes(workload_elf("hello"))
    inp = tmp_path / "in.txt"
    inp.write_bytes(b"some input\n")
    out = tmp_path / "cfg"
    r = subprocess.run([sys.executable, CFG, "--workload", str(elf), "--cmd", "hello", "--input", str(inp),
                        "--trials", "2000", "--seed", "0x5EED0001", "--structures", "int_reg",
                        "--output", str(out)], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    s = json.loads(r.stdout.strip().splitlines()[-1])
    assert s["trials"] == 2000
    from shrewd_amd import FaultCampaign
    c = FaultCampaign(str(elf), cmd=["hello"], trials=2000, seed=0x5EED0001, structures=["int_reg"], input=str(inp))
    dev = c.run()
    assert np.array_equal(np.load(str(out) + ".npy"), dev)
    sites = c.engine.sample(0, 2000)
    o = oracle_mod.Oracle(workload_elf("hello"), "hello")
    o.set_stdin(b"some input\n")
    o.run_golden()
    ref = o.run_trials(sites, protect_mask=0)
    assert np.array_equal(dev, ref)
    # the host escapes left are write lengths >= 2 GiB (a flipped a2), not fd 0
    host = (dev["cls"] == 5) & (dev["sub"] == 4)
    assert s["escape_sub"].get("host", 0) == int(host.sum())
    assert (sites["target"][host] == 12).all() and (sites["mask"][host] >= 1 << 31).all()
