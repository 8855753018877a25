"""Builds the in-tree HIP extension shrewd_amd/_lib/libshrewd_fi.so for gfx950."""
from __future__ import annotations

import os
import subprocess

ROOT = os.path.dirname(os.path.abspath(__file__))
SRCS = [os.path.join(ROOT, "csrc", "hip", "fi_kernels.hip"), os.path.join(ROOT, "csrc", "hip", "fi_trial.hip"),
        os.path.join(ROOT, "csrc", "fi_engine.cpp")]
DEPS = SRCS + [os.path.join(ROOT, "csrc", "fi_types.h"), os.path.join(ROOT, "csrc", "hip", "rv64_isa.h"),
               os.path.join(ROOT, "csrc", "hip", "fi_device.h"),
               os.path.join(ROOT, "csrc", "gem5_decode_table.h"),
               os.path.join(os.path.dirname(ROOT), "include", "fi_engine.h")]
REPO = os.path.dirname(ROOT)
CLI_SRCS = [os.path.join(REPO, "src", "campaign", "campaign.cc"),
            os.path.join(REPO, "src", "campaign", "fi_campaign_main.cc")]
CLI_DEPS = CLI_SRCS + [os.path.join(REPO, "src", "campaign", "campaign.hh")]
CLI_OUT = os.path.join(ROOT, "_lib", "fi_campaign")
OUT = os.path.join(ROOT, "_lib", "libshrewd_fi.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def needs_build(out: str = OUT) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(p) > t for p in DEPS if os.path.exists(p))


def build(force: bool = False, out: str = OUT, extra: list[str] | None = None) -> str:
    if not force and not needs_build(out):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-shared", "-std=c++17", "-Wall",
           # keep wave-uniform branch trees as scalar branches (no flow-block chains)
           "-mllvm", "-structurizecfg-skip-uniform-regions=true",
           "-o", out + ".tmp"] + (extra or []) + SRCS
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def build_cli(force: bool = False) -> str:
    """Native campaign driver (src/campaign) linked against the engine library."""
    lib = build(force=force)
    if not force and os.path.exists(CLI_OUT) and all(
            os.path.getmtime(p) <= os.path.getmtime(CLI_OUT) for p in CLI_DEPS + [lib]):
        return CLI_OUT
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-Wall", "-o", CLI_OUT + ".tmp"] + CLI_SRCS + [
        "-L" + os.path.dirname(lib), "-lshrewd_fi", "-Wl,-rpath,$ORIGIN", "-pthread"]
    subprocess.run(cmd, check=True)
    os.replace(CLI_OUT + ".tmp", CLI_OUT)
    return CLI_OUT


if __name__ == "__main__":
    print(build(force=True))
    print(build_cli())
