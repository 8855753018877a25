"""Rank-aware JIT cold start: the ranks of one node that load
the same workload need the same translated code objects; they queue on a lock
next to the cache file and exactly one of them runs the build
(shrewd_amd/csrc/fi_jit.cpp jit_compile / BuildLock), with the disk cache on
and in FI_CFG_JIT_NO_CACHE mode alike.  CPU only: the build goes through a
stand-in helper ($SHREWD_FI_JITC) that logs each invocation and writes a fake
code object, so no compiler and no device are involved."""
import json
import os
import stat
import subprocess
import sys
import textwrap

import pytest

from conftest import ROOT

SPLIT = "\n/*@TX_SPLIT@*/\n"
BODY = "/* 64-lane */" + SPLIT + "/* solo */" + SPLIT + SPLIT + "/* S_dispatch */"

RANK = textwrap.dedent("""
    import ctypes as C, json, os, sys, time
    sys.path.insert(0, sys.argv[1])
    from shrewd_amd import library_path
    L = C.CDLL(library_path())
    L.fi_debug_jit_build.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_uint64),
                                     C.POINTER(C.c_int), C.c_char_p, C.c_uint64]
    use_cache, calls = int(sys.argv[2]), int(sys.argv[3])
    go = float(sys.argv[4])
    while time.time() < go:      # every rank asks at about the same moment
        time.sleep(0.002)
    res = []
    for k in range(calls):
        n, cached, err = C.c_uint64(0), C.c_int(-1), C.create_string_buffer(4096)
        st = L.fi_debug_jit_build(sys.argv[5].encode(), b"gfx950", 1, use_cache, C.byref(n), C.byref(cached), err, 4096)
        res.append({"st": st, "len": n.value, "cached": cached.value, "err": err.value.decode()})
    print(json.dumps(res))
""")


def _helper(tmp_path):
    log = tmp_path / "builds.log"
    h = tmp_path / "fi_jitc_stub"
    # fi_jitc SRC OUT OPTS...: one log line per build, a slow "compile", a code object
    h.write_text("#!/bin/sh\necho $$ >> \"$FAKE_JITC_LOG\"\nsleep 1\nprintf 'CODEOBJ' > \"$2\"\n")
    h.chmod(h.stat().st_mode | stat.S_IXUSR)
    return h, log


def _ranks(tmp_path, n, use_cache, calls=1):
    import time
    h, log = _helper(tmp_path)
    env = dict(os.environ, SHREWD_FI_JITC=str(h), SHREWD_FI_JIT_CACHE=str(tmp_path / "cache"),
               FAKE_JITC_LOG=str(log))
    env.pop("SHREWD_FI_JIT_INPROC", None)
    go = time.time() + 3.0
    procs = [subprocess.Popen([sys.executable, "-c", RANK, ROOT, str(use_cache), str(calls), repr(go), BODY],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env) for _ in range(n)]
    out = []
    for p in procs:
        o, e = p.communicate(timeout=120)
        assert p.returncode == 0, e[-2000:]
        out.append(json.loads(o.strip().splitlines()[-1]))
    builds = log.read_text().split() if log.exists() else []
    return out, builds


@pytest.mark.parametrize("use_cache", [1, 0])
def test_one_build_per_node(tmp_path, use_cache):
    """8 ranks, one code object: one helper run; every rank gets its bytes.
    With the cache on the other seven report a cache hit; with it off
    (FI_CFG_JIT_NO_CACHE) they take the file another rank of this run wrote
    after they loaded, and report a cold build."""
    from shrewd_amd import build_library
    build_library()
    out, builds = _ranks(tmp_path, 8, use_cache)
    assert len(builds) == 1, builds
    flat = [r for rank in out for r in rank]
    assert all(r["st"] == 0 and r["len"] == len(b"CODEOBJ") for r in flat), flat
    hits = sorted(r["cached"] for r in flat)
    assert hits == ([0] + [1] * 7 if use_cache else [0] * 8), hits


def test_cold_start_stays_cold_in_one_process(tmp_path):
    """FI_CFG_JIT_NO_CACHE: a second build of the same code object in the
    same process runs the helper again (the file it wrote itself is not
    taken); with the cache on, a file from an earlier run is loaded."""
    from shrewd_amd import build_library
    build_library()
    out, builds = _ranks(tmp_path, 1, 0, calls=2)
    assert len(builds) == 2 and [r["cached"] for r in out[0]] == [0, 0]
    out, builds = _ranks(tmp_path, 1, 1, calls=1)
    assert len(builds) == 2 and out[0][0]["cached"] == 1       # no new build: the earlier run's file
