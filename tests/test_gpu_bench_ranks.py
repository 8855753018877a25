"""bench.py's own multi-rank path (one process per GPU, launched by
torch.distributed.run as the driver does for N > 1), rehearsed with two ranks
on device 0 and the histogram reduce over gloo: the reduced histogram equals a
one-process run of both shards, and rank 0's line reports n_gpus 2 with the
value over both shards.  (RCCL itself needs two GPUs; the driver's 8-GPU
run exercises it.)"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

T = 4000


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


def test_bench_two_ranks_gloo(tmp_path):
    from shrewd_amd.fi import HIST_DT
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    common = ["--steps", "2", "--warmup", "1", "--workloads", "", "--no-cpu-baseline"]
    h2 = str(tmp_path / "h2.npy")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--trials", str(T), "--dist-backend", "gloo", "--device-index", "0",
                        "--hist-out", h2] + common,
                       capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    two = _line(r.stdout)
    h1 = str(tmp_path / "h1.npy")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--trials", str(2 * T), "--hist-out", h1]
                       + common, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    one = _line(r.stdout)
    a, b = np.load(h2).astype(HIST_DT)[0], np.load(h1).astype(HIST_DT)[0]
    for f in ("counts", "crash_sub", "escape_sub", "trials", "guest_insts"):
        assert np.array_equal(a[f], b[f]), f
    assert int(a["trials"]) == 2 * T
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["outcomes"] == one["outcomes"]
    # value = trials of both shards over the max-over-ranks time of the steps
    assert abs(two["value"] * two["ms_per_step"] / 1e3 - 2 * T) < 1e-6 * 2 * T
    assert "x2" in two["config"]["parallelism"]
