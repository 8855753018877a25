"""Multi-process (world size 2, gloo, CPU) test of the campaign's sharding and
its only exchange step, the outcome-histogram all-reduce
(shrewd_amd.fi.shard_range / allreduce_histogram).  Trial
outcomes come from the oracle here (no GPU); on the GPU box the same two
functions run with RCCL."""
import os
import socket
import tempfile

import numpy as np
import torch.multiprocessing as mp

from conftest import ROOT, np_histogram, workload_elf

SEED, TRIALS, STRUCT = 0x5EED0001, 301, ((1 << 32) - 2) | (1 << 32)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, outdir):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from oracle.pyoracle import Oracle
    from shrewd_amd.fi import allreduce_histogram, shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        o = Oracle(workload_elf("crc32"), "crc32")
        o.run_golden()
        first, n = shard_range(TRIALS, world, rank)
        sites = o.sample(SEED, first, n, STRUCT, 1)
        out = o.run_trials(sites, threads=2)
        h = allreduce_histogram(np_histogram(sites, out))
        np.save(os.path.join(outdir, f"hist{rank}.npy"), np.frombuffer(h.tobytes(), np.uint8))
        np.save(os.path.join(outdir, f"out{rank}.npy"), out)
        o.close()
    finally:
        dist.destroy_process_group()


def test_shard_ranges_partition():
    from shrewd_amd.fi import shard_range
    for total in (0, 1, 7, 100_000, 1_000_000):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0
            assert all(a[0] + a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert sum(c for _, c in spans) == total
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def test_two_rank_histogram_allreduce(oracle_mod):
    from shrewd_amd.fi import HIST_DT
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rank_main, args=(world, _free_port(), d), nprocs=world, join=True)
        hists = [np.frombuffer(np.load(os.path.join(d, f"hist{r}.npy")).tobytes(), HIST_DT)[0] for r in range(world)]
        outs = np.concatenate([np.load(os.path.join(d, f"out{r}.npy")) for r in range(world)])
    # every rank holds the same reduced histogram ...
    assert hists[0].tobytes() == hists[1].tobytes()
    # ... equal to the single-process campaign over all trial ids
    o = oracle_mod.Oracle(workload_elf("crc32"), "crc32")
    o.run_golden()
    sites = o.sample(SEED, 0, TRIALS, STRUCT, 1)
    ref = o.run_trials(sites, threads=4)
    o.close()
    assert outs.tobytes() == ref.tobytes()
    assert hists[0].tobytes() == np_histogram(sites, ref).tobytes()
    assert int(hists[0]["trials"]) == TRIALS


def test_engine_two_ranks_one_gpu_script_is_cpu_importable():
    """The rank script of the GPU test below imports on CPU (no work at import)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("dist_engine_rank", os.path.join(ROOT, "tests", "dist_engine_rank.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert callable(mod.main)


import pytest  # noqa: E402


@pytest.mark.gpu
def test_engine_two_ranks_one_gpu(tmp_path):
    """The product's multi-rank path on one GPU: two processes (gloo, both on
    device 0), each FaultCampaign.run(num_gpus=2) over its contiguous shard of
    the trial ids, the outcome histogram all-reduced.  The ranks' outcomes in
    shard order and the reduced histogram equal a single-process run of the
    same campaign."""
    import subprocess
    import sys
    from shrewd_amd.fi import HIST_DT, FaultCampaign
    trials, seed, world = 3001, 0x5EED2222, 2
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dist_engine_rank.py"),
                                       str(tmp_path), str(trials), hex(seed)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    logs = [p.communicate(timeout=240)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), logs
    outs = [np.load(tmp_path / f"out{r}.npy") for r in range(world)]
    hists = [np.frombuffer(np.load(tmp_path / f"hist{r}.npy").tobytes(), HIST_DT)[0] for r in range(world)]
    firsts = [int((tmp_path / f"first{r}.txt").read_text()) for r in range(world)]
    assert firsts == [0, len(outs[0])] and len(outs[0]) + len(outs[1]) == trials
    assert hists[0].tobytes() == hists[1].tobytes()
    fc = FaultCampaign(os.path.join(ROOT, "workloads", "crc32.elf"), cmd=["crc32"], trials=trials, seed=seed,
                       structures=("int_reg", "pc"))
    ref = fc.run()
    h = fc.histogram()
    fc.engine.close()
    assert np.concatenate(outs).tobytes() == ref.tobytes()
    for f in ("counts", "crash_sub", "escape_sub", "trials", "guest_insts"):
        assert np.array_equal(hists[0][f], h[f]), f
