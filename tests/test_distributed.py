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
