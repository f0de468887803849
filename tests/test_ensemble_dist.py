"""Multi-process (gloo, world_size 2, CPU) coverage of the seed-sharded ensemble
path: sharding and the single all_gather + per-iteration mean/std
(runner.py:131-147, analysis.py:66-73)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mfgp_coverage_amd.ensemble import gather_trajectories, shard_seeds


def test_shard_seeds_partition():
    for total in (1, 7, 8, 64, 65):
        for world in (1, 2, 3, 8):
            parts = [shard_seeds(total, world, r) for r in range(world)]
            flat = [s for p in parts for s in p]
            assert flat == list(range(total))
            assert max(map(len, parts)) - min(map(len, parts)) <= 1


def _traj(seed, T):
    return np.random.default_rng(seed).random(T)


def _worker(rank, world, port, T, S, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seeds = shard_seeds(S, world, rank)
    traj = torch.tensor(np.stack([_traj(s, T) for s in seeds])) if seeds else torch.zeros((0, T), dtype=torch.float64)
    allt, mean, std = gather_trajectories(traj, world)
    if rank == 0:
        out_q.put((allt.numpy(), mean.numpy(), std.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,S", [(2, 6), (3, 7), (8, 100), (3, 2)])
def test_gather_trajectories_gloo(world, S):
    """Even and uneven shards: 7 seeds over 3 ranks (3/2/2), the reference's
    default 100 simulations (runner.py:85) over 8 ranks (13/12), and a rank with
    no seeds at all (2 over 3)."""
    T = 12
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, T, S, q)) for r in range(world)]
    for p in procs:
        p.start()
    allt, mean, std = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = np.stack([_traj(s, T) for s in range(S)])
    np.testing.assert_array_equal(allt, ref)
    np.testing.assert_allclose(mean, ref.mean(0), rtol=1e-14)
    np.testing.assert_allclose(std, ref.std(0, ddof=1), rtol=1e-12)
