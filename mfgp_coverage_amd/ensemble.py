"""Seed-sharded Monte-Carlo ensembles across GPUs (one process per GPU).

The reference runs its S Monte-Carlo simulations as ``Pool(n).map(run_sim)``
(runner.py:131-141) and concatenates the per-simulation logs in the parent
(runner.py:144-147); the per-iteration mean / std over simulations is then taken
by analysis.py:66-73 (``groupby("Iteration").mean()/.std()``). Here every rank
owns a contiguous slice of the seeds, runs them as one batched GP per step, and
the per-seed trajectories (loss, VarMax, ...) meet in ONE all_gather at the end
(RCCL over xGMI with the "nccl" backend; gloo on CPU for the tests). There is
no collective on the data path: the simulations share nothing.
"""
from __future__ import annotations


def shard_seeds(total_seeds: int, world: int, rank: int):
    """Contiguous block of seeds for `rank` (sizes differ by at most one)."""
    base, extra = divmod(int(total_seeds), int(world))
    start = rank * base + min(rank, extra)
    return list(range(start, start + base + (1 if rank < extra else 0)))


def gather_trajectories(traj, world: int, group=None):
    """All-gather per-seed trajectories and aggregate them per iteration.

    traj: tensor [seeds_on_this_rank, iterations]. The seed counts may differ
    between ranks (``shard_seeds`` of 100 seeds over 8 ranks gives 13 or 12, and a
    rank may hold none); the iteration count must be the same on every rank.
    Returns (all [total_seeds, iterations] in rank order, mean [iterations],
    std [iterations]) -- the analysis.py:66-73 statistics (pandas' std is the
    sample std, ddof = 1).

    Two collectives: the per-rank seed counts, then the blocks padded to the
    largest one (all_gather needs equal shapes).
    """
    import torch
    import torch.distributed as dist

    if world > 1:
        n = torch.tensor([traj.shape[0]], dtype=torch.int64, device=traj.device)
        counts = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(counts, n, group=group)
        counts = [int(c.item()) for c in counts]
        rows = max(counts)
        pad = traj.new_zeros((rows,) + tuple(traj.shape[1:]))
        pad[:traj.shape[0]] = traj
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad, group=group)
        allt = torch.cat([p[:c] for p, c in zip(parts, counts)], 0)
    else:
        allt = traj
    mean = allt.mean(0)
    std = allt.std(0, unbiased=True) if allt.shape[0] > 1 else torch.full_like(mean, float("nan"))
    return allt, mean, std

