"""One large GP with its grid sharded across ranks (secondary mode).

The seed ensemble (ensemble.py) is the main multi-GPU mode: simulations share
nothing. This module covers the other case, a single GP whose grid is too large
or too slow for one GPU. It follows the precedent of the numba variant, which
splits the rows of X* over workers (gaussian_process_numba.py:478-503).

* Every rank holds the whole training set and builds the same factor. The factor
  is O(N^3) and small next to the grid term O(M N^2). Broadcasting L
  (8 N^2 bytes, 33.5 MB at N = 2048) over one xGMI link would cost about as much
  as computing it, so the factor is recomputed on each rank instead.
* Each rank predicts mean and variance on its own contiguous block of grid
  cells. When the grid is the reference's x-outer lattice
  (distribution.py:86-88), the blocks are cut on whole grid rows, so each block
  is a lattice too and the device's lattice cell lookup still applies.
* The blocks meet in one all_gather of ``[mu | var]`` per predict. This is RCCL
  over xGMI with the "nccl" backend, or gloo on the CPU.

A new sample that falls outside a rank's block is not one of that rank's grid
cells. Its bordered append then takes the blocked forward solve instead of the
V-column gather. The results are the same either way.
"""
from __future__ import annotations

import numpy as np


def lattice_row(X_star) -> int:
    """Cells per outer grid row if X* is in x-outer lattice order (distribution.py:86-88), else 1."""
    xs = np.asarray(X_star, dtype=np.float64).reshape(-1, 2)
    M = xs.shape[0]
    if M == 0:
        return 1
    ne = np.nonzero(xs[:, 0] != xs[0, 0])[0]
    G = int(ne[0]) if ne.size else M
    if M % G:
        return 1
    blk = xs.reshape(M // G, G, 2)
    if np.all(blk[:, :, 0] == blk[:, :1, 0]) and np.all(blk[:, :, 1] == blk[:1, :, 1]):
        return G
    return 1


def shard_cells(M: int, world: int, rank: int, row: int = 1):
    """Contiguous block [lo, hi) of the M cells for `rank`.

    Blocks are whole multiples of `row` cells and differ by at most one row.
    """
    M, world, rank, row = int(M), int(world), int(rank), max(int(row), 1)
    if M % row:
        row = 1
    rows = M // row
    base, extra = divmod(rows, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo * row, hi * row


def _gather_blocks(block, M, world, group):
    """All-gather the ranks' [2, m_r] blocks (padded to the largest one) into [2, M].
    block["data"]: this rank's block as host [2, m] (gloo), or block["mine"]: a
    device [2, mmax] tensor the predict wrote into (nccl: no host round trip before
    the collective, one device-to-host copy of the gathered blocks after it)."""
    import torch
    import torch.distributed as dist

    mmax = max(hi - lo for lo, hi in block["bounds"])
    mine = block.get("mine")
    if mine is None:
        dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
        mine = torch.zeros((2, mmax), dtype=torch.float64, device=dev)
        m = block["data"].shape[1]
        if m:
            mine[:, :m] = torch.from_numpy(block["data"]).to(dev)
    parts = torch.empty((world, 2, mmax), dtype=torch.float64, device=mine.device)
    dist.all_gather(list(parts.unbind(0)), mine, group=group)
    ph = parts.cpu().numpy()
    out = np.empty((2, M), dtype=np.float64)
    for r, (lo, hi) in enumerate(block["bounds"]):
        out[:, lo:hi] = ph[r, :, :hi - lo]
    return out


def _model_device(model):
    """The device of the model's context (MFGP_DEVICE / _lib.set_device), or None."""
    dev = getattr(model, "_dev", None)
    if dev is None:
        return None
    return int(dev().ctx.device)


def predict_block_device(model, xs_blk, mmax):
    """The posterior of `model` at the cells xs_blk written straight into a device
    tensor [2, mmax] (row 0 mean, row 1 variance; columns past the block zero) by
    the batched C ABI's device-output path: no host copy of mean / variance.

    The tensor lives on the model context's device. Its zero fill runs on torch's
    current stream and the predict on the context's own (non-blocking) stream, so
    the fill is waited for before the predict is enqueued; the predict itself
    returns synchronised, so the collective that follows on torch's stream reads
    finished data."""
    import torch

    from . import _lib

    dev = torch.device("cuda", _model_device(model))
    mine = torch.zeros((2, mmax), dtype=torch.float64, device=dev)
    if xs_blk.shape[0]:
        torch.cuda.current_stream(dev).synchronize()
        model._sync_data()
        model._push_hyp()
        model._grid_to_device(xs_blk)
        _lib.batch_predict([model._dev()], mine[0].data_ptr(), mine[1].data_ptr())
    return mine


def _current_cuda_device():
    import torch

    return torch.cuda.current_device() if torch.cuda.is_available() else None


def predict_sharded(model, X_star, world=None, rank=None, group=None):
    """``model.predict(X_star)`` with the cells split over the ranks of `group`.

    Every rank must call this with the same model state (data, hyp) and the same
    X_star. Every rank returns the full ``(mu [M,1], DiagCov)``, equal to an
    unsharded predict. With world == 1 it is a plain predict.
    """
    from .gaussian_process import DiagCov

    if world is None or rank is None:
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            world, rank = dist.get_world_size(group), dist.get_rank(group)
        else:
            world, rank = 1, 0
    if world == 1:
        return model.predict(X_star)
    xs = np.ascontiguousarray(np.asarray(X_star, dtype=np.float64).reshape(-1, 2))
    M = xs.shape[0]
    row = lattice_row(xs)
    bounds = [shard_cells(M, world, r, row) for r in range(world)]
    lo, hi = bounds[rank]
    import torch.distributed as dist

    nccl = dist.get_backend(group) == "nccl"
    if nccl and hasattr(model, "_dev") and _model_device(model) == _current_cuda_device():
        mmax = max(b - a for a, b in bounds)
        block = {"bounds": bounds, "mine": predict_block_device(model, xs[lo:hi], mmax)}
    else:
        if hi > lo:
            mu, cov = model.predict(xs[lo:hi])
            data = np.stack([np.asarray(mu, dtype=np.float64).reshape(-1), np.diag(cov)])
        else:
            data = np.empty((2, 0))
        block = {"bounds": bounds, "data": data}
    full = _gather_blocks(block, M, world, group)
    return full[0].reshape(-1, 1), DiagCov(full[1])
