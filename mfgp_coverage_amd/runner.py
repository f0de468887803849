"""Seed-sharded simulation runner with the reference's log schemas.

The reference's runner (runner.py:72-161) maps ``run_sim`` over
``simulations`` seeds with ``multiprocessing.Pool`` and concatenates the
per-simulation logs in seed order before writing ``<out>_loss.csv``,
``<out>_agent.csv`` and ``<out>_sample.csv`` (the dict schemas of
simulator.py:918-931). Here one process per GPU owns a contiguous block of
seeds (``ensemble.shard_seeds``); each process runs its simulations (e.g. the
reference's ``run_sim`` with this package's SFGP/MFGP as the GP classes) and the
logs meet on rank 0 over the process group (RCCL over
xGMI with the "nccl" backend, gloo on CPU): the records are encoded as float64
columns in the reference's column order, so the exchange is two plain tensor
all_gathers for the three logs (row counts, then the packed rows). Rank 0 then writes the same CSVs and can summarise losses the way
analysis.py:62-73 does.
"""
from __future__ import annotations

import numpy as np

from .ensemble import shard_seeds

# simulator.py:918-931 (key order of the logged dicts)
LOSS_COLUMNS = ("SimNum", "Iteration", "Period", "Fidelity", "Loss")
AGENT_COLUMNS = ("SimNum", "Iteration", "Period", "Fidelity", "Agent", "X", "Y", "XMax", "YMax", "VarMax", "Var0",
                 "XCentroid", "YCentroid", "ProbExplore", "Explore", "Distance")
SAMPLE_COLUMNS = ("SimNum", "Iteration", "Period", "Fidelity", "Agent", "X", "Y", "Sample")
SCHEMAS = (LOSS_COLUMNS, AGENT_COLUMNS, SAMPLE_COLUMNS)
_FIDELITY = {"S": 0.0, "M": 1.0}
_FIDELITY_INV = {0.0: "S", 1.0: "M"}
_INT_COLUMNS = ("SimNum", "Iteration", "Period")


def encode(records, columns):
    """list of log dicts -> float64 [rows, len(columns)] (missing keys -> NaN)."""
    out = np.full((len(records), len(columns)), np.nan, dtype=np.float64)
    for i, rec in enumerate(records):
        for j, c in enumerate(columns):
            if c in rec:
                v = rec[c]
                out[i, j] = _FIDELITY[v] if c == "Fidelity" else float(np.asarray(v).reshape(-1)[0])
    return out


def decode(arr, columns):
    """float64 [rows, cols] -> DataFrame in the reference's column order and types."""
    import pandas as pd
    df = pd.DataFrame(np.asarray(arr, dtype=np.float64).reshape(-1, len(columns)), columns=list(columns))
    if "Fidelity" in df:
        df["Fidelity"] = df["Fidelity"].map(_FIDELITY_INV)
    for c in _INT_COLUMNS:
        if c in df and not df[c].isna().any():
            df[c] = df[c].astype(np.int64)
    if "Agent" in df and columns is AGENT_COLUMNS and not df["Agent"].isna().any():
        df["Agent"] = df["Agent"].astype(np.int64)
    return df.dropna(axis=1, how="all")


def gather_tables(arrs, world, group=None, device=None):
    """All-gather several [rows, cols] float64 blocks per rank (row counts may differ
    between ranks and blocks) -> for each block, the rows of every rank concatenated
    in rank order (every rank gets them). Two collectives in all: the row counts,
    then every block padded to its largest count and packed into one flat tensor."""
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in arrs]
    if world <= 1:
        return arrs
    import torch
    import torch.distributed as dist
    dev = device if device is not None else "cpu"
    n = torch.tensor([a.shape[0] for a in arrs], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = torch.stack(counts).cpu().numpy()            # [world, blocks]
    rows = counts.max(axis=0)
    sizes = [int(r) * a.shape[1] for r, a in zip(rows, arrs)]
    flat = torch.full((sum(sizes),), float("nan"), dtype=torch.float64, device=dev)
    off = 0
    for a, sz in zip(arrs, sizes):
        if a.size:
            flat[off:off + a.size] = torch.from_numpy(a.reshape(-1)).to(dev)
        off += sz
    parts = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(parts, flat, group=group)
    parts = [p.cpu().numpy() for p in parts]
    out, off = [], 0
    for b, (a, sz) in enumerate(zip(arrs, sizes)):
        cols = a.shape[1]
        out.append(np.concatenate([p[off:off + counts[r, b] * cols].reshape(-1, cols) for r, p in enumerate(parts)],
                                  axis=0))
        off += sz
    return out


def gather_table(arr, world, group=None, device=None):
    """One block of gather_tables."""
    return gather_tables([arr], world, group, device)[0]


def run(sim_fn, simulations, world=1, rank=0, group=None, device=None, out_name=None):
    """Run sim_fn(sim_num) -> (loss_log, agent_log, sample_log) for this rank's seeds,
    gather the logs (seed order; two collectives for the three logs) and, on rank 0,
    return the three DataFrames and write ``<out_name>_{loss,agent,sample}.csv`` as
    runner.py:151-157 does."""
    logs = ([], [], [])
    for sim_num in shard_seeds(simulations, world, rank):
        for acc, part in zip(logs, sim_fn(sim_num)):
            acc.extend(part)
    tables = gather_tables([encode(recs, cols) for recs, cols in zip(logs, SCHEMAS)], world, group, device)
    if rank != 0:
        return None
    dfs = [decode(t, cols) for t, cols in zip(tables, SCHEMAS)]
    if out_name:
        for df, kind in zip(dfs, ("loss", "agent", "sample")):
            df.to_csv(f"{out_name}_{kind}.csv")
    return tuple(dfs)


def loss_summary(loss_df, title):
    """analysis.py:62-73: per-iteration mean and sample std of the loss over simulations."""
    import pandas as pd
    mean = pd.DataFrame(loss_df.groupby(by="Iteration")["Loss"].mean())
    std = pd.DataFrame(loss_df.groupby(by="Iteration")["Loss"].std())
    mean.columns = [title]
    std.columns = [title]
    return mean, std
