"""Benchmark: GP posterior updates/sec (128x128 grid, N_train = 2048), BASELINE.json.

Workload (BASELINE.json configs[3], "australia8 MFGP, 8 agents x 64 Monte-Carlo
seeds sharded over 8 MI355X"): each rank owns B = 8 independent seeds (one MF GP
each, australia8_mf hyperparameters). One step = one GP posterior update of
every seed (simulator.py:888-892): append the k = 8 agents' new hifi samples to
N_L = 1024 lofi + 1016 hifi points (N = 2048), refactor from scratch, and
compute the posterior mean and variance at all M = 16384 grid cells. Inputs are
resident in HBM before the timed region. After the timed steps each rank's
per-seed max-variance trajectory (the VarMax log, simulator.py:925) is
all-gathered over RCCL for the loss/variance aggregation of runner.py:144-147.

value = (ranks x seeds x steps) / max-over-ranks wall time.
roofline: the fused predict kernel (dominant), algorithmic f64 flops per launch
  = B x (M*N^2 + 4*M*N) [V = L^-1 psi^T triangular solve + mean/variance
  reductions], over its average launch time measured with HIP events on the
  launch stream; peak = MI355X f64 MFMA spec.
cpu_baseline: the oracle's diag-only NumPy restatement (Cholesky, triangular
  solves, row-sum of squares) on one seed's update, on the host cores
  (rank 0, N = 1 only); the reference-faithful op sequence is timed beside it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GP posterior updates/sec (128×128 grid, N_train=2048) at 1/2/4/8 MI355X"
PEAK_F64_TFLOPS = 78.6   # MI355X f64 matrix (= vector) spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--seeds-per-gpu", type=int, default=8)
    p.add_argument("--grid", type=int, default=128)
    p.add_argument("--nl", type=int, default=1024)
    p.add_argument("--nh", type=int, default=1024)
    p.add_argument("--agents", type=int, default=8)
    p.add_argument("--hyp", default="australia8_mf")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-faithful", type=int, default=1, help="also time the reference-faithful op sequence")
    return p.parse_args()


def pmc_traffic(kernel="k_predict"):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC
    summary (profiles/<round>_hbm_traffic.csv, written by tools/summarize_profile.py
    from separate FETCH_SIZE / WRITE_SIZE passes; FETCH_SIZE x2 per the gfx950
    correction of MI355X_MICROARCH.md section HBM)."""
    import glob
    import csv
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_hbm_traffic.csv")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        for row in csv.DictReader(f):
            if kernel in row["Name"]:
                tot = float(row["fetch_bytes_corrected"]) + float(row["write_bytes"])
                return tot, os.path.relpath(files[-1], ROOT)
    return None, None


def cpu_baseline(wl, hyp, s, NL, NH0, k, reps=3):
    """Time the oracle on one seed's update (same inputs as step s)."""
    from oracle import gp_oracle as O
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"] or [1])
    except Exception:  # pragma: no cover
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    XH = np.vstack([wl.XH[:NH0], wl.Xnew[s]])
    yH = np.concatenate([wl.yH[:NH0], wl.ynew[s]])
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        O.mf_diag(wl.XL, wl.yL, XH, yH, hyp, wl.xs)
        ts.append(time.perf_counter() - t0)
    out = {"value": 1.0 / float(np.median(ts)), "unit": "GP-updates/s", "cores": int(threads), "kind": "port",
           "sample": f"oracle.mf_diag (Cholesky + triangular solves + row-sum, fp64 NumPy/BLAS), 1 seed x "
                     f"{reps} updates at the full config (M={wl.xs.shape[0]}, N={NL + NH0 + k}), median"}
    return out, (XH, yH)


def cpu_faithful(wl, hyp, XH, yH):
    from oracle import gp_oracle as O
    t0 = time.perf_counter()
    O.mf_faithful(wl.XL, wl.yL, XH, yH, hyp, wl.xs)
    dt = time.perf_counter() - t0
    return {"value": 1.0 / dt, "unit": "GP-updates/s",
            "sample": "oracle.mf_faithful (the reference's op sequence: dense K(X*,X*), 4x np.linalg.solve, "
                      "dense psi@beta), 1 update at the full config"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    from mfgp_coverage_amd import _lib, synthetic
    from mfgp_coverage_amd.ensemble import gather_trajectories, shard_seeds

    _lib.set_device(local)
    ctx = _lib.context()
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)

    B, G, NL, NH, k = a.seeds_per_gpu, a.grid, a.nl, a.nh, a.agents
    NH0 = NH - k
    W, K = a.warmup, a.steps
    total = W + K
    hyp = synthetic.HYP[a.hyp]
    M = G * G
    N = NL + NH
    wls, models = [], []
    for seed in shard_seeds(world * B, world, rank):
        wl = synthetic.Workload(G, NL, NH0, k, total, seed=seed)
        mdl = _lib.Model(ctx, _lib.MF, hyp, 1e-8)
        mdl.set_grid(wl.xs)
        mdl.set_data(wl.XL, wl.yL, wl.XH, wl.yH)
        wls.append(wl)
        models.append(mdl)
    Xnew = torch.from_numpy(np.ascontiguousarray(np.stack([w.Xnew for w in wls], 1).reshape(total, B * k, 2))).to(dev)
    ynew = torch.from_numpy(np.ascontiguousarray(np.stack([w.ynew for w in wls], 1).reshape(total, B * k))).to(dev)
    mu = torch.empty(B * M, dtype=torch.float64, device=dev)
    var = torch.empty(B * M, dtype=torch.float64, device=dev)
    varmax = torch.zeros(total, B, dtype=torch.float64, device=dev)
    ks = [k] * B

    def step(s):
        for mdl in models:
            mdl.truncate(NH0)
        _lib.batch_append_predict(models, Xnew[s].data_ptr(), ynew[s].data_ptr(), ks, mu.data_ptr(),
                                  var.data_ptr(), asynchronous=True)
        varmax[s] = var.view(B, M).amax(dim=1)

    for s in range(W):
        step(s)
    ctx.synchronize()
    ctx.enable_timing(True)
    ctx.reset_timing()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    host_t = []
    for s in range(W, total):
        th = time.perf_counter()
        step(s)
        host_t.append(time.perf_counter() - th)
    traj = varmax[W:].transpose(0, 1).contiguous()           # [B, K] per-seed VarMax trajectory
    _, agg_mean, agg_std = gather_trajectories(traj, world)   # the single RCCL exchange
    agg = torch.stack([agg_mean, torch.nan_to_num(agg_std)])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    ctx.synchronize()   # raises LinAlgError if any factor was not positive definite
    tm = ctx.timing()
    el = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    if not os.environ.get("MFGP_LIB"):   # diagnostic library builds compute garbage on purpose
        assert torch.isfinite(agg).all()

    if rank == 0:
        flops = B * (M * N * N + 4 * M * N)
        avg_ms = tm["predict_ms"] / max(1, tm["predict_launches"])
        achieved = flops / (avg_ms * 1e-3) / 1e12
        traffic, traffic_src = pmc_traffic()
        out = {
            "metric": METRIC,
            "value": world * B * K / elapsed,
            "unit": "GP-updates/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": f"{a.hyp} MFGP seed ensemble (BASELINE configs[3]): {B} seeds/GPU, "
                            f"{G}x{G} grid (M={M}), N_L={NL} lofi + N_H={NH} hifi ({NH0} + {k} new agent "
                            f"samples appended per update), full refactor + mean/var at every cell, fp64",
                "seeds_per_gpu": B, "grid": G, "N_train": N, "N_lofi": NL, "N_hifi": NH, "agents": k,
                "global_seeds": world * B, "parallelism": f"seed-sharded x{world}, 1 RCCL all_gather",
            },
            "roofline": {
                "bound": "mfma", "achieved": achieved, "peak": PEAK_F64_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / PEAK_F64_TFLOPS, "traffic": traffic, "traffic_source": traffic_src,
                "kernel": "k_predict", "flops_per_launch": flops, "avg_launch_ms": avg_ms,
            },
            "host_enqueue_ms_per_step": 1e3 * float(np.mean(host_t)),
            "breakdown_ms_per_step": {
                "predict": tm["predict_ms"] / K, "factor": tm["factor_ms"] / K,
            },
        }
        if world == 1 and not a.no_cpu_baseline:
            cb, (XH, yH) = cpu_baseline(wls[0], hyp, W, NL, NH0, k)
            if a.cpu_faithful:
                cb["faithful"] = cpu_faithful(wls[0], hyp, XH, yH)
            out["cpu_baseline"] = cb
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
