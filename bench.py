"""Benchmark: GP posterior updates/sec (128x128 grid, N_train = 2048), BASELINE.json.

Workload (BASELINE.json configs[3], "australia8 MFGP, 8 agents x 64 Monte-Carlo
seeds sharded over 8 MI355X"): each rank owns B = 8 independent seeds (one MF GP
each, australia8_mf hyperparameters). One step = one GP posterior update of
every seed (simulator.py:888-892): append the k = 8 agents' new hifi samples to
N_L = 1024 lofi + 1016 hifi points (N = 2048), update the factor, and compute
the posterior mean and variance at all M = 16384 grid cells. Inputs are
resident in HBM before the timed region. After the timed steps each rank's
per-seed max-variance trajectory (the VarMax log, simulator.py:925) is
all-gathered over RCCL for the loss/variance aggregation of runner.py:144-147.

Two update paths are timed back to back on the same workload, with identical
results (tests/test_gpu_incremental.py, tests/test_gpu_lattice*.py):
  value          -- the library's default path. On the headline's lattice grid
                    that is the lattice-separable step,
                    two launches per step at B = 8 (k_inc_lat_arg: bordered-
                    Cholesky append, w = K11^-1 K12 from the resident L^-1 and the
                    Z sums; k_lat_gemm2_arg: the separable SE kernel turns L21 V_old
                    into a K = 2 ny GEMM, and mean / variance are updated from the
                    resident posterior); elsewhere the one-pass V stream
                    (k_inc_stream, one launch);
  full_recompute -- what the reference does per update: full refactor
                    (k_assemble/potrf/panel/syrk) and V recomputed from scratch
                    (k_predict).

value = (ranks x seeds x steps) / max-over-ranks wall time.

--workload configs4 (BASELINE configs[4]): 256x256 grid, N_L = N_H = 4096,
australia9_mf, 32 seeds/GPU, the MFGP_F32 mode (V stored and streamed in fp32;
factor, solves and reductions fp64); dtype "f32". The default workload is the
headline (configs[3] sizes, fp64).

--gpus N without a torch.distributed launcher: the process starts N ranks itself
(python -m torch.distributed.run as a child; this process never touches the GPU)
and exits with their status. Under a launcher WORLD_SIZE must equal N.
The timed region holds exactly the K steps (a barrier + device synchronisation
on both sides, no HIP events inside); the trajectory gather runs after it and is
reported on its own (gather_ms).
roofline (value): the step's kernel, HBM-bound (k_inc_lat: F's lower triangle
  streamed once, the posterior in / out, the new V rows, the Z rows; k_inc_stream:
  the resident V read once) over its average launch time from HIP events on the
  launch stream around each launch of an untimed pass after the timed region;
  peak = MI355X HBM3E 8 TB/s.
roofline (full_recompute): k_predict, MFMA-bound; B x (M N^2 + 4 M N) f64 flops
  per launch; peak = MI355X f64 MFMA spec. full_recompute.breakdown_ms_per_step:
  predict, factor (assembly + blocked Cholesky) and lattice_entry (F = L^-1, the
  separable and axis tables a refactor adds before the next lattice step, timed
  on the incremental path's first warm-up step).
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
PEAK_HBM_GBS = 8000.0    # MI355X HBM3E
FUSED = os.environ.get("MFGP_FUSED", "1") != "0"
F32_RTOL = 1e-4          # oracle.gp_oracle.F32_TOL: incremental vs full VarMax in the fp32 mode


def launch_plan(gpus, env):
    """How this invocation runs: ("run", world) under a launcher or for one GPU,
    ("spawn", gpus) to start `gpus` ranks as a child launcher, or ("error", msg)."""
    if gpus < 1:
        return "error", f"--gpus must be >= 1 (got {gpus})"
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            return "error", f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks"
        return "run", world
    return ("spawn", gpus) if gpus > 1 else ("run", 1)


def spawn(gpus, argv):
    """Start `gpus` ranks (one per GPU) with torch.distributed.run as a child
    process; the parent initialises nothing on the GPU. Returns the exit status."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--workload", choices=["headline", "configs4"], default="headline",
                   help="headline: BASELINE configs[3] sizes in fp64; configs4: BASELINE configs[4] in MFGP_F32")
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--warmup", type=int, default=None)
    p.add_argument("--full-steps", type=int, default=None, help="timed steps of the full-recompute run")
    p.add_argument("--seeds-per-gpu", type=int, default=None)
    p.add_argument("--seeds", type=int, default=None,
                   help="total seeds over all ranks (default gpus x seeds-per-gpu); need not divide evenly")
    p.add_argument("--streams", type=int, default=None,
                   help="sub-batches of the rank's seeds stepped concurrently on their own streams")
    p.add_argument("--warm-ms", type=float, default=300.0,
                   help="after the warm-up steps, keep stepping (untimed) until this much wall time has passed")
    p.add_argument("--sim-iterations", type=int, default=None,
                   help="iterations of the lockstep Todescato simulation leg (0: skip)")
    p.add_argument("--grid", type=int, default=None)
    p.add_argument("--nl", type=int, default=None)
    p.add_argument("--nh", type=int, default=None)
    p.add_argument("--agents", type=int, default=8)
    p.add_argument("--hyp", default=None)
    p.add_argument("--dtype", choices=["f64", "f32"], default=None)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-faithful", type=int, default=1, help="also time the reference-faithful op sequence")
    p.add_argument("--no-full", action="store_true", help="skip the full-recompute comparison run")
    p.add_argument("--diagnostic", action="store_true",
                   help="allow a diagnostic library (MFGP_LIB); its line is marked and is not a headline number")
    a = p.parse_args()
    pre = {"headline": dict(steps=200, warmup=20, full_steps=None, seeds_per_gpu=8, grid=128, nl=1024, nh=1024,
                            hyp="australia8_mf", dtype="f64", sim_iterations=40, streams=1),
           "configs4": dict(steps=20, warmup=3, full_steps=2, seeds_per_gpu=32, grid=256, nl=4096, nh=4096,
                            hyp="australia9_mf", dtype="f32", sim_iterations=0, streams=1)}[a.workload]
    for key, v in pre.items():
        if getattr(a, key) is None:
            setattr(a, key, v)
    if a.full_steps is None:
        a.full_steps = a.steps
    return a


def source_sha():
    """sha256 (hex, 16 chars) of the library's sources (mfgp_coverage_amd/csrc/*, the
    C header): the identity of the build a committed counter summary was collected on
    (tools/summarize_profile.py writes it to profiles/<tag>_build.json)."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "mfgp_coverage_amd", "csrc")
    for f in sorted(os.listdir(csrc)) + ["../../include/mfgp_hip.h"]:
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def _pmc_summaries(suffix, tag=None):
    """The committed rocprofv3 summaries profiles/<round>[_<tag>]_<suffix>.csv collected
    on THIS build (their profiles/<round>[_<tag>]_build.json holds the current
    source_sha()), oldest first -> (files, None), or ([], reason)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{suffix}.csv")))
    # profiles/<round>_<suffix>.csv: the headline; <round>_<tag>_<suffix>.csv: another workload
    files = [f for f in files if (f"_{tag}_" in os.path.basename(f)) == (tag is not None)
             and (tag is not None or "configs4" not in os.path.basename(f))]
    if not files:
        return [], f"no committed {suffix} summary"
    sha = source_sha()
    same = []
    for f in files:
        bj = f[: -len(f"_{suffix}.csv")] + "_build.json"
        try:
            with open(bj) as fh:
                if json.load(fh).get("src_sha") == sha:
                    same.append(f)
        except (OSError, ValueError):
            pass
    if not same:
        return [], f"no {suffix} summary of this build (sources {sha}); newest: {os.path.relpath(files[-1], ROOT)}"
    return same, None


def pmc_traffic(kernel="k_predict", tag=None):
    """HBM bytes per launch of `kernel` from a committed rocprofv3 PMC summary
    (profiles/<round>_hbm_traffic.csv, written by tools/summarize_profile.py from
    separate FETCH_SIZE / WRITE_SIZE passes; FETCH_SIZE x2 per the gfx950 correction of
    MI355X_MICROARCH.md section HBM) collected on THIS build: its profiles/<round>_build.json
    must hold the current source_sha(). Returns (bytes, source) or (None, reason)."""
    import csv
    import re
    same, why = _pmc_summaries("hbm_traffic", tag)
    if not same:
        return None, why
    sha = source_sha()
    # kernel: one name, or several (the launches of one step: their bytes add up)
    names = [kernel] if isinstance(kernel, str) else list(kernel)
    tot, found = 0.0, set()
    with open(same[-1]) as f:
        for row in csv.DictReader(f):
            for n in names:
                if n not in found and re.search(rf"::{n}(?![A-Za-z0-9_])", row["Name"]):
                    tot += float(row["fetch_bytes_corrected"]) + float(row["write_bytes"])
                    found.add(n)
    if len(found) != len(names):
        return None, f"{os.path.relpath(same[-1], ROOT)} lacks {sorted(set(names) - found)}"
    return tot, f"{os.path.relpath(same[-1], ROOT)} (sources {sha})"


def pmc_mfma(kernel, tag=None):
    """MFMA utilisation of `kernel` from the newest committed rocprofv3 summary of THIS
    build (profiles/<round>_mfma_util.csv, tools/summarize_profile.py, whose
    <round>_build.json holds the current source_sha(), as for pmc_traffic): the busy
    cycles over the kernel's own duration at the measured shader clock. Returns the
    figure with its source, or {"mfma_util": None, "reason": ...}."""
    import csv
    import re
    same, why = _pmc_summaries("mfma_util", tag)
    if not same:
        return {"mfma_util": None, "reason": why}
    with open(same[-1]) as f:
        for row in csv.DictReader(f):
            if re.search(rf"::{kernel}(?![A-Za-z0-9_])", row["Name"]) or kernel == row["Name"]:
                out = {"mfma_util": float(row["mfma_util"]),
                       "source": f"{os.path.relpath(same[-1], ROOT)} (sources {source_sha()})"}
                if row.get("sclk_ghz"):
                    out["sclk_ghz"] = float(row["sclk_ghz"])
                return out
    return {"mfma_util": None, "reason": f"{os.path.relpath(same[-1], ROOT)} lacks {kernel}"}


def cpu_baseline(wl, hyp, s, NL, NH0, k, reps=5):
    """Time the oracle on one seed's update (same inputs as step s): one untimed
    warm-up, then the median of `reps` updates."""
    from oracle import gp_oracle as O
    XH = np.vstack([wl.XH[:NH0], wl.Xnew[s]])
    yH = np.concatenate([wl.yH[:NH0], wl.ynew[s]])
    with blas_all_cores():
        threads = _blas_threads()
        O.mf_diag(wl.XL, wl.yL, XH, yH, hyp, wl.xs)   # warm-up (BLAS threads, page faults)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            O.mf_diag(wl.XL, wl.yL, XH, yH, hyp, wl.xs)
            ts.append(time.perf_counter() - t0)
    avail, aff, quota = host_cores()
    out = {"value": 1.0 / float(np.median(ts)), "unit": "GP-updates/s", "cores": int(threads), "kind": "port",
           "nproc": os.cpu_count(), "affinity_cores": aff, "cgroup_cpu_quota": quota, "cpu_model": cpu_model(),
           "sample": f"oracle.mf_diag (Cholesky + triangular solves + row-sum, fp64 NumPy/BLAS, {threads} BLAS "
                     f"threads), 1 seed x {reps} updates after one warm-up at the full config "
                     f"(M={wl.xs.shape[0]}, N={NL + NH0 + k}), median"}
    return out, (XH, yH)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline_sampled(wl, hyp, s, NL, NH0, k, cells=4096, reps=3):
    """configs[4] sizes (M = 65536, N = 8192): the diag oracle's full update needs
    psi and V at 4.3 GB each and minutes of CPU, so it is timed on a bounded
    sample -- the factor at the full N plus the solve, mean and variance for
    `cells` grid cells -- and scaled linearly in M (the factor is per update, the
    rest per cell). Median of `reps`."""
    import scipy.linalg as sla
    from oracle import gp_oracle as O
    XH = np.vstack([wl.XH[:NH0], wl.Xnew[s]])
    yH = np.concatenate([wl.yH[:NH0], wl.ynew[s]])
    M = wl.xs.shape[0]
    sub = wl.xs[np.random.default_rng(0).choice(M, cells, replace=False)]
    tf, tc = [], []
    lim = blas_all_cores()
    threads = _blas_threads()
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        K = O.mf_K(wl.XL, XH, hyp)
        Lc = np.linalg.cholesky(K)
        t1 = time.perf_counter()
        psi = O.mf_psi(sub, wl.XL, XH, hyp)
        V = sla.solve_triangular(Lc, psi.T, lower=True, check_finite=False)
        _ = np.einsum("ij,ij->j", V, V)
        t2 = time.perf_counter()
        tf.append(t1 - t0)
        tc.append(t2 - t1)
    lim.restore_original_limits()
    t = float(np.median(tf[1:])) + float(np.median(tc[1:])) * M / cells
    return {"value": 1.0 / t, "unit": "GP-updates/s", "cores": int(threads), "kind": "port",
            "nproc": os.cpu_count(), "cpu_model": cpu_model(),
            "sample": f"oracle.mf_diag steps (fp64 NumPy/BLAS, {threads} BLAS threads) for 1 seed at N={NL + NH0 + k}: "
                      f"K + Cholesky at full N, psi / triangular solve / row-sums for {cells} of the M={M} cells, "
                      f"scaled to M; median of {reps} after one warm-up"}


def host_cores():
    """The host cores this process may run on: the scheduler affinity, capped by a
    cgroup CPU quota when one is set (a GPU box shares its host: os.cpu_count()
    reports every core of the machine, the quota what this job gets)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return (min(n, quota) if quota else n), n, quota


def _blas_threads():
    try:
        from threadpoolctl import threadpool_info
        return max([i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"] or [1])
    except Exception:  # pragma: no cover
        return int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))


def blas_all_cores():
    """Context manager: BLAS threads = every host core available."""
    from threadpoolctl import threadpool_limits
    return threadpool_limits(limits=host_cores()[0], user_api="blas")


def cpu_faithful(wl, hyp, XH, yH, reps=3):
    from oracle import gp_oracle as O
    ts = []
    with blas_all_cores():
        threads = _blas_threads()
        for _ in range(reps):
            t0 = time.perf_counter()
            O.mf_faithful(wl.XL, wl.yL, XH, yH, hyp, wl.xs)
            ts.append(time.perf_counter() - t0)
    return {"value": 1.0 / float(np.median(ts)), "unit": "GP-updates/s", "cores": int(threads),
            "sample": "oracle.mf_faithful (the reference's op sequence: dense K(X*,X*), 4x np.linalg.solve, "
                      f"dense psi@beta), median of {reps} updates at the full config"}


def simulation_leg(a, world, rank, my_seeds, wls, hyp, dev, backend):
    """The planners on top of the GP step: this rank's seeds
    run the reference's Todescato loop (simulator.py:788-954) in lockstep
    (coverage.run_lockstep: one batched append + predict and one batched cell
    reduction per iteration, host Voronoi per seed), from the lofi prior of the
    headline workload (1024 points, shared by all seeds as runner.py:131-132 shares
    its prior), 8 agents, the headline grid. Timed with a barrier and device
    synchronisation on both sides, max over ranks; beside it one seed through the
    drop-in API (coverage.simulate, the reference's one-simulation-per-process
    model) for a few iterations."""
    import torch
    import torch.distributed as dist
    from mfgp_coverage_amd import coverage, synthetic
    T = a.sim_iterations
    w0 = wls[0]
    truth = np.column_stack([w0.xs, synthetic.field(w0.xs, np.random.default_rng(1234).random((4, 2)))])
    prior = np.column_stack([w0.XL, w0.yL])
    stats = coverage.LockstepStats()
    # one untimed iteration first (first-use kernel loads of the cell reduction)
    coverage.run_lockstep("todescato", my_seeds[:1], 1, a.agents, truth, 0.1, prior, hyp, log=False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    logs = coverage.run_lockstep("todescato", my_seeds, T, a.agents, truth, 0.1, prior, hyp, stats=stats)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    Td = min(T, 8)
    t1 = time.perf_counter()
    coverage.simulate("todescato", my_seeds[0], Td, a.agents, truth, 0.1, prior, hyp)
    el1 = time.perf_counter() - t1
    tt = torch.tensor([el, el1], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    el, el1 = float(tt[0].item()), float(tt[1].item())
    total = a.seeds if a.seeds is not None else world * a.seeds_per_gpu
    it = max(1, stats.iterations)
    return {
        "metric": "coverage-simulation iterations/s (Todescato planner, seeds in lockstep)",
        "value": total * T / el, "unit": "seed-iterations/s", "per_gpu": len(my_seeds) * T / el,
        "seeds_per_gpu": len(my_seeds), "iterations": T, "agents": a.agents,
        "ms_per_iteration": el / T * 1e3,
        "breakdown_ms_per_iteration": {"gp_step_enqueue": 1e3 * stats.gp / it, "voronoi_host": 1e3 * stats.voronoi / it,
                                       "cell_reduce_and_wait": 1e3 * stats.cells / it,
                                       "samples_logs_decisions": 1e3 * stats.host / it},
        "hifi_rows_appended": stats.rows, "seed_steps_without_samples": stats.post_copy,
        "log_rows": [sum(len(x[j]) for x in logs) for j in range(3)],
        "workload": f"{a.grid}x{a.grid} grid, australia8_mf, prior = {prior.shape[0]} lofi points, "
                    f"{a.agents} agents, sigma_n = 0.1, synthetic truth field",
        "dropin_one_seed": {"value": Td / el1, "unit": "seed-iterations/s", "iterations": Td,
                            "note": "one seed through SFGP/MFGP + geometry (the reference's process model)"},
    }


def main():
    a = parse()
    plan, arg = launch_plan(a.gpus, os.environ)
    if plan == "error":
        sys.exit(f"bench.py: {arg}")
    if plan == "spawn":
        sys.exit(spawn(arg, sys.argv[1:]))
    diag_lib = os.environ.get("MFGP_LIB")
    if diag_lib and not a.diagnostic:
        sys.exit("bench.py: MFGP_LIB selects a diagnostic library build; pass --diagnostic to time it "
                 "(its line is marked and is not a headline number)")
    world = arg
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    # ranks map onto the visible GPUs (identity on a full node; the gloo rehearsal
    # below can stack several ranks on one GPU)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # MFGP_DIST_BACKEND=gloo rehearses the N>1 path (sharding, barriers, the
    # gather, max-over-ranks) with host-side collectives; the default is RCCL
    backend = os.environ.get("MFGP_DIST_BACKEND", "nccl")
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        assert dist.get_world_size() == a.gpus, (dist.get_world_size(), a.gpus)
    from mfgp_coverage_amd import _lib, synthetic
    from mfgp_coverage_amd.ensemble import gather_trajectories, shard_seeds

    _lib.set_device(local)
    # one explicit stream for the library's launches and torch's reductions
    # (the null stream would not order against the library's non-blocking stream)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)

    f32 = a.dtype == "f32"
    dtype = _lib.F32 if f32 else _lib.F64
    total_seeds = a.seeds if a.seeds is not None else world * a.seeds_per_gpu
    if total_seeds < world:
        sys.exit(f"bench.py: --seeds {total_seeds} leaves a rank without seeds ({world} ranks)")
    my_seeds = shard_seeds(total_seeds, world, rank)   # contiguous, sizes differ by at most one
    B, G, NL, NH, k = len(my_seeds), a.grid, a.nl, a.nh, a.agents
    NH0 = NH - k
    W, K = a.warmup, a.steps
    KF = min(a.full_steps, K)
    total = W + K
    hyp = synthetic.HYP[a.hyp]
    M = G * G
    N = NL + NH
    wls = [synthetic.Workload(G, NL, NH0, k, total, seed=seed) for seed in my_seeds]
    Xnew = torch.from_numpy(np.ascontiguousarray(np.stack([w.Xnew for w in wls], 1).reshape(total, B * k, 2))).to(dev)
    ynew = torch.from_numpy(np.ascontiguousarray(np.stack([w.ynew for w in wls], 1).reshape(total, B * k))).to(dev)
    mu = torch.empty(B * M, dtype=torch.float64, device=dev)
    var = torch.empty(B * M, dtype=torch.float64, device=dev)
    ks = [k] * B

    def run(incremental, W, K, nstreams=1):
        total = W + K
        # the rank's seeds as `nstreams` contiguous sub-batches, each stepped by its
        # own context on its own stream (concurrent launches: mfgp_ctx_set_concurrent);
        # one sub-batch: the library's context on the bench's torch stream
        NS = max(1, min(nstreams, B))
        glo = [g * B // NS for g in range(NS + 1)]
        ctxs = []
        for g in range(NS):
            if NS == 1:
                c = _lib.context() if incremental else _lib.Context(local)
                c.set_stream(stream.cuda_stream)
            else:
                c = _lib.Context(local)
                c.set_concurrent(True)
            c.set_incremental(incremental)
            # MFGP_FUSED=0: the append and the predict as two launches (diagnostic)
            c.set_fused(FUSED)
            ctxs.append(c)
        models, batches = [], []
        for g in range(NS):
            mg = []
            for wl in wls[glo[g]:glo[g + 1]]:
                mdl = _lib.Model(ctxs[g], _lib.MF, hyp, 1e-8, dtype=dtype)
                mdl.set_grid(wl.xs)
                mdl.set_data(wl.XL, wl.yL, wl.XH, wl.yH)
                mg.append(mdl)
            models.extend(mg)
            batches.append(_lib.Batch(mg, ks[glo[g]:glo[g + 1]]))
        varmax = torch.zeros(total, B, dtype=torch.float64, device=dev)
        xp0, yp0, vp0 = Xnew.data_ptr(), ynew.data_ptr(), varmax.data_ptr()
        mup, varp = mu.data_ptr(), var.data_ptr()
        # the posterior of the base rows (N - k), as the simulator predicts before
        # every update (sim:885-892); the incremental steps start from it
        for g in range(NS):
            _lib.batch_predict(batches[g].models, mup + 8 * glo[g] * M, varp + 8 * glo[g] * M)

        def sync_all():
            for c in ctxs:
                c.synchronize()

        def step(s):
            for g in range(NS):
                lo = glo[g]
                batches[g].truncate(NH0)
                # VarMax of every seed (np.amax(cov), simulator.py:1014) fused into the predict epilogue
                batches[g].append_predict(xp0 + 8 * (s * B * k * 2 + lo * k * 2), yp0 + 8 * (s * B * k + lo * k),
                                          mup + 8 * lo * M, varp + 8 * lo * M, asynchronous=True,
                                          vmax_ptr=vp0 + 8 * (s * B + lo))

        def timing_all():
            ts = [c.timing() for c in ctxs]
            return {key: sum(t[key] for t in ts) for key in ts[0]}

        def set_timing(on, predict_only=False):
            for c in ctxs:
                c.enable_timing(on, predict_only=predict_only)
                if on:
                    c.set_timing_stride(1)
                    c.reset_timing()

        def aggregate(traj):
            if backend != "nccl":
                traj = traj.cpu()
            _, agg_mean, agg_std = gather_trajectories(traj, world)   # the single RCCL exchange
            return torch.stack([agg_mean, torch.nan_to_num(agg_std)])

        # the first (warm-up) step of the incremental path enters the lattice mode
        # after the full factor: F = L^-1 (k_trinv_f), the separable tables and the
        # axis tables, timed as factor work (reported with full_recompute: every
        # refactor of a lattice-eligible model pays it once)
        lat_build_ms = None
        tw0 = time.perf_counter()
        for s in range(W):
            if s == 0 and incremental:
                set_timing(True)
            step(s)
            if s == 0 and incremental:
                sync_all()
                lat_build_ms = timing_all()["factor_ms"]
                set_timing(False)
        # a short run (the driver's --steps 20 is ~2 ms of GPU work) would otherwise
        # time the clock ramp: keep stepping, untimed, on the warm-up inputs (every
        # step truncates back to the same rows, so any input is a valid step) until
        # warm_ms of wall time has passed
        extra = 0
        sync_all()
        aggregate(varmax[:W].transpose(0, 1).contiguous())   # first-use kernel loads / communicator setup
        sync_all()
        set_timing(False)
        if world > 1:
            dist.barrier()
        # (the warm-up steps end right before the timed region: no idle gap in which
        # the clocks could drop between them)
        while W > 1 and (time.perf_counter() - tw0) * 1e3 < a.warm_ms:
            for _ in range(16):
                step(1 + extra % (W - 1))
                extra += 1
            sync_all()
        # the timed region: exactly K steps, nothing else on the streams (no HIP events)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        host_t = []
        for s in range(W, total):
            th = time.perf_counter()
            step(s)
            host_t.append(time.perf_counter() - th)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        # the job's one exchange (the per-seed VarMax trajectories, runner.py:144-147),
        # once per job: timed on its own, not part of the per-step rate
        traj = varmax[W:].transpose(0, 1).contiguous()           # [B, K] per-seed VarMax trajectory
        tg0 = time.perf_counter()
        agg = aggregate(traj)
        torch.cuda.synchronize(dev)
        tg1 = time.perf_counter()
        sync_all()   # raises LinAlgError if any factor was not positive definite
        # the kernel's launch time (roofline): R more untimed steps on the same
        # inputs, HIP events around every launch on each launch stream
        R = min(K, 50) if incremental else min(K, 3)
        set_timing(True, predict_only=True)
        for s in range(W, W + R):
            step(s)
        sync_all()
        tm = timing_all()
        # per-stage breakdown: a few more (untimed) steps with every stage bracketed by events
        set_timing(True)
        nb_steps = min(5 if incremental else 1, K)
        for s in range(W, W + nb_steps):
            step(s)
        sync_all()
        tb = timing_all()
        set_timing(False)
        el = torch.tensor([t1 - t0, tg1 - tg0], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        if world > 1:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        if not diag_lib:   # diagnostic library builds compute garbage on purpose
            assert torch.isfinite(agg).all()
        st = models[0].stats()
        del models, batches
        return {"elapsed": float(el[0].item()), "gather_ms": 1e3 * float(el[1].item()), "tm": tm,
                "lat_build_ms": lat_build_ms, "extra_warmup_steps": extra, "streams": NS,
                "gps_per_launch": B / NS,
                "host_ms": 1e3 * float(np.mean(host_t)), "stats": st, "traj": traj.cpu().numpy(), "R": R,
                "breakdown": {"predict": tb["predict_ms"] / nb_steps / NS, "factor": tb["factor_ms"] / nb_steps / NS}}

    inc = run(True, W, K, a.streams)
    full = None if a.no_full else run(False, W, KF)
    sim = simulation_leg(a, world, rank, my_seeds, wls, hyp, dev, backend) if a.sim_iterations else None
    if os.environ.get("MFGP_BENCH_DUMP") and rank == 0:
        np.savez(os.environ["MFGP_BENCH_DUMP"], inc=inc["traj"], full=full["traj"] if full else inc["traj"])
    if full is not None and rank == 0 and not diag_lib:
        # the two paths produce the same posterior (VarMax trajectories to rounding;
        # the fp32 mode's to its tolerance) on the steps both ran
        np.testing.assert_allclose(inc["traj"][:, :KF], full["traj"], rtol=F32_RTOL if f32 else 1e-9)

    if rank == 0:
        elapsed, tm = inc["elapsed"], inc["tm"]
        assert inc["stats"]["inc_factor"] >= K and inc["stats"]["vstream"] >= K, inc["stats"]
        n0 = N - k
        es = 4 if f32 else 8
        lattice = inc["stats"].get("lattice", 0) >= K
        # algorithmic bytes of one k_inc_stream launch: V_old read once, V_new written,
        # grid read and mu / var written, and per training row the L21 gather, its
        # store into A and read back, the compact rows and z
        if f32:
            vbytes = B * (4 * M * (n0 + k) + 32 * M + n0 * (16 * k + 4 * 16 + 8))
        else:
            vbytes = B * 8 * (M * (n0 + k + 4) + n0 * (3 * k + 1))
        # (sub-batches on concurrent streams: a launch covers B / streams GPs)
        shr = inc["gps_per_launch"] / B
        vbytes = vbytes * shr
        v_ms = tm["predict_ms"] / max(1, tm["predict_launches"])
        v_gbs = vbytes / (v_ms * 1e-3) / 1e9 if v_ms > 0 else float("nan")
        # the lattice step in axis form (k_inc_lat). Bytes: F's
        # lower triangle read once by the w pass (the dominant stream; es bytes per element), the resident
        # posterior in and out plus the caller's mu / var, the new V rows, the Z rows
        # written once and read by every 64-column tile row; flops: the w pass (16 n0^2),
        # the Z sums (2 KA nx n_t) and the K = parts x ny GEMM (2 KA M parts ny8)
        ka = 8 if k <= 8 else 16
        parts = 2
        n_t = n0 + (n0 - NL)
        ny8 = -(-G // 8) * 8
        # (F's elements: fp32 for MFGP_F32 models, whose w units stream the rounded copy)
        fbytes = es * sum((n0 - 64 * jb) * 64 for jb in range(-(-n0 // 64)))
        zbytes = 8 * parts * ny8 * G * ka * (1 + -(-G // 64))
        lat_bytes = B * (fbytes + 8 * 6 * M + es * M * k + zbytes) * shr
        lat_flops = B * (16 * n0 * n0 + 2 * ka * G * n_t + 2 * ka * M * parts * ny8) * shr
        lat_gbs = lat_bytes / (v_ms * 1e-3) / 1e9 if v_ms > 0 else float("nan")
        lat_tf = lat_flops / (v_ms * 1e-3) / 1e12 if v_ms > 0 else float("nan")
        value = total_seeds * K / elapsed
        # SURVEY.md section 8d's algorithmic cost of one update as the reference
        # computes it (refactor + V from scratch): F = N^3/3 + M N^2 + 2 N^2 + 4 M N flop,
        # B_8d = 8 (4M + 3N + 2 N^2) bytes. The incremental path does not do that work
        # (it reuses the resident V): expressed in F per second it exceeds the f64
        # MFMA peak, which is the point of the algorithm, not a measurement error.
        F8d = N ** 3 / 3 + M * N * N + 2 * N * N + 4 * M * N
        B8d = 8 * (4 * M + 3 * N + 2 * N * N)
        # PMC bytes come from the committed profile of the default configuration
        default_cfg = (a.workload, G, NL, NH, B, k, a.hyp, a.dtype) == ("headline", 128, 1024, 1024, 8, 8,
                                                                         "australia8_mf", "f64")
        c4_cfg = (G, NL, NH, B, a.hyp, a.dtype) == (256, 4096, 4096, 32, "australia9_mf", "f32")
        # the lattice step is two launches (k_inc_lat: producers, w, Z; k_lat_gemm2: the
        # GEMM and cells) where k_lat_gemm2's tiles fill the chip once or twice (the
        # library's rule, mfgp_capi.hip), else one (the GEMM inside k_inc_lat);
        # MFGP_LAT_GEMM2=1 / 0 forces either
        # (the model's lattice_g2 counter says which ran)
        g2 = inc["stats"].get("lattice_g2", 0) >= K
        kern = "k_inc_lat" if lattice else ("k_inc_stream" if FUSED else "k_vstream")
        if lattice and g2:
            kern = ("k_inc_lat", "k_lat_gemm2")
        traffic, traffic_src = None, None
        if default_cfg or c4_cfg:
            # batches of <= 8 GPs run the step with its descriptors as the kernel argument
            # (k_inc_lat_arg, k_lat_gemm2_arg); larger ones upload them (k_inc_lat, k_lat_gemm2)
            if lattice and B <= 8:
                ka_ = ("k_inc_lat_arg", "k_lat_gemm2_arg") if g2 else "k_inc_lat_arg"
                traffic, traffic_src = pmc_traffic(ka_, "configs4" if c4_cfg else None)
                if traffic is not None:
                    kern = ka_
            if traffic is None:
                traffic, traffic_src = pmc_traffic(kern, "configs4" if c4_cfg else None)
        kern = kern if isinstance(kern, str) else " + ".join(kern)
        if lattice:
            update = ("incremental, lattice-separable, " + ("two launches per step (k_inc_lat: append, w, Z; "
                      "k_lat_gemm2: GEMM + cells)" if g2 else "one launch per step (k_inc_lat)") +
                      ": bordered-Cholesky append, "
                      "w = K11^-1 K12 from the resident L^-1; every training term lies on the grid's lattice, so "
                      "L21 V_old = sum over lattice rows of Z (w c ex summed per row) times axis-table rows: a "
                      "K = 2 ny f64 MFMA GEMM, no pass over V; mean / variance updated from the previous posterior")
            roof = {"bound": "hbm", "achieved": lat_gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": lat_gbs / PEAK_HBM_GBS, "traffic": traffic, "traffic_source": traffic_src,
                    "kernel": kern, "bytes_per_launch": lat_bytes, "flops_per_launch": lat_flops,
                    "mfma_tflops": lat_tf, "avg_launch_ms": v_ms, "launches_timed": tm["predict_launches"],
                    "timing": f"HIP events around each of {inc['R']} launches of an untimed pass after the timed "
                              "region (no events inside the timed region)",
                    "design_note": "bytes = F's lower triangle (the w pass), the posterior in / out, the new V rows "
                                   "and the Z rows; avg_launch_ms spans the step's launches (HIP events before the "
                                   "first, after the last); the step is a chain of dependent phases (producers -> "
                                   "w -> Z | GEMM -> cells), latency- not bandwidth-bound (DESIGN.md section 2.4)"}
        else:
            update = ("incremental, one launch per step (k_inc_stream): bordered-Cholesky append + one pass over "
                      "the resident V = L^-1 psi^T" if FUSED else
                      "incremental: bordered-Cholesky append (k_inc_stream) + one pass over the resident "
                      "V = L^-1 psi^T (k_vstream)")
            roof = {"bound": "hbm", "achieved": v_gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": v_gbs / PEAK_HBM_GBS, "traffic": traffic, "traffic_source": traffic_src,
                    "kernel": kern, "bytes_per_launch": vbytes, "avg_launch_ms": v_ms,
                    "launches_timed": tm["predict_launches"],
                    "timing": f"HIP events around each of {inc['R']} launches of an untimed pass after the timed "
                              "region (no events inside the timed region)",
                    "design_bytes_note": f"{es}-byte V: bytes_per_launch = the resident V read once plus the new "
                                         "rows, grid, outputs and per-row L21 / z terms (DESIGN.md section 4)"}
        # the step's algorithmic bytes over the whole step's wall time (all sub-batches)
        step_bytes = roof["bytes_per_launch"] / shr
        roof["streams"] = inc["streams"]
        if roof.get("traffic"):
            roof["traffic_over_algorithmic"] = roof["traffic"] / roof["bytes_per_launch"]
        roof["step_aggregate_gbs"] = step_bytes / (elapsed / K) / 1e9
        roof["step_aggregate_frac"] = roof["step_aggregate_gbs"] / PEAK_HBM_GBS
        if default_cfg:
            wl_name = "australia8_mf MFGP seed ensemble (BASELINE configs[3])"
        elif c4_cfg:
            wl_name = "BASELINE configs[4]: synthetic australia9_mf MFGP seed ensemble"
        else:
            wl_name = f"{a.hyp} MFGP seed ensemble"
        out = {
            "metric": METRIC if not diag_lib else f"DIAGNOSTIC library {diag_lib}: " + METRIC,
            "value": value,
            "unit": "GP-updates/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": a.dtype,
            "data": "synthetic",
            "config": {
                "workload": f"{wl_name}: {B} seeds/GPU, "
                            f"{G}x{G} grid (M={M}), N_L={NL} lofi + N_H={NH} hifi ({NH0} + {k} new agent "
                            f"samples appended per update), factor update + mean/var at every cell, "
                            + ("MFGP_F32: V = L^-1 psi^T stored and streamed in fp32, factor / solves / "
                               "reductions in fp64" if f32 else "fp64"),
                "update": update + "; full_recompute below is the reference's per-update work",
                "seeds_per_gpu": B, "grid": G, "N_train": N, "N_lofi": NL, "N_hifi": NH, "agents": k,
                "global_seeds": total_seeds, "parallelism": f"seed-sharded x{world}, 1 RCCL all_gather",
            },
            "roofline": roof,
            "algorithmic_8d": {
                "flops_per_update": F8d, "bytes_per_update": B8d,
                "flop_equivalent_tflops": F8d * value / 1e12,
                "frac_of_f64_mfma_peak": F8d * value / 1e12 / PEAK_F64_TFLOPS,
                "byte_rate_gbs": B8d * value / 1e9,
                "note": "SURVEY.md 8d's per-update work is the reference's (refactor + V from scratch); the "
                        "incremental path does not recompute V, so this flop-equivalent rate is above the MFMA "
                        "peak by construction; the roofline above is the kernel's own work",
            },
            "host_enqueue_ms_per_step": inc["host_ms"],
            "extra_warmup_steps": inc["extra_warmup_steps"],
            "gather_ms": inc["gather_ms"],
            "breakdown_ms_per_step": inc["breakdown"],
        }
        if full is not None:
            ft = full["tm"]
            flops = B * (M * N * N + 4 * M * N)
            avg_ms = ft["predict_ms"] / max(1, ft["predict_launches"])
            achieved = flops / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else float("nan")
            ftraffic, _ = pmc_traffic("k_predict") if default_cfg else (None, None)
            out["full_recompute"] = {
                "value": total_seeds * KF / full["elapsed"],
                "steps": KF,
                "ms_per_step": full["elapsed"] / KF * 1e3,
                "roofline": {
                    "bound": "mfma", "achieved": achieved, "peak": PEAK_F64_TFLOPS, "unit": "TFLOP/s",
                    "frac": achieved / PEAK_F64_TFLOPS, "traffic": ftraffic,
                    "kernel": "k_predict" + (" (+ k_vnarrow: V computed in fp64, stored fp32)" if f32 else ""),
                    "flops_per_launch": flops, "avg_launch_ms": avg_ms,
                    "pmc": pmc_mfma("k_predict") if default_cfg else None,
                },
                "host_enqueue_ms_per_step": full["host_ms"],
                "breakdown_ms_per_step": dict(full["breakdown"], **({"lattice_entry": inc["lat_build_ms"]}
                                                              if inc.get("lat_build_ms") else {})),
            }
        if sim is not None:
            out["simulation"] = sim
        if world == 1 and not a.no_cpu_baseline:
            if M * N > 16384 * 2048:
                out["cpu_baseline"] = cpu_baseline_sampled(wls[0], hyp, W, NL, NH0, k)
            else:
                cb, (XH, yH) = cpu_baseline(wls[0], hyp, W, NL, NH0, k)
                if a.cpu_faithful:
                    cb["faithful"] = cpu_faithful(wls[0], hyp, XH, yH)
                out["cpu_baseline"] = cb
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
