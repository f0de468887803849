"""Time compute_sample_points (simulator.py:326-374) on the device at the headline
size: one MF GP (australia8 hyperparameters, 128x128 grid, N_L = 1024 lofi +
N_H hifi points), threshold = a fraction of the current max variance.
Prints one JSON line: points chosen, wall time, time per iteration, and the CPU
oracle's time for ONE iteration of the same loop (refactor + diag predict at the
final size) for scale.

With --batch B: B such GPs (seeds 0..B-1), compute_sample_points_batch (one
batched step per iteration, mfgp_batch_sample_points) against the same B loops
run one model at a time; the line reports both and whether the point sets agree.

usage: python tools/bench_planner.py [--nh 512] [--frac 0.5] [--cpu] [--batch 8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--grid", type=int, default=128)
    p.add_argument("--nl", type=int, default=1024)
    p.add_argument("--nh", type=int, default=512)
    p.add_argument("--frac", type=float, default=0.5)
    p.add_argument("--cpu", action="store_true")
    p.add_argument("--batch", type=int, default=0)
    a = p.parse_args()
    if a.batch:
        return batch(a)
    from mfgp_coverage_amd import gaussian_process as gp, synthetic
    from mfgp_coverage_amd.planners import compute_sample_points
    hyp = synthetic.HYP["australia8_mf"]
    wl = synthetic.Workload(a.grid, a.nl, a.nh, 1, 1, seed=0)
    m = gp.MFGP(wl.XL, wl.yL[:, None], wl.XH, wl.yH[:, None], 1, 1)
    m.hyp = hyp.copy()
    m.updt_info(m.X_L, m.y_L, m.X_H, m.y_H)
    _, cov = m.predict(wl.xs)
    thr = a.frac * float(np.amax(cov))
    compute_sample_points(m, wl.xs, 0.99 * float(np.amax(cov)), False)   # warm-up
    t0 = time.perf_counter()
    pts = compute_sample_points(m, wl.xs, thr, False)
    dt = time.perf_counter() - t0
    out = {"points": int(pts.shape[0]), "seconds": dt, "ms_per_iteration": 1e3 * dt / max(1, pts.shape[0]),
           "grid": a.grid, "N_start": a.nl + a.nh, "threshold_frac": a.frac}
    if a.cpu:
        from oracle import gp_oracle as O
        XH = np.vstack([wl.XH, pts])
        yH = np.concatenate([wl.yH, np.zeros(pts.shape[0])])
        t0 = time.perf_counter()
        O.mf_diag(wl.XL, wl.yL, XH, yH, hyp, wl.xs)
        out["cpu_oracle_s_per_iteration"] = time.perf_counter() - t0
    print(json.dumps(out), flush=True)


def batch(a):
    from mfgp_coverage_amd import gaussian_process as gp, synthetic
    from mfgp_coverage_amd.planners import compute_sample_points, compute_sample_points_batch
    hyp = synthetic.HYP["australia8_mf"]
    ms, thr = [], []
    for s in range(a.batch):
        wl = synthetic.Workload(a.grid, a.nl, a.nh, 1, 1, seed=s)
        m = gp.MFGP(wl.XL, wl.yL[:, None], wl.XH, wl.yH[:, None], 1, 1)
        m.hyp = hyp.copy()
        m.updt_info(m.X_L, m.y_L, m.X_H, m.y_H)
        _, cov = m.predict(wl.xs)
        ms.append(m)
        thr.append(a.frac * float(np.amax(cov)))
    xs = wl.xs
    compute_sample_points_batch(ms, xs, [0.99 * t / a.frac for t in thr])   # warm-up
    compute_sample_points(ms[0], xs, 0.99 * thr[0] / a.frac, False)
    from mfgp_coverage_amd import _lib
    ctx = _lib.context()

    def timed_batch():
        ctx.planner_stats(reset=True)
        t0 = time.perf_counter()
        pb = compute_sample_points_batch(ms, xs, thr)
        tb = time.perf_counter() - t0
        return pb, tb, ctx.planner_stats(reset=True)   # which step form the iterations took

    def timed_single():
        t0 = time.perf_counter()
        ps = [compute_sample_points(m, xs, t, False) for m, t in zip(ms, thr)]
        return ps, time.perf_counter() - t0, ctx.planner_stats(reset=True)

    # cold: the first selection at these thresholds, which grows each model's capacity
    # (and so rebuilds its F) for the rows it appends -- what the period's own appends
    # would pay next (the planners work in place and keep the grown capacity); warm: the
    # same selection again, the models' state as it is between periods of a running
    # simulation (same capacity, F current)
    pb_c, tb_c, st_bc = timed_batch()
    ps_c, t1_c, st_sc = timed_single()
    pb, tb, st_b = timed_batch()
    ps, t1, st_s = timed_single()
    same = [int(np.array_equal(x, y)) for x, y in zip(pb, ps)]
    same_cold = [int(np.array_equal(x, y)) for x, y in zip(pb, pb_c)]
    its = max(p.shape[0] for p in pb)
    out = {"batch": a.batch, "points": [int(p.shape[0]) for p in pb], "batched_s": tb, "one_at_a_time_s": t1,
           "speedup": t1 / tb, "batched_ms_per_iteration": 1e3 * tb / max(1, its),
           "seed_iterations_per_s": sum(p.shape[0] for p in pb) / tb, "equal_to_single": same,
           "cold": {"batched_s": tb_c, "one_at_a_time_s": t1_c, "speedup": t1_c / tb_c,
                    "batched_ms_per_iteration": 1e3 * tb_c / max(1, its), "equal_to_warm": same_cold,
                    "batched_paths": st_bc, "single_paths": st_sc},
           "grid": a.grid, "N_start": a.nl + a.nh, "threshold_frac": a.frac,
           "batched_paths": st_b, "single_paths": st_s}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
