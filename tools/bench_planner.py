"""Time compute_sample_points (simulator.py:326-374) on the device at the headline
size: one MF GP (australia8 hyperparameters, 128x128 grid, N_L = 1024 lofi +
N_H hifi points), threshold = a fraction of the current max variance.
Prints one JSON line: points chosen, wall time, time per iteration, and the CPU
oracle's time for ONE iteration of the same loop (refactor + diag predict at the
final size) for scale.

usage: python tools/bench_planner.py [--nh 512] [--frac 0.5] [--cpu]
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
    a = p.parse_args()
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


if __name__ == "__main__":
    main()
