"""Full-path factor at the headline size: the fused step (k_fstep, one launch
per 64-column step) against the three-launch form (k_potrf_diag / k_panel /
k_syrk), 8 MF GPs at 128x128, N = 2048, full refactor + predict per step
(incremental off: what the reference does on every update, gp:493-529).
Prints one JSON line: factor ms per step (HIP events around the factor
stages) for both, and whether mu / var / L agree bit for bit.

usage (GPU box): python tools/bench_factor.py [--steps 10] [--gp 8]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mfgp_coverage_amd import _lib, synthetic  # noqa: E402


def run(fused, wls, steps, k, NH0, hyp, dev):
    ctx = _lib.Context(0)
    ctx.set_incremental(False)
    ctx.set_fused_factor(fused)
    B, M = len(wls), wls[0].xs.shape[0]
    models = []
    for wl in wls:
        m = _lib.Model(ctx, _lib.MF, hyp, 1e-8)
        m.set_grid(wl.xs)
        m.set_data(wl.XL, wl.yL, wl.XH, wl.yH)
        models.append(m)
    Xn = torch.from_numpy(np.ascontiguousarray(np.stack([w.Xnew for w in wls], 1).reshape(-1, B * k, 2))).to(dev)
    yn = torch.from_numpy(np.ascontiguousarray(np.stack([w.ynew for w in wls], 1).reshape(-1, B * k))).to(dev)
    mu = torch.empty(B * M, dtype=torch.float64, device=dev)
    var = torch.empty(B * M, dtype=torch.float64, device=dev)
    batch = _lib.Batch(models, [k] * B)
    per = []
    for s in range(steps + 2):
        ctx.enable_timing(s >= 2)
        ctx.reset_timing()
        batch.truncate(NH0)
        batch.append_predict(Xn.data_ptr() + s * B * k * 16, yn.data_ptr() + s * B * k * 8, mu.data_ptr(),
                             var.data_ptr())
        ctx.synchronize()
        if s >= 2:
            per.append(ctx.timing()["factor_ms"])
    L0 = models[0].factor()
    out = (float(np.median(per)), mu.cpu().numpy(), var.cpu().numpy(), L0, models[0].stats())
    del models, batch
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--gp", type=int, default=8)
    ap.add_argument("--G", type=int, default=128)
    ap.add_argument("--NL", type=int, default=1024)
    ap.add_argument("--NH", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    k = 8
    NH0 = a.NH - k
    wls = [synthetic.Workload(a.G, a.NL, NH0, k, a.steps + 2, seed=s) for s in range(a.gp)]
    hyp = synthetic.HYP["australia8_mf"]
    t3, mu3, var3, L3, st3 = run(False, wls, a.steps, k, NH0, hyp, dev)
    t1, mu1, var1, L1, st1 = run(True, wls, a.steps, k, NH0, hyp, dev)
    assert st1["full_factor"] > a.steps and st3["full_factor"] > a.steps, (st1, st3)
    print(json.dumps({"gp": a.gp, "G": a.G, "N": a.NL + a.NH, "steps": a.steps,
                      "factor_ms_three_launch": t3, "factor_ms_fused": t1, "speedup": t3 / t1,
                      "mu_bit_equal": bool(np.array_equal(mu1, mu3)),
                      "var_bit_equal": bool(np.array_equal(var1, var3)),
                      "L_bit_equal": bool(np.array_equal(L1, L3)),
                      "max_abs_dL": float(np.max(np.abs(L1 - L3)))}))


if __name__ == "__main__":
    main()
