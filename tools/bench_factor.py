"""Full-path factor at the headline size: 8 MF GPs at 128x128, N = 2048, full
refactor + predict per step (incremental off: what the reference does on every
update, gp:493-529). Prints one JSON line: the median factor ms per step (HIP
events around the factor stages: k_assemble, k_potrf_diag / k_panel / k_syrk per
64-column step, k_extract_z). Round 2 used it for the A/B of a one-launch-per-step
factor (commit 3c145a2, profiles/r02_fstep_ab.json; not kept).

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


def run(wls, steps, k, NH0, hyp, dev):
    ctx = _lib.Context(0)
    ctx.set_incremental(False)
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
    t, _, _, _, st = run(wls, a.steps, k, NH0, hyp, dev)
    assert st["full_factor"] > a.steps, st
    print(json.dumps({"gp": a.gp, "G": a.G, "N": a.NL + a.NH, "steps": a.steps, "factor_ms": t}))


if __name__ == "__main__":
    main()
