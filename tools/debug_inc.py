"""Debug: bench-pattern incremental vs full vs oracle, per step (GPU)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from mfgp_coverage_amd import _lib, synthetic
from oracle import gp_oracle as O

B, G, NL, NH, k, T = int(sys.argv[1]), int(sys.argv[2]), 1024, 1024, 8, int(sys.argv[3])
asyn = int(sys.argv[4]) if len(sys.argv) > 4 else 1
NH0 = NH - k
M = G * G
hyp = synthetic.HYP["australia8_mf"]
wls = [synthetic.Workload(G, NL, NH0, k, T, seed=s) for s in range(B)]
dev = torch.device("cuda", 0)
Xnew = torch.from_numpy(np.ascontiguousarray(np.stack([w.Xnew for w in wls], 1).reshape(T, B * k, 2))).to(dev)
ynew = torch.from_numpy(np.ascontiguousarray(np.stack([w.ynew for w in wls], 1).reshape(T, B * k))).to(dev)
res = {}
for inc in (True, False):
    ctx = _lib.Context(0)
    ctx.set_incremental(inc)
    models = []
    for wl in wls:
        m = _lib.Model(ctx, _lib.MF, hyp, 1e-8)
        m.set_grid(wl.xs)
        m.set_data(wl.XL, wl.yL, wl.XH, wl.yH)
        models.append(m)
    outs = []
    for s in range(T):
        for m in models:
            m.truncate(NH0)
        mu = torch.empty(B * M, dtype=torch.float64, device=dev)
        var = torch.empty(B * M, dtype=torch.float64, device=dev)
        _lib.batch_append_predict(models, Xnew[s].data_ptr(), ynew[s].data_ptr(), [k] * B, mu.data_ptr(),
                                  var.data_ptr(), asynchronous=bool(asyn))
        outs.append((mu, var))
    ctx.synchronize()
    res[inc] = [(a.cpu().numpy(), b.cpu().numpy()) for a, b in outs]
    print("stats", inc, models[0].stats())
kss = O.prior_variance(hyp)
for s in range(T):
    row = []
    for b in range(B):
        mi, vi = res[True][s][0][b * M:(b + 1) * M], res[True][s][1][b * M:(b + 1) * M]
        mf, vf = res[False][s][0][b * M:(b + 1) * M], res[False][s][1][b * M:(b + 1) * M]
        row.append(max(O.parity_errors(mi, vi, mf, vf, kss)))
    print(s, " ".join(f"{e:.1e}" for e in row), flush=True)
for s in (0, 1, T - 1):
    b = 0
    wl = wls[b]
    XH = np.vstack([wl.XH, wl.Xnew[s]]); yH = np.concatenate([wl.yH, wl.ynew[s]])
    mu_r, var_r = O.mf_diag(wl.XL, wl.yL, XH, yH, hyp, wl.xs)
    for inc in (True, False):
        mi, vi = res[inc][s][0][:M], res[inc][s][1][:M]
        print("oracle step", s, "inc" if inc else "full", O.parity_errors(mi, vi, mu_r, var_r, kss), flush=True)
