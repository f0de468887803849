"""Lattice-separable step vs V stream at the headline workload (diagnostic).

usage: python tools/bench_lattice.py [B] [steps] [grid] [N_L] [N_H]
Per mode: ms per step (HIP events around every launch of the update kernel),
the path counters, and the max parity difference between the two modes."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from mfgp_coverage_amd import _lib, synthetic

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
T = int(sys.argv[2]) if len(sys.argv) > 2 else 50
G = int(sys.argv[3]) if len(sys.argv) > 3 else 128
NL = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
NH = int(sys.argv[5]) if len(sys.argv) > 5 else 1024
K = 8
hyp = synthetic.HYP["australia8_mf"]
NH0 = NH - K
wls = [synthetic.Workload(G, NL, NH0, K, T + 5, seed=s) for s in range(B)]
M = G * G
dev = torch.device("cuda", 0)
Xn = torch.from_numpy(np.ascontiguousarray(np.stack([w.Xnew for w in wls], 1).reshape(T + 5, B * K, 2))).to(dev)
yn = torch.from_numpy(np.ascontiguousarray(np.stack([w.ynew for w in wls], 1).reshape(T + 5, B * K))).to(dev)
res = {}
for mode in ("vstream", "lattice"):
    ctx = _lib.Context(0)
    ctx.set_lattice(("force" if os.environ.get("MFGP_LAT_FORCE") else True) if mode == "lattice" else False)
    models = []
    for w in wls:
        m = _lib.Model(ctx, _lib.MF, hyp, 1e-8)
        m.set_grid(w.xs)
        m.set_data(w.XL, w.yL, w.XH, w.yH)
        models.append(m)
    mu = torch.empty(B * M, dtype=torch.float64, device=dev)
    var = torch.empty(B * M, dtype=torch.float64, device=dev)
    _lib.batch_predict(models, mu.data_ptr(), var.data_ptr())   # the posterior of the base rows
    ks = [K] * B

    def step(s):
        for m in models:
            m.truncate(NH0)
        _lib.batch_append_predict(models, Xn[s].data_ptr(), yn[s].data_ptr(), ks, mu.data_ptr(), var.data_ptr(),
                                  asynchronous=True)

    for s in range(5):
        step(s)
    ctx.synchronize()
    ctx.enable_timing(True, predict_only=True)
    ctx.reset_timing()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(T):
        step(5 + s - 5 if False else s % 5)
    ctx.synchronize()
    wall = (time.perf_counter() - t0) / T
    tm = ctx.timing()
    res[mode] = (mu.cpu().numpy().copy(), var.cpu().numpy().copy())
    print(f"{mode}: wall {1e3 * wall:.3f} ms/step, kernel {tm['predict_ms'] / max(tm['predict_launches'], 1):.3f} ms "
          f"({tm['predict_launches']} launches), {B / wall:.0f} GP-updates/s, stats {models[0].stats()}", flush=True)
mv, vv = res["vstream"]
ml, vl = res["lattice"]
kss = float(np.exp(2 * hyp[6]) * np.exp(hyp[1]) + np.exp(hyp[4]))
print("max |dmu|/|mu|", float(np.max(np.abs(ml - mv) / np.abs(mv))),
      "max |dvar|/max(var,1e-6 kss)", float(np.max(np.abs(vl - vv) / np.maximum(np.abs(vv), 1e-6 * kss))))
