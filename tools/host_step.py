"""Diagnostic: host time of one headline step, split by call (bench.py's step).
usage: python tools/host_step.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from mfgp_coverage_amd import _lib, synthetic

T = int(sys.argv[1]) if len(sys.argv) > 1 else 200
B, G, NL, NH, k = 8, 128, 1024, 1024, 8
NH0 = NH - k
hyp = synthetic.HYP["australia8_mf"]
wls = [synthetic.Workload(G, NL, NH0, k, T + 5, seed=s) for s in range(B)]
dev = torch.device("cuda", 0)
Xn = torch.from_numpy(np.ascontiguousarray(np.stack([w.Xnew for w in wls], 1).reshape(T + 5, B * k, 2))).to(dev)
yn = torch.from_numpy(np.ascontiguousarray(np.stack([w.ynew for w in wls], 1).reshape(T + 5, B * k))).to(dev)
M = G * G
ctx = _lib.context()
models = []
for w in wls:
    m = _lib.Model(ctx, _lib.MF, hyp, 1e-8)
    m.set_grid(w.xs)
    m.set_data(w.XL, w.yL, w.XH, w.yH)
    models.append(m)
mu = torch.empty(B * M, dtype=torch.float64, device=dev)
var = torch.empty(B * M, dtype=torch.float64, device=dev)
vmax = torch.zeros(T + 5, B, dtype=torch.float64, device=dev)
_lib.batch_predict(models, mu.data_ptr(), var.data_ptr())
ks = [k] * B
acc = {"truncate x8": 0.0, "tensor views": 0.0, "batch_append_predict": 0.0}
for s in range(T + 5):
    t0 = time.perf_counter()
    for m in models:
        m.truncate(NH0)
    t1 = time.perf_counter()
    xp, yp, vp = Xn[s].data_ptr(), yn[s].data_ptr(), vmax[s].data_ptr()
    t2 = time.perf_counter()
    _lib.batch_append_predict(models, xp, yp, ks, mu.data_ptr(), var.data_ptr(), asynchronous=True, vmax_ptr=vp)
    t3 = time.perf_counter()
    if s >= 5:
        acc["truncate x8"] += t1 - t0
        acc["tensor views"] += t2 - t1
        acc["batch_append_predict"] += t3 - t2
ctx.synchronize()
print({kk: round(1e6 * v / T, 1) for kk, v in acc.items()}, "us per step", models[0].stats())
