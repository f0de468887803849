"""Diagnostic: k_vstream / k_inc_stream rate with and without the appended rows' MFMA
(k = 8 bordered appends vs k = 0 re-predicts of the same resident V), HIP-event timed."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from mfgp_coverage_amd import _lib, synthetic

B, G, NL, NH, k, T = 8, 128, 1024, 1024, 8, 40
NH0 = NH - k
M = G * G
hyp = synthetic.HYP["australia8_mf"]
wls = [synthetic.Workload(G, NL, NH0, k, T, seed=s) for s in range(B)]
dev = torch.device("cuda", 0)
Xnew = torch.from_numpy(np.ascontiguousarray(np.stack([w.Xnew for w in wls], 1).reshape(T, B * k, 2))).to(dev)
ynew = torch.from_numpy(np.ascontiguousarray(np.stack([w.ynew for w in wls], 1).reshape(T, B * k))).to(dev)
ctx = _lib.context()
models = []
for wl in wls:
    m = _lib.Model(ctx, _lib.MF, hyp, 1e-8)
    m.set_grid(wl.xs)
    m.set_data(wl.XL, wl.yL, wl.XH, wl.yH)
    models.append(m)
mu = torch.empty(B * M, dtype=torch.float64, device=dev)
var = torch.empty(B * M, dtype=torch.float64, device=dev)
for fused in (True, False):
    ctx.set_fused(fused)
    for kk in (k, 0):
        for s in range(4):
            for m in models:
                m.truncate(NH0)
            _lib.batch_append_predict(models, Xnew[s].data_ptr(), ynew[s].data_ptr(), [k] * B, mu.data_ptr(), var.data_ptr())
        ctx.synchronize()
        ctx.enable_timing(True, predict_only=True)
        ctx.reset_timing()
        for s in range(4, T):
            if kk:
                for m in models:
                    m.truncate(NH0)
            _lib.batch_append_predict(models, Xnew[s].data_ptr(), ynew[s].data_ptr(), [kk] * B, mu.data_ptr(),
                                      var.data_ptr())
        ctx.synchronize()
        tm = ctx.timing()
        ctx.enable_timing(False)
        n0 = NL + NH0 if kk else NL + NH
        ms = tm["predict_ms"] / tm["predict_launches"]
        by = B * 8 * M * n0
        print(f"fused={fused} k={kk}: {ms * 1e3:7.1f} us per launch, V_old {by / 1e9:.3f} GB -> {by / ms / 1e9:.2f} TB/s")
