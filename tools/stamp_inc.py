"""Diagnostic: phase stamps (s_memtime) of the incremental kernels (build_diag/libmfgp_stamps.so)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MFGP_LIB"] = os.path.join(ROOT, "build_diag", "libmfgp_stamps.so")
sys.path.insert(0, ROOT)
import numpy as np
import torch
from mfgp_coverage_amd import _lib, synthetic

B, G, NL, NH, k, T = 8, 128, 1024, 1024, 8, 6
NH0 = NH - k
M = G * G
hyp = synthetic.HYP["australia8_mf"]
wls = [synthetic.Workload(G, NL, NH0, k, T, seed=s) for s in range(B)]
dev = torch.device("cuda", 0)
st = torch.zeros(64, dtype=torch.int64, device=dev)
L = _lib.lib()
L.mfgp_debug_set_stamps.argtypes = [ctypes.c_void_p]
assert L.mfgp_debug_set_stamps(ctypes.c_void_p(st.data_ptr())) == 0
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
for s in range(T):
    for m in models:
        m.truncate(NH0)
    _lib.batch_append_predict(models, Xnew[s].data_ptr(), ynew[s].data_ptr(), [k] * B, mu.data_ptr(), var.data_ptr())
torch.cuda.synchronize()
v = st.cpu().numpy()
names = {21: "init+Lb", 22: "ssum", 23: "Ln", 24: "chol+z2", 25: "linv"}
for i in range(21, 26):
    print(f"{names[i]:10s} {v[i] - v[i-1]:8d} ticks")
print("total", v[25] - v[20])
