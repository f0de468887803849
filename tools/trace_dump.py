"""Diagnostic: run the headline lattice step with a -DMFGP_STAMPS library (argv[1]) and
save the raw per-workgroup stamps of the last step to argv[2] (.npz) for offline
analysis (tools/trace_analyze.py). Rows: g_stamps[64 + 8 * linear WG id + slot]; slot 7
holds the HW_ID / XCC_ID registers. Launch 1's WGs are (GP, role) with the GP fastest;
k_lat_gemm2's WGs sit at 1024 + tile (WTRACE2)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MFGP_LIB"] = sys.argv[1]
sys.path.insert(0, ROOT)
import numpy as np
import torch
from mfgp_coverage_amd import _lib, synthetic

B = int(os.environ.get("TRACE_B", "8"))
G, NL, NH, k = 128, 1024, 1024, 8
T = int(os.environ.get("TRACE_T", "12"))
NH0 = NH - k
M = G * G
hyp = synthetic.HYP["australia8_mf"]
wls = [synthetic.Workload(G, NL, NH0, k, T, seed=s) for s in range(B)]
dev = torch.device("cuda", 0)
NWG = B * 2048
st = torch.zeros(64 + 8 * NWG + 64, dtype=torch.int64, device=dev)
L = _lib.lib()
L.mfgp_debug_set_stamps.argtypes = [ctypes.c_void_p]
assert L.mfgp_debug_set_stamps(ctypes.c_void_p(st.data_ptr())) == 0
Xnew = torch.from_numpy(np.ascontiguousarray(np.stack([w.Xnew for w in wls], 1).reshape(T, B * k, 2))).to(dev)
ynew = torch.from_numpy(np.ascontiguousarray(np.stack([w.ynew for w in wls], 1).reshape(T, B * k))).to(dev)
ctx = _lib.context()
ctx.set_lattice("force")
models = []
for wl in wls:
    m = _lib.Model(ctx, _lib.MF, hyp, 1e-8)
    m.set_grid(wl.xs)
    m.set_data(wl.XL, wl.yL, wl.XH, wl.yH)
    models.append(m)
mu = torch.empty(B * M, dtype=torch.float64, device=dev)
var = torch.empty(B * M, dtype=torch.float64, device=dev)
_lib.batch_predict(models, mu.data_ptr(), var.data_ptr())
reps = []
for s in range(T):
    for m in models:
        m.truncate(NH0)
    if s >= T - 3:
        torch.cuda.synchronize()
        st.zero_()
    _lib.batch_append_predict(models, Xnew[s].data_ptr(), ynew[s].data_ptr(), [k] * B, mu.data_ptr(), var.data_ptr(),
                              asynchronous=True)
    if s >= T - 3:
        ctx.synchronize()
        reps.append(st.cpu().numpy()[64:64 + 8 * NWG].reshape(NWG, 8).copy())
ctx.synchronize()
stats = models[0].stats()
assert stats["lattice"] == T, stats
np.savez_compressed(sys.argv[2], raw=np.stack(reps), B=B, stats=np.array(sorted(stats.items()), dtype=object).astype(str))
print("saved", sys.argv[2], "steps", len(reps))
