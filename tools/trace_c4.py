"""Diagnostic: per-workgroup timeline of k_inc_lat at configs[4]'s size (a -DMFGP_STAMPS
build, argv[1]): 32 MFGP_F32 GPs, 256x256, N_L = N_H = 4096, one launch (producers, w
units, Z units, GEMM tiles as roles). Slots as in tools/trace_lat.py."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MFGP_LIB"] = sys.argv[1]
sys.path.insert(0, ROOT)
import numpy as np
import torch
from mfgp_coverage_amd import _lib, synthetic

B = int(os.environ.get("TRACE_B", "32"))
G, NL, NH, k = 256, 4096, 4096, 8
T = 4
NH0 = NH - k
M = G * G
hyp = synthetic.HYP["australia9_mf"]
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
models = []
for wl in wls:
    m = _lib.Model(ctx, _lib.MF, hyp, 1e-8, dtype=_lib.F32)
    m.set_grid(wl.xs)
    m.set_data(wl.XL, wl.yL, wl.XH, wl.yH)
    models.append(m)
mu = torch.empty(B * M, dtype=torch.float64, device=dev)
var = torch.empty(B * M, dtype=torch.float64, device=dev)
_lib.batch_predict(models, mu.data_ptr(), var.data_ptr())
for s in range(T):
    for m in models:
        m.truncate(NH0)
    if s == T - 1:
        torch.cuda.synchronize()
        st.zero_()
    _lib.batch_append_predict(models, Xnew[s].data_ptr(), ynew[s].data_ptr(), [k] * B, mu.data_ptr(), var.data_ptr(),
                              asynchronous=True)
ctx.synchronize()
print(models[0].stats())
raw = st.cpu().numpy()[64:64 + 8 * NWG].reshape(NWG, 8)
tr = raw[:, :7].astype(np.float64)
used = tr[:, 0] > 0
t0 = tr[used, 0].min()
tr = np.where(tr > 0, (tr - t0) / 100.0, np.nan)
role = np.arange(NWG) // B - int(os.environ.get("TRACE_ROFF", "2"))   # (the scan units: the first roles)
n0 = NL + NH0
nprod = -(-n0 // 128)
C = -(-n0 // 16)
nwb = -(-n0 // 64)
wsteps = nwb * C - 2 * nwb * (nwb - 1)
ncu = 256
wsum = B * wsteps
wu_total = max(ncu // 2, wsum // 8)
if wu_total > 2 * ncu:
    wu_total = max(2 * ncu, min(8 * ncu, wsum // 512))
nwu = max(1, min((wu_total * wsteps + wsum // 2) // wsum, 512, wsteps))
tabw = 256
zq = 2 * 256 // tabw
nzu = 2 * (-(-G // zq))
q = lambda a: " ".join(f"{np.nanpercentile(a, p):8.1f}" for p in (0, 10, 50, 90, 100)) if np.isfinite(a).any() else "-"
print(f"B={B}: nprod {nprod}, nwu {nwu}, nzu {nzu}; last stamp {np.nanmax(tr):.1f} us; percentiles 0/10/50/90/100")
bands = (("producer", (role < nprod), (0, 1, 4)), ("w unit", (role >= nprod) & (role < nprod + nwu), (0, 1, 3, 2)),
         ("Z unit", (role >= nprod + nwu) & (role < nprod + nwu + nzu), (0, 1, 3, 4, 5, 6, 2)),
         ("gemm", (role >= nprod + nwu + nzu) & used, (0, 1, 2, 3, 5, 6, 4)))
for name, sel, slots in bands:
    sel = sel & used
    print(f"  {name}: {int(sel.sum())} WGs")
    for sl in slots:
        print(f"    slot {sl}: {q(tr[sel, sl])}")
