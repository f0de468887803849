"""Diagnostic: per-workgroup timeline of the g3 lattice step (a -DMFGP_STAMPS build,
argv[1]): launch 1's roles (scan units first) end, then k_lat_gemm3's phases: slots
0 start / 5 prologue issued / 1 chunks summed / 2 K loop (and virtual chunks) done / 3 T~ stored /
6 cells done / 4 end. Headline batch (B = 8, 128x128, N = 2048); the last step."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MFGP_LIB"] = sys.argv[1]
sys.path.insert(0, ROOT)
import numpy as np
import torch
from mfgp_coverage_amd import _lib, synthetic

B = int(os.environ.get("TRACE_B", "8"))
G, NL, NH, k = 128, 1024, 1024, 8
T = 12
NH0 = NH - k
M = G * G
hyp = synthetic.HYP["australia8_mf"]
SEEDS = [int(v) for v in os.environ.get("TRACE_SEEDS", ",".join(str(s) for s in range(B))).split(",")]
wls = [synthetic.Workload(G, NL, NH0, k, T, seed=SEEDS[s]) for s in range(B)]
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
CHECK = os.environ.get("TRACE_NOCHECK") is None
raw = st.cpu().numpy()[64:64 + 8 * NWG].reshape(NWG, 8)
tr = raw[:, :7].astype(np.float64)
used = tr[:, 0] > 0
t0 = tr[used, 0].min()
tr = np.where(tr > 0, (tr - t0) / 100.0, np.nan)
role = np.arange(NWG) // B
q = lambda a: " ".join(f"{np.nanpercentile(a, p):7.1f}" for p in (0, 10, 50, 90, 100)) if np.isfinite(a).any() else "-"
l1 = (role < 1024) & used
gm = (role >= 1024) & used
print(f"B={B}: launch-1 WGs {l1.sum()}, last stamp {np.nanmax(tr[l1]):.1f}; gemm WGs {gm.sum()}; percentiles 0/10/50/90/100 us")
for sl in (0, 5, 1, 2, 3, 6, 4):
    print(f"  gemm slot {sl}: {q(tr[gm, sl])}")
print(f"  prologue (5-0): {q(tr[gm, 5] - tr[gm, 0])}; chunks + Z rows (1-5): {q(tr[gm, 1] - tr[gm, 5])}")
print(f"  K loop (2-1): {q(tr[gm, 2] - tr[gm, 1])}")
print(f"  T~ (3-2): {q(tr[gm, 3] - tr[gm, 2])}; cells (6-3): {q(tr[gm, 6] - tr[gm, 3])}; argmax (4-6): {q(tr[gm, 4] - tr[gm, 6])}")
# K-loop duration by XCD, by GP and by tile (which workgroups are slow)
hw = raw[:, 7]
xcc = (hw >> 32) & 0xF
gp_ = np.arange(NWG) % B
tile = role - 1024
dur = tr[:, 2] - tr[:, 1]
for name, key in (("xcc", xcc), ("gp", gp_)):
    print(f"  K loop by {name}:", {int(v): round(float(np.nanmedian(dur[gm & (key == v)])), 1) for v in np.unique(key[gm])})
print("  K loop by tile (median over GPs):", [round(float(np.nanmedian(dur[gm & (tile == t)])), 1) for t in range(32)])
cu = ((hw >> 32) & 0xF) * 1024 + ((hw >> 13) & 0x7) * 64 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 0xF)
ucu, cnt = np.unique(cu[gm], return_counts=True)
print("  gemm WGs per CU:", dict(zip(*np.unique(cnt, return_counts=True))))
