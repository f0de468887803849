"""Diagnostic: timeline of one k_inc_stream launch for GP 0 (s_memrealtime, 100 MHz),
from a -DMFGP_STAMPS build named by argv[1] (default build_diag/libmfgp_stamps.so)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MFGP_LIB"] = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "build", "libmfgp_stamps.so")
BACK_TO_BACK = "--b2b" in sys.argv   # launches back to back (stamps: max over launches = the last one)
UNFUSED = "--unfused" in sys.argv     # the append alone (producers + finish), then k_vstream
sys.path.insert(0, ROOT)
import numpy as np
import torch
from mfgp_coverage_amd import _lib, synthetic

B, G, NL, NH, k, T = 8, 128, 1024, 1024, 8, (24 if BACK_TO_BACK else 6)
NH0 = NH - k
M = G * G
hyp = synthetic.HYP["australia8_mf"]
wls = [synthetic.Workload(G, NL, NH0, k, T, seed=s) for s in range(B)]
dev = torch.device("cuda", 0)
st = torch.zeros(64 + 8 * 8 * (16 + 256) + 64, dtype=torch.int64, device=dev)   # + per-WG traces
L = _lib.lib()
L.mfgp_debug_set_stamps.argtypes = [ctypes.c_void_p]
assert L.mfgp_debug_set_stamps(ctypes.c_void_p(st.data_ptr())) == 0
Xnew = torch.from_numpy(np.ascontiguousarray(np.stack([w.Xnew for w in wls], 1).reshape(T, B * k, 2))).to(dev)
ynew = torch.from_numpy(np.ascontiguousarray(np.stack([w.ynew for w in wls], 1).reshape(T, B * k))).to(dev)
ctx = _lib.context()
if UNFUSED:
    ctx.set_fused(False)
models = []
for wl in wls:
    m = _lib.Model(ctx, _lib.MF, hyp, 1e-8)
    m.set_grid(wl.xs)
    m.set_data(wl.XL, wl.yL, wl.XH, wl.yH)
    models.append(m)
mu = torch.empty(B * M, dtype=torch.float64, device=dev)
var = torch.empty(B * M, dtype=torch.float64, device=dev)
vmax = torch.empty(T, B, dtype=torch.float64, device=dev)
for s in range(T):
    for m in models:
        m.truncate(NH0)
    if not BACK_TO_BACK or s == 0:
        torch.cuda.synchronize()
        st.zero_()
        torch.cuda.synchronize()
    _lib.batch_append_predict(models, Xnew[s].data_ptr(), ynew[s].data_ptr(), [k] * B, mu.data_ptr(), var.data_ptr(),
                              vmax_ptr=vmax[s].data_ptr(), asynchronous=BACK_TO_BACK)
    if not BACK_TO_BACK:
        torch.cuda.synchronize()
try:
    ctx.synchronize()
except Exception as e:   # diagnostic builds that compute garbage on purpose
    print("(synchronize:", type(e).__name__, ")")
v = st.cpu().numpy()
t0 = v[30]
names = {30: "producer 0 start", 38: "producers: cells found", 39: "producers: gathered", 40: "producers: partials stored",
         31: "last producer arrival", 32: "L22/z2 published", 33: "tile 0 start",
         34: "tile 0 past wait 1", 35: "tile 0 streamed", 36: "tile 0 past wait 2", 37: "last tile end"}
for i in (30, 38, 39, 40, 31, 32, 33, 34, 35, 36, 37):
    print(f"{names[i]:24s} {(v[i] - t0) / 100.0:9.2f} us")
print(models[0].stats())
