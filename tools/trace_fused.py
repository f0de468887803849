"""Diagnostic: per-workgroup timeline of k_inc_stream (a -DMFGP_STAMPS build, argv[1]).
Slots per WG: 0 start, 1 past L21 wait (producers: arrival), 2 streamed, 3 past L22 wait, 4 end.
--b2b: launches back to back (the trace is the last launch's). Prints a summary and
saves gpurun_out/trace_<tag>.npz."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MFGP_LIB"] = sys.argv[1]
B2B = "--b2b" in sys.argv
sys.path.insert(0, ROOT)
import numpy as np
import torch
from mfgp_coverage_amd import _lib, synthetic

B = int(os.environ.get("TRACE_B", "8"))
G, NL, NH, k = 128, 1024, 1024, 8
T = 24 if B2B else 6
NH0 = NH - k
M = G * G
hyp = synthetic.HYP["australia8_mf"]
wls = [synthetic.Workload(G, NL, NH0, k, T, seed=s) for s in range(B)]
dev = torch.device("cuda", 0)
NWG = B * (16 + 1024)   # room for the row-split launches of small batches
st = torch.zeros(64 + 8 * NWG + 64, dtype=torch.int64, device=dev)
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
vmax = torch.empty(T, B, dtype=torch.float64, device=dev)
for s in range(T):
    for m in models:
        m.truncate(NH0)
    if not B2B:
        torch.cuda.synchronize()
    _lib.batch_append_predict(models, Xnew[s].data_ptr(), ynew[s].data_ptr(), [k] * B, mu.data_ptr(), var.data_ptr(),
                              vmax_ptr=vmax[s].data_ptr(), asynchronous=B2B)
    if not B2B:
        torch.cuda.synchronize()
ctx.synchronize()
raw = st.cpu().numpy()[64:64 + 8 * NWG].reshape(NWG, 8)
hw = raw[:, 7].copy()                       # (XCC_ID << 32) | HW_ID of each workgroup
tr = raw[:, :5].astype(np.float64)
t0 = tr[:, 0][tr[:, 0] > 0].min()
tr = np.where(tr > 0, (tr - t0) / 100.0, np.nan)   # us
nprod = 16
role = np.arange(NWG) // B
prod, tiles = tr[role < nprod], tr[role >= nprod]
tag = os.path.basename(sys.argv[1]).replace("libmfgp_", "").replace(".so", "") + ("_b2b" if B2B else "") + f"_B{B}"
np.savez(os.path.join(ROOT, "gpurun_out", f"trace_{tag}.npz"), tr=tr, hw=hw)
q = lambda a: " ".join(f"{np.nanpercentile(a, p):7.1f}" for p in (0, 10, 50, 90, 100))
print(f"[{tag}] percentiles 0/10/50/90/100 (us from the first WG start)")
print("producer start      ", q(prod[:, 0]))
print("producer arrival    ", q(prod[:, 1]))
print("producer end        ", q(prod[:, 4]))
fin = prod[~np.isnan(prod[:, 3])]
print("finish: L22 published", q(fin[:, 3]), " phase 2 end", q(fin[:, 2]))
print("tile start          ", q(tiles[:, 0]))
print("tile past L21 wait  ", q(tiles[:, 1]))
print("tile streamed       ", q(tiles[:, 2]))
print("tile past L22 wait  ", q(tiles[:, 3]))
print("tile end            ", q(tiles[:, 4]))
print("stream us per tile  ", q(tiles[:, 2] - tiles[:, 1]))
print("epilogue us per tile", q(tiles[:, 4] - tiles[:, 2]))
print("L22 wait us per tile", q(tiles[:, 3] - tiles[:, 2]))
print("startup us per tile ", q(tiles[:, 1] - tiles[:, 0]))
# bandwidth over time: tiles streaming concurrently, in 10 us bins
edges = np.arange(0, np.nanmax(tiles[:, 4]) + 10, 10)
conc = [int(np.sum((tiles[:, 1] <= e) & (tiles[:, 2] > e))) for e in edges]
print("streaming tiles per 10 us:", conc)
