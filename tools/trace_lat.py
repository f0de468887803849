"""Diagnostic: per-workgroup timeline of k_inc_lat (a -DMFGP_STAMPS build, argv[1]).
Slots: producers 0 start / 1 arrival / 4 end; w blocks 0 start / 1 past the L21 wait / 3 F loop done /
2 published; Z units 0 start / 1 scanned / 3 past the w wait / 2 published; GEMM 0 start / 1 past
the Z wait / 2 K loop done / 3 past the
L22 wait (reducers) / 5 new-row factors and L22^-1 done / 6 cells done / 4 end. Launches back to back; the trace is the last launch's."""
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
ctx.set_lattice("force")   # B = 1: past the cost gate
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
assert models[0].stats()["lattice"] == T, models[0].stats()
raw = st.cpu().numpy()[64:64 + 8 * NWG].reshape(NWG, 8)
tr = raw[:, :7].astype(np.float64)
used = tr[:, 0] > 0
t0 = tr[used, 0].min()
tr = np.where(tr > 0, (tr - t0) / 100.0, np.nan)   # us (100 MHz realtime counter)
nprod, nwb = 16, 32
# the host's rule (mfgp_capi.hip): two w units per CU over the batch (MFGP_LAT_WU: the
# total), each GP's count by its F steps (equal n0 here)
n0 = NL + NH0
C16 = (n0 + 15) // 16
wsteps = nwb * C16 - 2 * nwb * (nwb - 1)
wu_total = int(os.environ.get("MFGP_LAT_WU", "0")) or min(512, max(128, B * wsteps // 8))
nwu = max(1, min((wu_total * wsteps + (B * wsteps) // 2) // (B * wsteps), 512, wsteps))
wr = nwu
wch = wr
_zq = 2 * 256 // (((G + 63) // 64) * 64)
nzu = 2 * ((G + _zq - 1) // _zq)
role = np.arange(NWG) // B
# the two scan units are the first roles of launch 1 (k_lat_gemm2's stamps sit at 1024 + tile)
role = np.where(role >= 1024, role, role - int(os.environ.get("TRACE_ROFF", "2")))
G2 = bool(used[role >= 1024].any())   # the GEMM as a second launch (k_lat_gemm2): roles 1024 + tile
q = lambda a: " ".join(f"{np.nanpercentile(a, p):7.1f}" for p in (0, 10, 50, 90, 100)) if np.isfinite(a).any() else "-"
print(f"B={B} ({nwu} w units, {nzu} Z units per GP): percentiles 0/10/50/90/100 (us from the first WG start); last WG end {np.nanmax(tr):.1f}")
for name, sel, slots in (("producer", role < nprod, (0, 1, 4)), ("w unit", (role >= nprod) & (role < nprod + nwu), (0, 1, 3, 2)),
                         ("Z unit", (role >= nprod + nwu) & (role < nprod + nwu + nzu), (0, 1, 3, 4, 5, 6, 2)),
                         ("gemm", ((role >= 1024) if G2 else (role >= nprod + nwu + nzu)) & used,
                          (0, 2, 3, 6, 4) if G2 else (0, 1, 2, 3, 5, 6, 4))):
    for sl in slots:
        print(f"  {name:9s} slot {sl}: {q(tr[sel, sl])}")
gm = ((role >= 1024) if G2 else (role >= nprod + nwu + nzu)) & used
w = tr[(role >= nprod) & (role < nprod + nwu)]
print(f"  w units published (slot 2, last arrivers): {q(w[:, 2])}")
print(f"  w unit F loop (slot 3 - slot 1): {q(w[:, 3] - w[:, 1])}; reduce+publish (2 - 3): {q(w[:, 2] - w[:, 3])}")
print(f"  gemm K-loop durations (slot2 - slot1): {q(tr[gm, 2] - tr[gm, 1])}")
red = gm & np.isfinite(tr[:, 3])
print(f"  reducers: reduce+L22 wait (3 - 2) {q(tr[red, 3] - tr[red, 2])}; Fn/Li (5 - 3) {q(tr[red, 5] - tr[red, 3])}; "
      f"cells (6 - 5) {q(tr[red, 6] - tr[red, 5])}; argmax (4 - 6) {q(tr[red, 4] - tr[red, 6])}")
S = int(os.environ.get("MFGP_LAT_KSPLIT", "0")) or None
if S:
    g = role - nprod - nwu - nzu
    tiles = 16
    for sp in range(S):
        sel = gm & (g // tiles == sp)
        print(f"  split {sp}: start {q(tr[sel, 1])} | loop end {q(tr[sel, 2])}")
# placement: GEMM workgroups per CU (XCC, SE, SH, CU from the HW_ID / XCC_ID
# registers) and the K-loop duration against that count
hw = raw[:, 7]
cu = ((hw >> 32) & 0xF) * 1024 + ((hw >> 13) & 0x7) * 64 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 0xF)
gcu = cu[gm]
ucu, cnt = np.unique(gcu, return_counts=True)
print("  GEMM WGs per CU: histogram", dict(zip(*np.unique(cnt, return_counts=True))), "over", len(ucu), "CUs")
per = dict(zip(ucu, cnt))
ncnt = np.array([per[c] for c in gcu])
dur = tr[gm, 2] - tr[gm, 1]
for n in sorted(set(ncnt)):
    print(f"    CUs with {n} GEMM WGs: K-loop {q(dur[ncnt == n])}")
wsel = (role >= nprod) & (role < nprod + nwu)
wcu = dict(zip(*np.unique(cu[wsel], return_counts=True)))
nw = np.array([wcu.get(c, 0) for c in gcu])
for n in sorted(set(nw)):
    print(f"    GEMM WGs sharing their CU with {n} w units: K-loop {q(dur[nw == n])}")
# per w unit (index within its GP): start of its F loop, loop duration, end (medians over the GPs)
wsel_all = (role >= nprod) & (role < nprod + nwu) & used
uidx = role - nprod
st_ = {u: [] for u in range(nwu)}
for i in np.nonzero(wsel_all)[0]:
    st_[int(uidx[i])].append((tr[i, 1], tr[i, 3] - tr[i, 1], tr[i, 3]))
rows = []
for u in range(nwu):
    if st_[u]:
        a = np.array(st_[u])
        rows.append((u, *np.median(a, 0)))
print("  w unit: index, start, F-loop duration, end (medians over GPs)")
for r in rows:
    print("   ", f"{r[0]:3d} {r[1]:6.1f} {r[2]:6.1f} {r[3]:6.1f}")
