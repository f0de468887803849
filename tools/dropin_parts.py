import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np
from mfgp_coverage_amd import set_deferred_appends
from mfgp_coverage_amd.gaussian_process import MFGP
from mfgp_coverage_amd.synthetic import HYP, Workload
set_deferred_appends(True)
T = 60
w = Workload(128, 1024, 1016, 8, T, seed=0)
gp = MFGP(w.XL, w.yL.reshape(-1, 1), w.XH, w.yH.reshape(-1, 1), 1, 1)
gp.hyp = HYP["australia8_mf"].copy()
gp.updt_info(gp.X_L, gp.y_L, gp.X_H, gp.y_H)
gp.predict(w.xs)
parts = {k: [] for k in ("append", "sync_data", "push_hyp", "grid", "dev_predict", "wrap")}
for s in range(T):
    t0 = time.perf_counter(); gp.updt_hifi(w.Xnew[s], w.ynew[s].reshape(-1, 1)); t1 = time.perf_counter()
    gp._sync_data(); t2 = time.perf_counter()
    gp._push_hyp(); t3 = time.perf_counter()
    gp._grid_to_device(w.xs); t4 = time.perf_counter()
    mu, var = gp._dev().predict(); t5 = time.perf_counter()
    from mfgp_coverage_amd.gaussian_process import DiagCov
    out = (mu.reshape(-1, 1), DiagCov(var)); t6 = time.perf_counter()
    for k, a, b in (("append", t0, t1), ("sync_data", t1, t2), ("push_hyp", t2, t3), ("grid", t3, t4), ("dev_predict", t4, t5), ("wrap", t5, t6)):
        parts[k].append(b - a)
print({k: round(1e6 * float(np.median(v[10:])), 1) for k, v in parts.items()})
