"""Per-step latency of the drop-in Python API for one GP (the reference simulator's
pattern, simulator.py:888-892): updt_hifi(k new samples) then predict(X*) returning
host arrays. Headline sizes: 128x128 grid, N_L = 1024, N_H = 1016 + 8 per step;
--size=G,NL,NH0,k for others. The GP grows by k rows per step (as in the simulator)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from mfgp_coverage_amd import set_deferred_appends
from mfgp_coverage_amd.gaussian_process import MFGP
from mfgp_coverage_amd.synthetic import HYP, Workload

T = 60
DEFERRED = "--deferred" in sys.argv
# --size G,NL,NH0,k (default the headline: 128x128, N_L = 1024, N_H = 1016 + 8 per step;
# the reference's native size: --size 51,121,176,4, i.e. N ~ 300)
SIZE = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--size=")), "128,1024,1016,8")
G, NL, NH0, K = (int(v) for v in SIZE.split(","))
set_deferred_appends(DEFERRED)
w = Workload(G, NL, NH0, K, T, seed=0)
gp = MFGP(w.XL, w.yL.reshape(-1, 1), w.XH, w.yH.reshape(-1, 1), 1, 1)
gp.hyp = HYP["australia8_mf"].copy()
gp.updt_info(gp.X_L, gp.y_L, gp.X_H, gp.y_H)
gp.predict(w.xs)
ts = {"updt_hifi": [], "predict": [], "np.diag+amax": []}
for s in range(T):
    t0 = time.perf_counter()
    gp.updt_hifi(w.Xnew[s], w.ynew[s].reshape(-1, 1))
    t1 = time.perf_counter()
    mu, cov = gp.predict(w.xs)
    t2 = time.perf_counter()
    v = np.diag(cov); vm = np.amax(cov)
    t3 = time.perf_counter()
    ts["updt_hifi"].append(t1 - t0); ts["predict"].append(t2 - t1); ts["np.diag+amax"].append(t3 - t2)
import json
res = {"mode": "deferred" if DEFERRED else "eager", "grid": G, "N_L": NL, "N_H": NH0 + K, "agents": K,
       "steps_timed": T - 10, "us_median": {k: round(1e6 * float(np.median(v[10:])), 1) for k, v in ts.items()},
       "stats": {k: v for k, v in gp._dev().stats().items() if k in ("lattice", "lattice_arg", "vstream", "inc_factor")}}
print(json.dumps(res))
