"""Where the drop-in step's time goes (one GP, the reference simulator's pattern,
simulator.py:888-892): updt_hifi split into its Python part (vstack, hyperparameter
check) and the C append call, the kernel's own duration from HIP events, an idle
stream synchronise, and predict split into its parts. Headline size by default."""
import json
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from mfgp_coverage_amd import _lib  # noqa: E402
from mfgp_coverage_amd.gaussian_process import MFGP, _as1, _as2  # noqa: E402
from mfgp_coverage_amd.synthetic import HYP, Workload  # noqa: E402

T = 70
SIZE = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--size=")), "128,1024,1016,8")
G, NL, NH0, K = (int(v) for v in SIZE.split(","))
w = Workload(G, NL, NH0, K, T, seed=0)
gp = MFGP(w.XL, w.yL.reshape(-1, 1), w.XH, w.yH.reshape(-1, 1), 1, 1)
gp.hyp = HYP["australia8_mf"].copy()
gp.updt_info(gp.X_L, gp.y_L, gp.X_H, gp.y_H)
gp.predict(w.xs)
ctx = _lib.context()
parts = {k: [] for k in ("updt_hifi", "vstack", "push_hyp", "c_append", "kernel", "sync_idle", "predict",
                         "grid_check", "predict_view", "step")}
timing = "--timing" in sys.argv
for s in range(T):
    if timing:
        ctx.enable_timing(True, predict_only=True)
        ctx.set_timing_stride(1)
        ctx.reset_timing()
    Xa, ya = w.Xnew[s], w.ynew[s].reshape(-1, 1)
    t0 = time.perf_counter()
    # updt_hifi, statement by statement (gaussian_process.MFGP.updt_hifi)
    prev = (gp.X_L, gp.y_L, gp.X_H, gp.y_H)
    gp.X_H = np.vstack((gp.X_H, Xa))
    gp.y_H = np.vstack((gp.y_H, ya))
    t1 = time.perf_counter()
    syn = gp.__dict__.get("_synced")
    assert syn is not None and all(a is b for a, b in zip(syn, prev))
    gp._push_hyp()
    gp.__dict__["_synced"] = None
    t2 = time.perf_counter()
    gp._dev().append(_as2(Xa), _as1(ya))
    t3 = time.perf_counter()
    gp.__dict__["_synced"] = (gp.X_L, gp.y_L, gp.X_H, gp.y_H)
    t4 = time.perf_counter()
    ctx.synchronize()
    t5 = time.perf_counter()
    gp._grid_to_device(w.xs)
    t6 = time.perf_counter()
    mu, var = gp._dev().predict_view()
    t7 = time.perf_counter()
    if timing:
        tm = ctx.timing()
        parts["kernel"].append(tm["predict_ms"] * 1e-3 / max(1, tm["predict_launches"]))
        ctx.enable_timing(False)
    parts["updt_hifi"].append(t4 - t0)
    parts["vstack"].append(t1 - t0)
    parts["push_hyp"].append(t2 - t1)
    parts["c_append"].append(t3 - t2)
    parts["sync_idle"].append(t5 - t4)
    parts["grid_check"].append(t6 - t5)
    parts["predict_view"].append(t7 - t6)
    parts["predict"].append(t7 - t5)
    parts["step"].append((t4 - t0) + (t7 - t5))
print(json.dumps({"size": SIZE, "timing_events": timing,
                  "us_median": {k: round(1e6 * float(np.median(v[10:])), 1) for k, v in parts.items() if v},
                  "stats": {k: v for k, v in gp._dev().stats().items() if k in ("lattice", "vstream", "inc_factor")}}))
