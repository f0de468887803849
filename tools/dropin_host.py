"""Diagnostic: the host side of the drop-in step (one GP at the headline size, the
reference simulator's pattern): the C append of 8 rows split into enqueue and wait,
against a no-op C call, with the library's default wait and with HIP's spin
scheduling (hipDeviceScheduleSpin set before the context: --spin).
usage: python tools/dropin_host.py [--spin] [--lattice]"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

if "--spin" in sys.argv:
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipSetDeviceFlags(ctypes.c_uint(1)) == 0   # hipDeviceScheduleSpin
from mfgp_coverage_amd import _lib  # noqa: E402
from mfgp_coverage_amd.synthetic import HYP, Workload  # noqa: E402

T = 80
G, NL, NH0, K = 128, 1024, 1016, 8
w = Workload(G, NL, NH0, K, T, seed=0)
ctx = _lib.context()
if "--lattice" in sys.argv:
    ctx.set_lattice("force")
m = _lib.Model(ctx, _lib.MF, HYP["australia8_mf"], 1e-8)
m.set_grid(w.xs)
m.set_data(w.XL, w.yL, w.XH, w.yH)
m.predict()
out = (ctypes.c_int64 * 13)()
L = _lib.lib()
parts = {k: [] for k in ("noop", "append_sync", "append_enqueue", "wait", "predict_view")}
for s in range(T):
    Xa, ya = np.ascontiguousarray(w.Xnew[s]), np.ascontiguousarray(w.ynew[s])
    t0 = time.perf_counter()
    L.mfgp_model_stats(m.handle, out, 13)
    t1 = time.perf_counter()
    m.append(Xa, ya)                       # the drop-in's eager append: enqueue + wait inside
    t2 = time.perf_counter()
    mu, var = m.predict_view()
    t3 = time.perf_counter()
    parts["noop"].append(t1 - t0)
    parts["append_sync"].append(t2 - t1)
    parts["predict_view"].append(t3 - t2)
    del mu, var
m2 = _lib.Model(ctx, _lib.MF, HYP["australia8_mf"], 1e-8)
m2.set_grid(w.xs)
m2.set_data(w.XL, w.yL, w.XH, w.yH)
m2.predict()
import torch  # noqa: E402
mu_d = torch.empty(G * G, dtype=torch.float64, device="cuda")
var_d = torch.empty(G * G, dtype=torch.float64, device="cuda")
for s in range(T):
    Xa, ya = np.ascontiguousarray(w.Xnew[s]), np.ascontiguousarray(w.ynew[s])
    t0 = time.perf_counter()
    _lib.batch_append_predict([m2], Xa.ctypes.data, ya.ctypes.data, [K], mu_d.data_ptr(), var_d.data_ptr(),
                              asynchronous=True)
    t1 = time.perf_counter()
    ctx.synchronize()
    t2 = time.perf_counter()
    parts["append_enqueue"].append(t1 - t0)
    parts["wait"].append(t2 - t1)
print(json.dumps({"spin": "--spin" in sys.argv, "lattice": "--lattice" in sys.argv,
                  "us_median": {k: round(1e6 * float(np.median(v[10:])), 1) for k, v in parts.items()},
                  "stats": {k: v for k, v in m.stats().items() if k in ("lattice", "vstream", "inc_factor")}}))
