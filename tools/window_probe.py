"""Why a 20-step timed window runs slower per step than a 200-step one (VERDICT r03
item 7): the headline step (8 australia8 MF GPs, 128x128, N = 2048, the lattice
step) timed in windows of W steps bracketed by device synchronisation like
bench.py, back to back, after an idle sleep, and with HIP events around the
window's first and last step."""
import json
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mfgp_coverage_amd import _lib, synthetic  # noqa: E402

B, G, NL, NH, k = 8, 128, 1024, 1024, 8
NH0 = NH - k
S = 64
dev = torch.device("cuda", 0)
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
hyp = synthetic.HYP["australia8_mf"]
wls = [synthetic.Workload(G, NL, NH0, k, S, seed=s) for s in range(B)]
M = G * G
Xnew = torch.from_numpy(np.ascontiguousarray(np.stack([w.Xnew for w in wls], 1).reshape(S, B * k, 2))).to(dev)
ynew = torch.from_numpy(np.ascontiguousarray(np.stack([w.ynew for w in wls], 1).reshape(S, B * k))).to(dev)
mu = torch.empty(B * M, dtype=torch.float64, device=dev)
var = torch.empty(B * M, dtype=torch.float64, device=dev)
vmax = torch.zeros(S, B, dtype=torch.float64, device=dev)
ctx = _lib.context()
ctx.set_stream(stream.cuda_stream)
models = []
for w in wls:
    m = _lib.Model(ctx, _lib.MF, hyp, 1e-8)
    m.set_grid(w.xs)
    m.set_data(w.XL, w.yL, w.XH, w.yH)
    models.append(m)
_lib.batch_predict(models, mu.data_ptr(), var.data_ptr())
batch = _lib.Batch(models, [k] * B)
xp, yp, vp = Xnew.data_ptr(), ynew.data_ptr(), vmax.data_ptr()


def step(s):
    s %= S
    batch.truncate(NH0)
    batch.append_predict(xp + s * B * k * 16, yp + s * B * k * 8, mu.data_ptr(), var.data_ptr(), asynchronous=True,
                         vmax_ptr=vp + s * B * 8)


for s in range(400):
    step(s)
ctx.synchronize()
out = {}


def window(n, label, sleep_s=0.0, events=False):
    res = []
    for rep in range(5):
        if sleep_s:
            time.sleep(sleep_s)
        torch.cuda.synchronize(dev)
        e0, e1, e2, e3 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
        t0 = time.perf_counter()
        for i in range(n):
            if events and i == 0:
                e0.record(stream)
            step(i)
            if events and i == 0:
                e1.record(stream)
            if events and i == n - 1:
                e2.record(stream)
        if events:
            e3.record(stream)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        r = {"us_per_step": 1e6 * (t1 - t0) / n}
        if events:
            r["first_step_us"] = 1e3 * e0.elapsed_time(e1)
            r["last_step_us"] = 1e3 * e2.elapsed_time(e3)
            r["gpu_span_us"] = 1e3 * e0.elapsed_time(e3)
            r["wall_us"] = 1e6 * (t1 - t0)
        res.append(r)
    out[label] = res


window(20, "w20")
window(200, "w200")
window(20, "w20_events", events=True)
window(20, "w20_after_5ms_idle", sleep_s=0.005)
window(20, "w20_after_50ms_idle", sleep_s=0.05)
window(60, "w60")
print(json.dumps(out))
