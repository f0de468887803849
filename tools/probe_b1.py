"""One GP at the headline size (128x128, N = 2048, 8 new rows per step) through the
batched API on the V stream (k_inc_stream1; argv[2] "lat": the lattice step forced): steps back to back (asynchronous) and
steps separated by a host pause with a synchronise each (the drop-in simulator's
pattern), so that rocprofv3's kernel trace can tell the kernel's own duration in
both. argv: pause in microseconds (0 = back to back)."""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mfgp_coverage_amd import _lib, synthetic  # noqa: E402

PAUSE_US = float(sys.argv[1]) if len(sys.argv) > 1 else 0.0
LATTICE = len(sys.argv) > 2 and sys.argv[2] == "lat"   # the lattice step forced instead of the V stream
G, NL, NH, k, S = 128, 1024, 1024, 8, 64
NH0 = NH - k
dev = torch.device("cuda", 0)
wl = synthetic.Workload(G, NL, NH0, k, S, seed=0)
ctx = _lib.context()
ctx.set_lattice("force" if LATTICE else False)
m = _lib.Model(ctx, _lib.MF, synthetic.HYP["australia8_mf"], 1e-8)
m.set_grid(wl.xs)
m.set_data(wl.XL, wl.yL, wl.XH, wl.yH)
M = G * G
mu = torch.empty(M, dtype=torch.float64, device=dev)
var = torch.empty(M, dtype=torch.float64, device=dev)
_lib.batch_predict([m], mu.data_ptr(), var.data_ptr())
Xn = torch.from_numpy(np.ascontiguousarray(wl.Xnew)).to(dev)
yn = torch.from_numpy(np.ascontiguousarray(wl.ynew)).to(dev)
batch = _lib.Batch([m], [k])
torch.cuda.synchronize()
t0 = time.perf_counter()
T = 300
for s in range(T):
    batch.truncate(NH0)
    batch.append_predict(Xn.data_ptr() + (s % S) * k * 16, yn.data_ptr() + (s % S) * k * 8, mu.data_ptr(),
                         var.data_ptr(), asynchronous=True)
    if PAUSE_US > 0:
        ctx.synchronize()
        t = time.perf_counter()
        while (time.perf_counter() - t) * 1e6 < PAUSE_US:
            pass
ctx.synchronize()
print({"pause_us": PAUSE_US, "us_per_step": round(1e6 * (time.perf_counter() - t0) / T, 1), "stats": m.stats()})
