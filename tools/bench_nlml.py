"""Time likelihood + analytic gradient (mfgp_nlml) at N = 2048 (MF, australia9
hyperparameters) on the device, and the oracle's NumPy version on the host."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402


def main():
    from mfgp_coverage_amd import _lib, synthetic
    from oracle import gp_oracle as O
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    hyp = synthetic.HYP["australia9_mf"]
    wl = synthetic.Workload(128, N // 2, N - N // 2, 1, 1, seed=0)
    m = _lib.Model(_lib.context(), _lib.MF, hyp, 1e-8)
    m.set_data(wl.XL, wl.yL, wl.XH, wl.yH)
    m.nlml(hyp, grad=True)
    t0 = time.perf_counter()
    R = 5
    for _ in range(R):
        v, g = m.nlml(hyp, grad=True)
    gpu = (time.perf_counter() - t0) / R
    t0 = time.perf_counter()
    O.nlml(wl.XH, wl.yH, hyp, XL=wl.XL, yL=wl.yL, grad=True)
    cpu = time.perf_counter() - t0
    print(json.dumps({"N": N, "gpu_ms": gpu * 1e3, "cpu_oracle_ms": cpu * 1e3, "nlml": v}))


if __name__ == "__main__":
    main()
