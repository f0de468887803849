import sys, os, copy
sys.path.insert(0, os.getcwd())
import numpy as np
from tests.test_gpu_incremental import _points, HYP_MF
from mfgp_coverage_amd import gaussian_process as gpm
Xs, X, y = _points(40, 400, seed=9, ongrid=True)
m = gpm.MFGP(X[:200], y[:200, None], X[200:380], y[200:380, None], 1, 1)
m.hyp = HYP_MF.copy()
m.updt_info(m.X_L, m.y_L, m.X_H, m.y_H)
mu0, cov0 = m.predict(Xs)
mu1, cov1 = m.predict(Xs)
d = np.nonzero(mu0[:, 0] != mu1[:, 0])[0]
print("mu diff cells", len(d), d[:40])
dv = np.nonzero(np.diag(cov0) != np.diag(cov1))[0]
print("var diff cells", len(dv), dv[:40])
print(m._dev().stats())
