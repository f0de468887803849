"""Long horizons at the headline size (128x128 grid, australia8 MF): the
simulator's pattern (sim:864-892) of 150 consecutive updt_hifi(8 rows) +
predict steps, from N_L = 1024 lofi and no hifi data to N = 2224 -- every step
a bordered append on the resident V, across two 1.5x capacity reallocations
(the V rows move to the new row stride) -- checked against the oracle at every
cell at steps 1, 50, 100 and 150 (rounding drift over a real horizon). Also a
batch of 4 GPs growing the same way through the batched C ABI (every step the
lattice-separable k_inc_lat, so its drift is checked too), and an MFGP_F32 model
over the same horizon at the fp32 tolerance."""
import numpy as np
import pytest

from oracle import gp_oracle as O

pytestmark = pytest.mark.gpu

STEPS, K, NL0 = 150, 8, 1024
CHECK = (1, 50, 100, 150)


def _workload(seed):
    from mfgp_coverage_amd.synthetic import Workload
    return Workload(128, NL0, 0, K, STEPS, seed=seed)


def test_long_horizon_dropin_headline():
    from mfgp_coverage_amd.gaussian_process import MFGP
    from mfgp_coverage_amd.synthetic import HYP
    hyp = HYP["australia8_mf"]
    w = _workload(21)
    gp = MFGP(w.XL, w.yL.reshape(-1, 1), np.empty((0, 2)), np.empty((0, 1)), 1, 1)
    gp.hyp = hyp
    gp.updt_info(gp.X_L, gp.y_L, gp.X_H, gp.y_H)
    gp.predict(w.xs)
    for s in range(1, STEPS + 1):
        gp.updt_hifi(w.Xnew[s - 1], w.ynew[s - 1].reshape(-1, 1))
        mu, cov = gp.predict(w.xs)
        if s in CHECK:
            mu_r, var_r = O.mf_diag(w.XL, w.yL, gp.X_H, gp.y_H, hyp, w.xs)
            e = O.parity_errors(mu[:, 0], np.diag(cov), mu_r, var_r, O.prior_variance(hyp))
            assert max(e) < O.PARITY_TOL, (s, e)
    st = gp._dev().stats()
    assert gp.X_H.shape[0] == STEPS * K
    assert st["full_factor"] == 1 and st["inc_factor"] == STEPS and st["full_predict"] == 1, st


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_long_horizon_batched_growth(dtype):
    import torch
    from mfgp_coverage_amd import _lib
    from mfgp_coverage_amd.synthetic import HYP
    hyp = HYP["australia8_mf"] if dtype == "f64" else HYP["australia9_mf"]
    B = 4
    wls = [_workload(30 + i) for i in range(B)]
    M = wls[0].xs.shape[0]
    dt = _lib.F32 if dtype == "f32" else _lib.F64
    models = []
    for w in wls:
        m = _lib.Model(_lib.context(), _lib.MF, hyp, 1e-8, dtype=dt)
        m.set_grid(w.xs)
        m.set_data(w.XL, w.yL, np.empty((0, 2)), np.empty(0))
        models.append(m)
    mu = torch.empty(B * M, dtype=torch.float64, device="cuda")
    var = torch.empty(B * M, dtype=torch.float64, device="cuda")
    _lib.batch_predict(models, mu.data_ptr(), var.data_ptr())
    X = torch.from_numpy(np.ascontiguousarray(np.stack([w.Xnew for w in wls], 1))).cuda()   # [S, B, K, 2]
    Y = torch.from_numpy(np.ascontiguousarray(np.stack([w.ynew for w in wls], 1))).cuda()
    for s in range(1, STEPS + 1):
        _lib.batch_append_predict(models, X[s - 1].data_ptr(), Y[s - 1].data_ptr(), [K] * B, mu.data_ptr(),
                                  var.data_ptr(), asynchronous=True)
        if s in (75, STEPS):
            _lib.context().synchronize()
            mu_h, var_h = mu.cpu().numpy().reshape(B, M), var.cpu().numpy().reshape(B, M)
            for i in ((0,) if s == 75 else range(B)):
                w = wls[i]
                XH, yH = w.Xnew[:s].reshape(-1, 2), w.ynew[:s].reshape(-1)
                mu_r, var_r = O.mf_diag(w.XL, w.yL, XH, yH, hyp, w.xs)
                if dtype == "f64":
                    e = O.parity_errors(mu_h[i], var_h[i], mu_r, var_r, O.prior_variance(hyp))
                    assert max(e) < O.PARITY_TOL, (s, i, e)
                else:
                    e = O.parity_errors_f32(mu_h[i], var_h[i], mu_r, var_r, O.prior_variance(hyp))
                    assert max(e) < O.F32_TOL, (s, i, e)
    for m in models:
        st = m.stats()
        assert st["full_factor"] == 1 and st["inc_factor"] == STEPS and st["full_predict"] == 1, st
        # a lattice grid and kss / noise <= 1e4: the separable step wherever the host's
        # cost model prefers it to the V stream -- every step at fp64; at fp32 (half
        # the V bytes) the V stream may win while the factor is small
        if dtype == "f64":
            assert st["lattice"] == STEPS, st
        else:
            assert STEPS // 2 < st["lattice"] <= STEPS and st["lattice"] + st["vstream"] >= STEPS, st
