"""The full factor in one launch per 64-column step (k_fstep: panel, look-ahead
diagonal block, trailing update handed over inside the launch) against the
three-launch form (k_potrf_diag / k_panel / k_syrk) and the oracle.

Both forms run the same tile products in the same order, so the factor, the
mean and the variance must agree bit for bit; ragged batches cover GPs that
run out of blocks at different steps (their roles exit early) and sizes on
either side of the 64-row blocks. Reference: np.linalg.cholesky, gp:254 /
gp:529 (MF K blocks gp:523-529)."""
import numpy as np
import pytest
import torch

from oracle import gp_oracle as O
from mfgp_coverage_amd import _lib, synthetic

pytestmark = pytest.mark.gpu

HYP = synthetic.HYP["australia8_mf"]


def _models(ctx, specs, G):
    out = []
    for i, (NL, NH) in enumerate(specs):
        wl = synthetic.Workload(G, NL, NH, 1, 1, seed=100 + i)
        m = _lib.Model(ctx, _lib.MF, HYP, 1e-8)
        m.set_grid(wl.xs)
        m.set_data(wl.XL, wl.yL, wl.XH, wl.yH)
        out.append((m, wl))
    return out


def _run(fused, specs, G):
    ctx = _lib.Context(0)
    ctx.set_incremental(False)
    ctx.set_fused_factor(fused)
    ms = _models(ctx, specs, G)
    M = G * G
    mu = torch.empty(len(ms) * M, dtype=torch.float64, device="cuda:0")
    var = torch.empty_like(mu)
    _lib.batch_predict([m for m, _ in ms], mu.data_ptr(), var.data_ptr())
    ctx.synchronize()
    Ls = [m.factor() for m, _ in ms]
    stats = [m.stats() for m, _ in ms]
    return Ls, mu.cpu().numpy().reshape(len(ms), M), var.cpu().numpy().reshape(len(ms), M), [w for _, w in ms], stats


@pytest.mark.parametrize("specs", [
    [(64, 66), (0, 1), (300, 400), (1024, 1023), (63, 0)],   # ragged: 2 .. 33 blocks, N = 1 .. 2047
    [(1024, 1024)] * 4,                                       # the headline N = 2048, 4 GPs
])
def test_fused_factor_equals_three_launch(specs):
    G = 128
    L1, mu1, var1, wls, st = _run(True, specs, G)
    L3, mu3, var3, _, _ = _run(False, specs, G)
    for a, b in zip(L1, L3):
        assert np.array_equal(a, b)
    assert np.array_equal(mu1, mu3) and np.array_equal(var1, var3)
    assert all(s["full_factor"] >= 1 for s in st)
    # and against the oracle (numpy Cholesky of the reference's K) on every 7th cell
    for i, wl in enumerate(wls):
        X = np.vstack([wl.XL, wl.XH]) if wl.XL.size else wl.XH
        if X.shape[0] == 0:
            continue
        cells = np.arange(0, wl.xs.shape[0], 7)
        mu_r, var_r = O.mf_diag(wl.XL, wl.yL.reshape(-1, 1), wl.XH, wl.yH.reshape(-1, 1), HYP, wl.xs[cells])
        e_mu, e_var = O.parity_errors(mu1[i, cells], var1[i, cells], mu_r, var_r, O.prior_variance(HYP))
        assert e_mu < O.PARITY_TOL and e_var < O.PARITY_TOL, (i, e_mu, e_var)
