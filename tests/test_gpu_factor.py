"""The full-path factor and the lattice step's explicit inverse (round 3).

- Two-level blocked Cholesky (mfgp_capi.hip enqueue_factor, k_syrk_blk): the
  trailing matrix takes a group of 64-column steps in one pass. The MFMA
  sequence per tile is the one-level factor's, so L, mu and var must be
  bit-equal to MFGP_FACTOR_DEPTH=1 for every group depth, on a ragged batch.
- F = L^-1 by recursive doubling (mfgp_nlml.hip k_trinv_diag / k_trinv_lvl)
  against the block-column k_trinv_f (MFGP_TRINV_COLUMNS=1): a different
  operation order, so the lattice step's posteriors agree to rounding, and both
  meet the oracle (gp:401-438) at every cell; ragged block counts (partial
  second halves at every level).
"""
import numpy as np
import pytest

from oracle import gp_oracle as O

pytestmark = pytest.mark.gpu

TOL = O.PARITY_TOL


def _grid(G):
    g = np.linspace(0.0, 1.0, G)
    return np.array([(a, b) for a in g for b in g])


def _data(G, n, seed):
    rng = np.random.default_rng(seed)
    Xs = _grid(G)
    X = Xs[rng.choice(Xs.shape[0], n, replace=False)].copy()
    y = np.sin(4 * X[:, 0]) * np.cos(3 * X[:, 1]) + 0.1 * rng.standard_normal(n)
    return Xs, X, y


def _mf(ctx, hyp, X, y, NL, Xs):
    from mfgp_coverage_amd import _lib
    m = _lib.Model(ctx, _lib.MF, hyp, 1e-8)
    m.set_grid(Xs)
    m.set_data(X[:NL], y[:NL], X[NL:], y[NL:])
    return m


@pytest.mark.parametrize("depth", [2, 3, 4, 8])
def test_two_level_factor_bit_equal(monkeypatch, depth):
    from mfgp_coverage_amd import _lib
    from mfgp_coverage_amd.synthetic import HYP
    hyp = HYP["australia8_mf"].copy()
    monkeypatch.setenv("MFGP_FACTOR_DEPTH", "1")
    c1 = _lib.Context(0)
    monkeypatch.setenv("MFGP_FACTOR_DEPTH", str(depth))
    cd = _lib.Context(0)
    for c in (c1, cd):
        c.set_incremental(False)
    sizes = [(48, 300, 120), (64, 1000, 400), (64, 2047, 1024)]
    res = []
    for ctx in (c1, cd):
        ms = []
        for i, (G, n, NL) in enumerate(sizes):
            Xs, X, y = _data(G, n, seed=11 + i)
            ms.append((_mf(ctx, hyp, X, y, NL, Xs), Xs.shape[0]))
        # one ragged batch (every GP's factor in the same launches)
        M = sum(mm for _, mm in ms)
        import torch
        mu = torch.empty(M, dtype=torch.float64, device="cuda")
        var = torch.empty(M, dtype=torch.float64, device="cuda")
        _lib.batch_predict([m for m, _ in ms], mu.data_ptr(), var.data_ptr())
        ctx.synchronize()
        res.append(([m.factor() for m, _ in ms], mu.cpu().numpy(), var.cpu().numpy()))
    for L1, Ld in zip(res[0][0], res[1][0]):
        assert np.array_equal(L1, Ld), depth
    assert np.array_equal(res[0][1], res[1][1]) and np.array_equal(res[0][2], res[1][2]), depth


@pytest.mark.parametrize("n0", [300, 571, 1100])
def test_trinv_recursive_vs_columns_and_oracle(monkeypatch, n0):
    from mfgp_coverage_amd import _lib
    from mfgp_coverage_amd.synthetic import HYP
    hyp = HYP["australia8_mf"].copy()
    G, NL = 64, n0 // 3
    ctxs = []
    for cols in ("1", "0"):
        monkeypatch.setenv("MFGP_TRINV_COLUMNS", cols)
        c = _lib.Context(0)
        c.set_lattice("force")
        ctxs.append(c)
    Xs, X, y = _data(G, n0 + 16, seed=n0)
    ms = [_mf(c, hyp, X[:n0], y[:n0], NL, Xs) for c in ctxs]
    for m in ms:
        m.predict()
    n = n0
    for k in (8, 8):
        outs = []
        for m in ms:
            m.append(X[n:n + k], y[n:n + k])
            outs.append(m.predict())
        n += k
        mu_r, var_r = O.mf_diag(X[:NL], y[:NL], X[NL:n], y[NL:n], hyp, Xs)
        for mu, var in outs:
            assert max(O.parity_errors(mu, var, mu_r, var_r, O.prior_variance(hyp))) < TOL, (n0, n)
        (mu_c, var_c), (mu_d, var_d) = outs
        assert max(O.parity_errors(mu_d, var_d, mu_c, var_c, O.prior_variance(hyp))) < 1e-9, (n0, n)
    for m in ms:
        assert m.stats()["lattice"] == 2, m.stats()
