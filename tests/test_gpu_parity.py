"""Parity of the HIP path (libmfgp_hip.so through the SFGP/MFGP mirror and the
batched C ABI) against the reference's golden vectors, its logged runs and the
CPU oracle. Tolerance (oracle.gp_oracle.PARITY_TOL, BASELINE.json north_star):
mu rel <= 1e-6; var |d| <= 1e-6 * max(|ref|, 1e-6 * k**).
"""
import copy

import numpy as np
import pytest

from oracle import gp_oracle as O
from tests import _fixtures as F

pytestmark = pytest.mark.gpu

TOL = O.PARITY_TOL


@pytest.fixture(scope="module")
def gp():
    from mfgp_coverage_amd import gaussian_process as G
    return G


@pytest.fixture(scope="module")
def atc():
    return F.atc()


def _check(mu, cov, mu_ref, var_ref, hyp, tol=TOL):
    var = np.diag(cov)
    assert mu.shape == (mu_ref.shape[0], 1)
    e_mu, e_var = O.parity_errors(mu[:, 0], var, mu_ref, var_ref, O.prior_variance(hyp))
    assert e_mu < tol and e_var < tol, (e_mu, e_var)
    return e_mu, e_var


@pytest.mark.parametrize("grid", F.GRIDS)
@pytest.mark.parametrize("N", F.NS)
def test_sf_vs_reference_golden(gp, atc, grid, N):
    X, y = atc["train"][:N, :2].copy(), atc["train"][:N, 2:3].copy()
    m = gp.SFGP(X, y, 1)
    m.hyp = atc["hyp_sf"].copy()
    if N > 0:
        m.updt_info(m.X, m.y)
    mu, cov = m.predict(atc[f"grid_{grid}"])
    key = f"sf_{grid}_n{N}"
    _check(mu, cov, atc[key + "_mu"], atc[key + "_var"], atc["hyp_sf"])
    np.testing.assert_allclose(np.amax(cov), atc[key + "_amax"], rtol=TOL)


@pytest.mark.parametrize("grid", F.GRIDS)
@pytest.mark.parametrize("N", F.NS)
def test_mf_vs_reference_golden(gp, atc, grid, N):
    P = atc["prior"]
    X, y = atc["train"][:N, :2].copy(), atc["train"][:N, 2:3].copy()
    m = gp.MFGP(P[:, :2].copy(), P[:, 2:3].copy(), X, y, 1, 1)
    m.hyp = atc["hyp_mf"].copy()
    m.updt_info(m.X_L, m.y_L, m.X_H, m.y_H)
    mu, cov = m.predict(atc[f"grid_{grid}"])
    key = f"mf_{grid}_n{N}"
    _check(mu, cov, atc[key + "_mu"], atc[key + "_var"], atc["hyp_mf"])


@pytest.mark.parametrize("grid", F.GRIDS)
def test_empty_gp_exact(gp, atc, grid):
    e2, e1 = np.empty((0, 2)), np.empty((0, 1))
    sf = gp.SFGP(e2, e1, 1)
    sf.hyp = atc["hyp_sf"].copy()
    mu, cov = sf.predict(atc[f"grid_{grid}"])          # simulator.py:841-842 (no updt_info)
    assert np.all(mu == O.prior_mean(atc["hyp_sf"])) and np.all(np.diag(cov) == O.prior_variance(atc["hyp_sf"]))
    np.testing.assert_allclose(np.amax(cov), atc[f"sf_{grid}_n0_amax"], rtol=1e-15)
    mf = gp.MFGP(e2, e1, e2, e1, 1, 1)
    mf.hyp = atc["hyp_mf"].copy()
    mu, cov = mf.predict(atc[f"grid_{grid}"])
    np.testing.assert_allclose(mu[:, 0], atc[f"mfempty_{grid}_mu"], rtol=1e-15)
    np.testing.assert_allclose(np.diag(cov), atc[f"mfempty_{grid}_var"], rtol=1e-15)
    np.testing.assert_allclose(np.amax(cov), atc[f"mfempty_{grid}_amax"], rtol=1e-15)


def test_append_sequences_vs_reference(gp, atc):
    P, T = atc["prior"], atc["train"]
    sf = gp.SFGP(P[:, :2].copy(), P[:, 2:3].copy(), 1)
    sf.hyp = atc["hyp_sf"].copy()
    sf.updt_info(sf.X, sf.y)
    e2, e1 = np.empty((0, 2)), np.empty((0, 1))
    mf = gp.MFGP(P[:, :2].copy(), P[:, 2:3].copy(), e2, e1, 1, 1)
    mf.hyp = atc["hyp_mf"].copy()
    mf.updt_info(mf.X_L, mf.y_L, mf.X_H, mf.y_H)
    pos = 0
    for s, k in enumerate(atc["seq_chunks"]):
        xa, ya = T[pos:pos + k, :2].copy(), T[pos:pos + k, 2:3].copy()
        pos += int(k)
        sf.updt(xa, ya)                 # k = 0 is the empty append of simulator.py:719
        mf.updt_hifi(xa, ya)
        assert sf.X.shape[0] == 9 + pos and mf.X_H.shape[0] == pos
        mu, cov = sf.predict(atc["grid_g51"])
        _check(mu, cov, atc[f"sfseq_s{s}_mu"], atc[f"sfseq_s{s}_var"], atc["hyp_sf"])
        mu, cov = mf.predict(atc["grid_g51"])
        _check(mu, cov, atc[f"mfseq_s{s}_mu"], atc[f"mfseq_s{s}_var"], atc["hyp_mf"])


def _replay_model(gp, hyp, prior):
    e2, e1 = np.empty((0, 2)), np.empty((0, 1))
    if hyp.shape[0] == 4:
        X, y = (prior[:, :2].copy(), prior[:, 2:3].copy()) if prior is not None else (e2, e1)
        m = gp.SFGP(X, y, 1)
        m.hyp = hyp.copy()
        m.updt_info(m.X, m.y)
    else:
        XL, yL = (prior[:, :2].copy(), prior[:, 2:3].copy()) if prior is not None else (e2, e1)
        m = gp.MFGP(XL, yL, e2, e1, 1, 1)
        m.hyp = hyp.copy()
        m.updt_info(m.X_L, m.y_L, m.X_H, m.y_H)
    return m


def _replay_append(gp, m, X, y):
    if isinstance(m, gp.SFGP):
        m.updt(X, y)
    elif isinstance(m, gp.MFGP):
        m.updt_hifi(X, y)
    else:
        raise TypeError("Invalid model type: must be SFGP or MFGP")


@pytest.mark.parametrize("run", F.REPLAY_RUNS)
def test_replay_logged_runs(gp, run):
    """Replays Data/<run>_sample.csv and checks the logged per-iteration max VarMax."""
    fx = F.replay(run)
    for sim in fx["sims"]:
        logged, got = F.replay_run(
            fx, sim,
            make_model=lambda hyp, prior: _replay_model(gp, hyp, prior),
            append=lambda m, X, y: _replay_append(gp, m, X, y),
            predict_var=lambda m: np.diag(m.predict(fx["grid"])[1]))
        np.testing.assert_allclose(got, logged, rtol=TOL)


def test_not_positive_definite_raises(gp, atc):
    X, y = atc["train"][:20, :2].copy(), atc["train"][:20, 2:3].copy()
    m = gp.SFGP(X, y, 1)
    m.hyp = atc["hyp_sf"].copy()
    m.jitter = -1.0                        # K + jitter*I indefinite: np.linalg.cholesky raises
    with pytest.raises(np.linalg.LinAlgError):
        m.updt_info(m.X, m.y)
    m.jitter = 1e-8
    m.updt_info(m.X, m.y)                  # recovers
    mu, cov = m.predict(atc["grid_g32"])
    mu_r, var_r = O.sf_diag(X, y, atc["hyp_sf"], atc["grid_g32"])
    _check(mu, cov, mu_r, var_r, atc["hyp_sf"])


def test_deepcopy_is_independent(gp, atc):
    """copy.deepcopy as used by compute_sample_points (simulator.py:339-364)."""
    P, T = atc["prior"], atc["train"]
    e2, e1 = np.empty((0, 2)), np.empty((0, 1))
    mf = gp.MFGP(P[:, :2].copy(), P[:, 2:3].copy(), T[:30, :2].copy(), T[:30, 2:3].copy(), 1, 1)
    mf.hyp = atc["hyp_mf"].copy()
    mf.updt_info(mf.X_L, mf.y_L, mf.X_H, mf.y_H)
    grid = atc["grid_g51"]
    mu0, cov0 = mf.predict(grid)
    tmp = copy.deepcopy(mf)
    assert isinstance(tmp, gp.MFGP) and not isinstance(tmp, gp.SFGP)
    for i in range(3):
        v = np.diag(tmp.predict(grid)[1])
        j = int(np.argmax(v))
        tmp.updt_hifi(grid[j:j + 1], mu0[j:j + 1])
    assert tmp.X_H.shape[0] == 33 and mf.X_H.shape[0] == 30
    mu1, cov1 = mf.predict(grid)
    np.testing.assert_array_equal(mu1, mu0)
    np.testing.assert_array_equal(np.diag(cov1), np.diag(cov0))
    mu2, cov2 = tmp.predict(grid)
    XH = np.vstack([T[:30, :2]] + [tmp.X_H[30 + i:31 + i] for i in range(3)])
    mu_r, var_r = O.mf_diag(P[:, :2], P[:, 2], XH, tmp.y_H[:, 0], atc["hyp_mf"], grid)
    _check(mu2, cov2, mu_r, var_r, atc["hyp_mf"])
    del e2, e1


def test_factor_matches_numpy(gp, atc):
    X, y = atc["train"][:100, :2].copy(), atc["train"][:100, 2:3].copy()
    m = gp.SFGP(X, y, 1)
    m.hyp = atc["hyp_sf"].copy()
    m.updt_info(m.X, m.y)
    L = m.L
    h = atc["hyp_sf"]
    K = O.se_kernel(X, X, h[1], h[2]) + np.eye(100) * np.exp(h[3]) + np.eye(100) * O.JITTER
    np.testing.assert_allclose(L, np.linalg.cholesky(K), rtol=1e-6, atol=1e-9)


def _synthetic(G, N, seed, mf_NL=0):
    rng = np.random.default_rng(seed)
    g = np.linspace(0.0, 1.0, G)
    Xs = np.array([(a, b) for a in g for b in g])
    idx = rng.choice(Xs.shape[0], N, replace=False)
    X = Xs[idx]
    c = rng.random((3, 2))
    f = sum(np.exp(-np.sum((X - ci) ** 2, 1) / 0.05) for ci in c)
    y = (f / f.max() + 0.1 * rng.standard_normal(N)).reshape(-1, 1)
    return Xs, X, y


@pytest.mark.parametrize("kind,G,N,NL", [("sf", 64, 1000, 0), ("mf", 64, 1000, 300), ("mf", 48, 577, 577),
                                          ("sf", 40, 127, 0), ("sf", 40, 128, 0), ("mf", 40, 129, 64)])
def test_larger_vs_oracle(gp, kind, G, N, NL):
    """Ragged and block-boundary sizes (N = 127/128/129 around the 64-row blocks)."""
    Xs, X, y = _synthetic(G, N, seed=G + N)
    if kind == "sf":
        hyp = np.array([0.001, -2.368468757, -1.353149618, -4.596652374])   # australia3_sf_hyp.csv
        m = gp.SFGP(X, y, 1)
        m.hyp = hyp
        m.updt_info(m.X, m.y)
        mu_r, var_r = O.sf_diag(X, y, hyp, Xs)
    else:
        hyp = np.array([-1.700903132, -1.947362545, -0.309197345, -14.9598621, -3.655273338,
                        -1.317607182, -0.721748367, -5.926942955, -1.371689752])  # australia8_mf_hyp.csv
        m = gp.MFGP(X[:NL], y[:NL], X[NL:], y[NL:], 1, 1)
        m.hyp = hyp
        m.updt_info(m.X_L, m.y_L, m.X_H, m.y_H)
        mu_r, var_r = O.mf_diag(X[:NL], y[:NL], X[NL:], y[NL:], hyp, Xs)
    mu, cov = m.predict(Xs)
    _check(mu, cov, mu_r, var_r, hyp)


@pytest.mark.parametrize("src", ["host", "device"])
def test_batched_ragged_vs_single(gp, src):
    """mfgp_batch_append_predict over GPs of different N and M equals per-model results
    (new rows from host memory -> copies; from device memory -> the k_append kernel)."""
    import ctypes

    from mfgp_coverage_amd import _lib
    hyp = np.array([-1.700903132, -1.947362545, -0.309197345, -14.9598621, -3.655273338,
                    -1.317607182, -0.721748367, -5.926942955, -1.371689752])
    ctx = _lib.context()
    cases = [(32, 70, 20, 5), (40, 200, 64, 8), (24, 0, 0, 3), (33, 130, 9, 0)]
    models, news, refs, Ms = [], [], [], []
    for (G, N, NL, k) in cases:
        Xs, X, y = _synthetic(G, N + k, seed=N + G)
        mdl = _lib.Model(ctx, _lib.MF, hyp, 1e-8)
        mdl.set_grid(Xs)
        mdl.set_data(X[:NL], y[:NL, 0], X[NL:N], y[NL:N, 0])
        models.append(mdl)
        news.append((X[N:N + k], y[N:N + k, 0]))
        refs.append(O.mf_diag(X[:NL], y[:NL], X[NL:N + k], y[NL:N + k], hyp, Xs))
        Ms.append(Xs.shape[0])
    Xn = np.ascontiguousarray(np.vstack([a for a, _ in news]))
    yn = np.ascontiguousarray(np.concatenate([b for _, b in news]))
    tot = sum(Ms)
    import torch
    mu_d = torch.empty(tot, dtype=torch.float64, device="cuda")
    var_d = torch.empty(tot, dtype=torch.float64, device="cuda")
    if src == "host":
        xp, yp = Xn.ctypes.data, yn.ctypes.data
    else:
        Xd, yd = torch.from_numpy(Xn).cuda(), torch.from_numpy(yn).cuda()
        xp, yp = Xd.data_ptr(), yd.data_ptr()
    _lib.batch_append_predict(models, xp, yp, [c[3] for c in cases], mu_d.data_ptr(), var_d.data_ptr())
    mu, var = mu_d.cpu().numpy(), var_d.cpu().numpy()
    off = 0
    for (mu_r, var_r), M in zip(refs, Ms):
        e = O.parity_errors(mu[off:off + M], var[off:off + M], mu_r, var_r, O.prior_variance(hyp))
        assert max(e) < TOL, e
        off += M
    del ctypes


def test_headline_size_vs_oracle(gp):
    """Full headline size (128x128 grid, N = 1024 lofi + 1024 hifi, australia8 MF hyp) against
    the diag oracle: every cell, same tolerance."""
    Xs, X, y = _synthetic(128, 2048, seed=7)
    hyp = np.array([-1.700903132, -1.947362545, -0.309197345, -14.9598621, -3.655273338,
                    -1.317607182, -0.721748367, -5.926942955, -1.371689752])
    m = gp.MFGP(X[:1024], y[:1024], X[1024:2040], y[1024:2040], 1, 1)
    m.hyp = hyp
    m.updt_info(m.X_L, m.y_L, m.X_H, m.y_H)
    m.updt_hifi(X[2040:], y[2040:])
    mu, cov = m.predict(Xs)
    mu_r, var_r = O.mf_diag(X[:1024], y[:1024], X[1024:], y[1024:], hyp, Xs)
    _check(mu, cov, mu_r, var_r, hyp)
    var = np.diag(cov)
    assert np.all(var > -1e-12) and np.all(var <= O.prior_variance(hyp) * (1 + 1e-12))


def test_configs4_size_vs_oracle(gp):
    """BASELINE configs[4] sizes for one GP: 256x256 grid (M = 65536), N = 4096 lofi + 4096 hifi,
    australia9 MF hyp, at fp64 (the fp32 mode of configs[4] is tests/test_gpu_f32.py). The full
    factor + predict, then an 8-row bordered append (the incremental path), each against the
    diag oracle on 4096 sampled cells plus the new samples' cells and the device's argmax
    cell, at the parity tolerance."""
    from mfgp_coverage_amd.synthetic import HYP, Workload
    hyp = HYP["australia9_mf"]
    w = Workload(256, 4096, 4088, 8, 1, seed=11)
    m = gp.MFGP(w.XL, w.yL.reshape(-1, 1), w.XH, w.yH.reshape(-1, 1), 1, 1)
    m.hyp = hyp
    m.updt_info(m.X_L, m.y_L, m.X_H, m.y_H)
    M = w.xs.shape[0]
    rng = np.random.default_rng(5)
    Xn, yn = w.Xnew[0], w.ynew[0].reshape(-1, 1)
    new_cells = np.array([int(np.argmin(np.abs(w.xs - p).sum(1))) for p in Xn])
    for step in range(2):
        mu, cov = m.predict(w.xs)
        var = np.diag(cov)
        XH = m.X_H
        pick = np.unique(np.concatenate([rng.choice(M, 4096, replace=False), new_cells,
                                         [int(np.argmax(var))]]))
        mu_r, var_r = O.mf_diag(w.XL, w.yL, XH, m.y_H, hyp, w.xs[pick])
        e = O.parity_errors(mu[pick, 0], var[pick], mu_r, var_r, O.prior_variance(hyp))
        assert max(e) < TOL, (step, e)
        if step == 0:
            m.updt_hifi(Xn, yn)
    st = m._dev().stats()
    assert st["inc_factor"] >= 1 and st["vstream"] >= 1, st
