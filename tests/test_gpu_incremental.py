"""Incremental updates: bordered-Cholesky appends (k_inc_factor) and one-pass
predicts over the resident V (k_vstream), against the CPU oracle and against the
full-recompute path of the same library (mfgp_ctx_set_incremental(0)).

The reference refactors from scratch on every updt / updt_hifi (gp:257-268,
gp:531-542) and recomputes psi K^-1 psi^T in every predict (gp:121-148,
gp:401-438); the incremental path must give the same numbers to the parity
tolerance (oracle.gp_oracle.PARITY_TOL) on every step, on both of its L21
sources (new points on the grid -> V columns; off the grid -> solved), across
64-row block boundaries, from an empty GP, after truncation, clones, grid and
hyperparameter changes.
"""
import copy

import numpy as np
import pytest

from oracle import gp_oracle as O

pytestmark = pytest.mark.gpu

TOL = O.PARITY_TOL
HYP_SF = np.array([0.001, -2.368468757, -1.353149618, -4.596652374])        # australia3_sf_hyp.csv
HYP_MF = np.array([-1.700903132, -1.947362545, -0.309197345, -14.9598621, -3.655273338,
                   -1.317607182, -0.721748367, -5.926942955, -1.371689752])  # australia8_mf_hyp.csv


def _grid(G):
    g = np.linspace(0.0, 1.0, G)
    return np.array([(a, b) for a in g for b in g])


def _field(X, rng):
    c = rng.random((3, 2))
    f = sum(np.exp(-np.sum((X - ci) ** 2, 1) / 0.05) for ci in c)
    return f / f.max() + 0.1 * rng.standard_normal(X.shape[0])


def _points(G, n, seed, ongrid):
    """n distinct sample points: grid cells, or grid cells shifted off the grid."""
    rng = np.random.default_rng(seed)
    Xs = _grid(G)
    X = Xs[rng.choice(Xs.shape[0], n, replace=False)].copy()
    if not ongrid:
        X += 0.37 / (G - 1)
    y = _field(X, rng)
    return Xs, X, y


def _ref(kind, X, y, NL, Xs, hyp):
    if kind == "sf":
        return O.sf_diag(X, y, hyp, Xs)
    return O.mf_diag(X[:NL], y[:NL], X[NL:], y[NL:], hyp, Xs)


def _model(ctx, kind, X, y, NL, Xs):
    from mfgp_coverage_amd import _lib
    hyp = HYP_SF if kind == "sf" else HYP_MF
    m = _lib.Model(ctx, _lib.SF if kind == "sf" else _lib.MF, hyp, 1e-8)
    m.set_grid(Xs)
    if kind == "sf":
        m.set_data(np.empty((0, 2)), np.empty(0), X, y)
    else:
        m.set_data(X[:NL], y[:NL], X[NL:], y[NL:])
    return m, hyp


def _err(mu, var, mu_r, var_r, hyp):
    return max(O.parity_errors(mu, var, mu_r, var_r, O.prior_variance(hyp)))


@pytest.fixture(scope="module")
def full_ctx():
    from mfgp_coverage_amd import _lib
    c = _lib.Context(0)
    c.set_incremental(False)
    return c


STEPS = [8, 1, 16, 5, 0, 12, 3, 16, 16]   # crosses 64-row blocks from N0 = 250


@pytest.mark.parametrize("kind", ["sf", "mf"])
@pytest.mark.parametrize("ongrid", [True, False])
def test_incremental_sequence_vs_oracle(kind, ongrid, full_ctx):
    from mfgp_coverage_amd import _lib
    N0, NL = 250, (0 if kind == "sf" else 100)
    Xs, X, y = _points(48, N0 + sum(STEPS), seed=11 + ongrid, ongrid=ongrid)
    m, hyp = _model(_lib.context(), kind, X[:N0], y[:N0], NL, Xs)
    f, _ = _model(full_ctx, kind, X[:N0], y[:N0], NL, Xs)
    m.predict()
    n = N0
    for k in STEPS:
        m.append(X[n:n + k], y[n:n + k])
        f.append(X[n:n + k], y[n:n + k])
        n += k
        mu, var = m.predict()
        mu_r, var_r = _ref(kind, X[:n], y[:n], NL, Xs, hyp)
        assert _err(mu, var, mu_r, var_r, hyp) < TOL
        mu_f, var_f = f.predict()
        assert _err(mu, var, mu_f, var_f, hyp) < 1e-8       # incremental == full to rounding
    st = m.stats()
    assert st["full_factor"] == 1 and st["inc_factor"] == sum(1 for k in STEPS if k > 0)
    assert st["full_predict"] == 1 and st["vstream"] == len(STEPS)
    assert st["factor_rows"] == n and st["v_rows"] == n
    sf_ = f.stats()
    assert sf_["inc_factor"] == 0 and sf_["vstream"] == 0
    # the factor itself: rows appended by bordering equal a fresh Cholesky
    L = m.factor()
    np.testing.assert_allclose(L, f.factor(), rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("kind", ["sf", "mf"])
def test_empty_gp_grows_incrementally(gp_mod, kind):
    """updt from an empty GP (simulator.py:671/719): every step is a bordered append,
    the first predicts stream an empty V (n0 = 0)."""
    Xs, X, y = _points(32, 90, seed=5, ongrid=True)
    e2, e1 = np.empty((0, 2)), np.empty((0, 1))
    if kind == "sf":
        m = gp_mod.SFGP(e2, e1, 1)
        m.hyp = HYP_SF.copy()
        hyp = HYP_SF
    else:
        m = gp_mod.MFGP(e2, e1, e2, e1, 1, 1)
        m.hyp = HYP_MF.copy()
        hyp = HYP_MF
    m.predict(Xs)
    n = 0
    for k in [5, 11, 16, 16, 16, 16, 10]:
        a, b = X[n:n + k], y[n:n + k].reshape(-1, 1)
        (m.updt if kind == "sf" else m.updt_hifi)(a, b)
        n += k
        mu, cov = m.predict(Xs)
        mu_r, var_r = _ref(kind, X[:n], y[:n], 0, Xs, hyp)
        assert _err(mu[:, 0], np.diag(cov), mu_r, var_r, hyp) < TOL
    st = m._dev().stats()
    assert st["inc_factor"] == 7 and st["vstream"] == 8 and st["full_predict"] == 0


@pytest.fixture(scope="module")
def gp_mod():
    from mfgp_coverage_amd import gaussian_process as G
    return G


def test_truncate_and_reappend_vs_oracle():
    """The benchmark's step: drop the last k hifi rows, append k new ones, predict."""
    from mfgp_coverage_amd import _lib
    Xs, X, y = _points(40, 700, seed=3, ongrid=True)
    NL, NH0, k = 300, 380, 8
    m, hyp = _model(_lib.context(), "mf", X[:NL + NH0], y[:NL + NH0], NL, Xs)
    m.predict()
    for s in range(3):
        m.truncate(NH0)
        lo = NL + NH0 + s * k
        m.append(X[lo:lo + k], y[lo:lo + k])
        mu, var = m.predict()
        Xr = np.vstack([X[:NL + NH0], X[lo:lo + k]])
        yr = np.concatenate([y[:NL + NH0], y[lo:lo + k]])
        mu_r, var_r = _ref("mf", Xr, yr, NL, Xs, hyp)
        assert _err(mu, var, mu_r, var_r, hyp) < TOL
    st = m.stats()
    assert st["inc_factor"] == 3 and st["vstream"] == 3


def test_clone_keeps_resident_state(gp_mod):
    """compute_sample_points (simulator.py:339-364): deepcopy, then 1-point appends on the copy."""
    Xs, X, y = _points(40, 400, seed=9, ongrid=True)
    m = gp_mod.MFGP(X[:200], y[:200, None], X[200:380], y[200:380, None], 1, 1)
    m.hyp = HYP_MF.copy()
    m.updt_info(m.X_L, m.y_L, m.X_H, m.y_H)
    mu0, cov0 = m.predict(Xs)
    tmp = copy.deepcopy(m)
    for i in range(4):
        v = np.diag(tmp.predict(Xs)[1])
        j = int(np.argmax(v))
        tmp.updt_hifi(Xs[j:j + 1], mu0[j:j + 1])
    st = tmp._dev().stats()
    # each append follows a predict, so it runs the one-pass predict with it (the
    # speculative form of an eager append, kept for the next predict): 1 + 4 streams
    assert st["inc_factor"] == 4 and st["full_predict"] == 0 and st["vstream"] == 5
    mu1, cov1 = m.predict(Xs)
    np.testing.assert_array_equal(mu1, mu0)
    np.testing.assert_array_equal(np.diag(cov1), np.diag(cov0))
    mu2, cov2 = tmp.predict(Xs)
    mu_r, var_r = O.mf_diag(X[:200], y[:200], tmp.X_H, tmp.y_H[:, 0], HYP_MF, Xs)
    assert _err(mu2[:, 0], np.diag(cov2), mu_r, var_r, HYP_MF) < TOL


def test_grid_change_and_hyp_change():
    from mfgp_coverage_amd import _lib
    Xs, X, y = _points(32, 260, seed=21, ongrid=True)
    m, hyp = _model(_lib.context(), "sf", X[:240], y[:240], 0, Xs)
    m.predict()
    Xs2 = _grid(37)
    m.set_grid(Xs2)                        # V belongs to the old grid: full predict
    m.append(X[240:248], y[240:248])
    mu, var = m.predict()
    mu_r, var_r = _ref("sf", X[:248], y[:248], 0, Xs2, hyp)
    assert _err(mu, var, mu_r, var_r, hyp) < TOL
    st = m.stats()
    assert st["full_predict"] == 2 and st["inc_factor"] == 1
    hyp2 = hyp + np.array([0.0, 0.1, -0.05, 0.2])
    m.set_hyp(hyp2, 1e-8)                  # new hyperparameters: full refactor, full predict
    m.append(X[248:256], y[248:256])
    mu, var = m.predict()
    mu_r, var_r = _ref("sf", X[:256], y[:256], 0, Xs2, hyp2)
    assert _err(mu, var, mu_r, var_r, hyp2) < TOL
    st = m.stats()
    assert st["full_factor"] == 2 and st["full_predict"] == 3


def test_more_than_kinc_rows_falls_back():
    from mfgp_coverage_amd import _lib
    Xs, X, y = _points(32, 300, seed=4, ongrid=True)
    m, hyp = _model(_lib.context(), "sf", X[:250], y[:250], 0, Xs)
    m.predict()
    m.append(X[250:267], y[250:267])      # 17 rows > KINC: full refactor + full predict
    mu, var = m.predict()
    mu_r, var_r = _ref("sf", X[:267], y[:267], 0, Xs, hyp)
    assert _err(mu, var, mu_r, var_r, hyp) < TOL
    st = m.stats()
    assert st["full_factor"] == 2 and st["inc_factor"] == 0 and st["full_predict"] == 2


def test_incremental_not_pd_raises():
    """A bordered append whose Schur complement is not positive raises LinAlgError,
    as np.linalg.cholesky of the full matrix does (gp:529)."""
    from mfgp_coverage_amd import _lib
    Xs, X, y = _points(24, 30, seed=2, ongrid=True)
    hyp = np.array([0.0, 0.0, -1.0, 0.0, -3.0, -1.0, -1.0, 2.0, -20.0])   # noise_L e^2, noise_H e^-20
    m = _lib.Model(_lib.context(), _lib.MF, hyp, -1.0)                      # jitter -1
    m.set_grid(Xs)
    m.set_data(X[:20], y[:20], np.empty((0, 2)), np.empty(0))             # lofi block: PD
    with pytest.raises(np.linalg.LinAlgError):
        m.append(X[20:21], y[20:21])       # K_HH + noise_H - 1 - ... < 0
    assert m.stats()["inc_factor"] == 1


@pytest.fixture(scope="module")
def split_ctx():
    """Incremental, but appends and predicts as separate launch groups."""
    from mfgp_coverage_amd import _lib
    c = _lib.Context(0)
    c.set_fused(False)
    return c


@pytest.mark.parametrize("fused", [True, False])
def test_batched_device_incremental_headline_pattern(full_ctx, split_ctx, fused):
    """Batched device-source appends over four MF GPs with the benchmark's
    truncate/append step -- one k_inc_stream launch streaming the cells too
    (fused) or k_inc_stream + k_vstream -- against the full-recompute path and, on the last
    step, the oracle. GP 2 samples off the grid: its L21 is solved inside the
    launch before the cell tiles may read it."""
    import torch
    from mfgp_coverage_amd import _lib
    G, NL, NH0, k, B = 48, 400, 500, 8, 4
    ctx = _lib.context() if fused else split_ctx
    cases = [_points(G, NL + NH0 + 4 * k, seed=100 + b, ongrid=(b != 2)) for b in range(B)]
    inc = [_model(ctx, "mf", X[:NL + NH0], y[:NL + NH0], NL, Xs)[0] for Xs, X, y in cases]
    full = [_model(full_ctx, "mf", X[:NL + NH0], y[:NL + NH0], NL, Xs)[0] for Xs, X, y in cases]
    M = cases[0][0].shape[0]
    for step in range(4):
        lo = NL + NH0 + step * k
        Xn = np.ascontiguousarray(np.vstack([X[lo:lo + k] for _, X, _ in cases]))
        yn = np.ascontiguousarray(np.concatenate([y[lo:lo + k] for _, _, y in cases]))
        Xd, yd = torch.from_numpy(Xn).cuda(), torch.from_numpy(yn).cuda()
        outs = []
        for models, c in ((inc, ctx), (full, full_ctx)):
            for mdl in models:
                mdl.truncate(NH0)
            mu_d = torch.empty(B * M, dtype=torch.float64, device="cuda")
            var_d = torch.empty(B * M, dtype=torch.float64, device="cuda")
            vmax = torch.full((B,), -1.0, dtype=torch.float64, device="cuda")
            varg = torch.full((B,), -1, dtype=torch.int64, device="cuda")
            _lib.batch_append_predict(models, Xd.data_ptr(), yd.data_ptr(), [k] * B, mu_d.data_ptr(),
                                      var_d.data_ptr(), vmax_ptr=vmax.data_ptr(), vargmax_ptr=varg.data_ptr())
            v = var_d.cpu().numpy().reshape(B, M)
            # fused np.amax / np.argmax (k_vstream and k_predict epilogues)
            np.testing.assert_array_equal(vmax.cpu().numpy(), v.max(1))
            np.testing.assert_array_equal(varg.cpu().numpy(), v.argmax(1))
            outs.append((mu_d.cpu().numpy(), var_d.cpu().numpy()))
        (mu, var), (mu_f, var_f) = outs
        assert _err(mu, var, mu_f, var_f, HYP_MF) < 1e-8
    for b, (Xs, X, y) in enumerate(cases):
        Xr = np.vstack([X[:NL + NH0], X[lo:lo + k]])
        yr = np.concatenate([y[:NL + NH0], y[lo:lo + k]])
        mu_r, var_r = _ref("mf", Xr, yr, NL, Xs, HYP_MF)
        assert _err(mu[b * M:(b + 1) * M], var[b * M:(b + 1) * M], mu_r, var_r, HYP_MF) < TOL
    for mdl in inc:
        st = mdl.stats()   # step 0 has no resident V yet (set_data): one full predict
        assert st["inc_factor"] == 4 and st["full_predict"] == 1 and st["vstream"] == 3, st


def test_headline_size_incremental_vs_full(full_ctx):
    """Headline size (128x128 grid, N = 1024 + 1024, australia8): the benchmark's step on the
    incremental path equals the full recompute (size-independent property)."""
    from mfgp_coverage_amd import _lib
    Xs, X, y = _points(128, 2048 + 16, seed=7, ongrid=True)
    a, _ = _model(_lib.context(), "mf", X[:2040], y[:2040], 1024, Xs)
    b, _ = _model(full_ctx, "mf", X[:2040], y[:2040], 1024, Xs)
    a.predict()
    for lo in (2040, 2048):
        a.truncate(1016)
        b.truncate(1016)
        a.append(X[lo:lo + 8], y[lo:lo + 8])
        b.append(X[lo:lo + 8], y[lo:lo + 8])
        mu, var = a.predict()
        mu_f, var_f = b.predict()
        assert _err(mu, var, mu_f, var_f, HYP_MF) < 1e-8
        assert np.all(var > -1e-12)
    assert a.stats()["vstream"] == 2


@pytest.mark.parametrize("layout", ["x_major", "y_major", "warped", "shuffled", "line"])
def test_grid_layouts_locate_new_points(layout):
    """The append kernel finds a new point's grid cell (whose V column it gathers)
    by lattice probes when the grid is a meshgrid of monotone axes, in either
    order and with uneven spacing, and by a scan otherwise; both must pick the
    same cell, so every layout streams and matches the oracle."""
    from mfgp_coverage_amd import _lib
    rng = np.random.default_rng(17)
    gx = np.linspace(0.0, 1.0, 40)
    gy = np.linspace(-0.5, 0.7, 33)[::-1]                       # decreasing axis
    if layout == "warped":
        gx = gx ** 2.2
    if layout == "line":
        Xs = np.column_stack([gx, np.full_like(gx, 0.25)])
    elif layout == "y_major":
        Xs = np.array([(a, b) for b in gy for a in gx])
    else:
        Xs = np.array([(a, b) for a in gx for b in gy])
    if layout == "shuffled":
        Xs = Xs[rng.permutation(Xs.shape[0])]
    n0 = min(120, Xs.shape[0] - 16)
    idx = rng.choice(Xs.shape[0], n0 + 16, replace=False)
    X = Xs[idx]
    y = _field(X, rng)
    m, hyp = _model(_lib.context(), "sf", X[:n0], y[:n0], 0, Xs)
    st = m.stats()
    lattice = layout != "shuffled"
    assert (st["lattice_nx"] > 0) == lattice, st
    if layout == "line":
        assert (st["lattice_nx"], st["lattice_ny"]) == (40, 1)
    elif lattice:
        assert (st["lattice_nx"], st["lattice_ny"]) == (40, 33)
    m.predict()
    for a, b in ((n0, n0 + 9), (n0 + 9, n0 + 16)):
        m.append(X[a:b], y[a:b])
        mu, var = m.predict()
        mu_r, var_r = _ref("sf", X[:b], y[:b], 0, Xs, hyp)
        assert _err(mu, var, mu_r, var_r, hyp) < TOL
    st = m.stats()
    assert st["inc_factor"] == 2 and st["vstream"] == 2


@pytest.mark.parametrize("fused", [True, False])
def test_batched_ragged_fused_append_predict(full_ctx, split_ctx, fused):
    """k_inc_stream over GPs with different producer counts and cell-tile counts:
    new rows entering a fresh 64-row block (n0 = 256), straddling one (n0 = 127),
    KINC = 16 rows at once and a single row; device sources; the fused VarMax."""
    import torch
    from mfgp_coverage_amd import _lib
    ctx = _lib.context() if fused else split_ctx
    specs = [(48, 100, 156, 8), (40, 50, 250, 16), (32, 30, 90, 1), (33, 60, 67, 5)]   # G, NL, NH0, k
    steps = 3
    cases = [_points(G, NL + NH0 + steps * k, seed=300 + i, ongrid=True) for i, (G, NL, NH0, k) in enumerate(specs)]
    inc = [_model(ctx, "mf", X[:NL + NH0], y[:NL + NH0], NL, Xs)[0]
           for (Xs, X, y), (G, NL, NH0, k) in zip(cases, specs)]
    full = [_model(full_ctx, "mf", X[:NL + NH0], y[:NL + NH0], NL, Xs)[0]
            for (Xs, X, y), (G, NL, NH0, k) in zip(cases, specs)]
    Ms = [c[0].shape[0] for c in cases]
    off = np.concatenate([[0], np.cumsum(Ms)])
    for step in range(steps):
        Xn, yn = [], []
        for (Xs, X, y), (G, NL, NH0, k) in zip(cases, specs):
            lo = NL + NH0 + step * k
            Xn.append(X[lo:lo + k])
            yn.append(y[lo:lo + k])
        Xd = torch.from_numpy(np.ascontiguousarray(np.vstack(Xn))).cuda()
        yd = torch.from_numpy(np.ascontiguousarray(np.concatenate(yn))).cuda()
        outs = []
        for models in (inc, full):
            for mdl, sp in zip(models, specs):
                mdl.truncate(sp[2])
            mu_d = torch.empty(int(off[-1]), dtype=torch.float64, device="cuda")
            var_d = torch.empty(int(off[-1]), dtype=torch.float64, device="cuda")
            vmax = torch.full((len(specs),), -1.0, dtype=torch.float64, device="cuda")
            _lib.batch_append_predict(models, Xd.data_ptr(), yd.data_ptr(), [sp[3] for sp in specs],
                                      mu_d.data_ptr(), var_d.data_ptr(), vmax_ptr=vmax.data_ptr())
            v = var_d.cpu().numpy()
            np.testing.assert_array_equal(vmax.cpu().numpy(), [v[off[i]:off[i + 1]].max() for i in range(len(specs))])
            outs.append((mu_d.cpu().numpy(), v))
        (mu, var), (mu_f, var_f) = outs
        for i in range(len(specs)):
            s_ = slice(off[i], off[i + 1])
            assert _err(mu[s_], var[s_], mu_f[s_], var_f[s_], HYP_MF) < 1e-8, (step, i)
    for i, ((Xs, X, y), (G, NL, NH0, k)) in enumerate(zip(cases, specs)):
        lo = NL + NH0 + (steps - 1) * k
        Xr = np.vstack([X[:NL + NH0], X[lo:lo + k]])
        yr = np.concatenate([y[:NL + NH0], y[lo:lo + k]])
        mu_r, var_r = _ref("mf", Xr, yr, NL, Xs, HYP_MF)
        s_ = slice(off[i], off[i + 1])
        assert _err(mu[s_], var[s_], mu_r, var_r, HYP_MF) < TOL
        # the factor itself equals a fresh Cholesky of the same rows
        np.testing.assert_allclose(inc[i].factor(), full[i].factor(), rtol=1e-6, atol=1e-9)
        st = inc[i].stats()
        assert st["inc_factor"] == steps and st["vstream"] == steps - 1, st


@pytest.mark.gpu
@pytest.mark.parametrize("B", [2, 4, 8])
def test_headline_batch_default_step_vs_full(full_ctx, B):
    """Batches of B headline-size MF GPs (128x128, N = 2040 + 8) through the library's
    default gates. On MI355X (256 CUs) the bordered append + predict of every batch is
    the lattice-separable step: one launch (k_inc_lat_arg, GEMM tiles in the launch)
    at B = 2 / 4, two launches at B = 8 (k_inc_lat_arg + k_lat_gemm2_arg: its 256
    tiles fill the chip). Each must equal the full recompute (the reference's work:
    refactor + V from scratch) to 1e-8 in the parity metric, the fused np.amax /
    np.argmax must be those of its variance, and GP 0 must equal the oracle at every
    cell."""
    import torch
    from mfgp_coverage_amd import _lib
    G, NL, NH0, k = 128, 1024, 1016, 8
    ctx = _lib.context()
    cases = [_points(G, NL + NH0 + k, seed=300 + b, ongrid=True) for b in range(B)]
    inc = [_model(ctx, "mf", X[:NL + NH0], y[:NL + NH0], NL, Xs)[0] for Xs, X, y in cases]
    full = [_model(full_ctx, "mf", X[:NL + NH0], y[:NL + NH0], NL, Xs)[0] for Xs, X, y in cases]
    for mdl in inc:
        mdl.predict()                      # V resident: the appends below are bordered steps
    M = G * G
    lo = NL + NH0
    Xn = np.ascontiguousarray(np.vstack([X[lo:lo + k] for _, X, _ in cases]))
    yn = np.ascontiguousarray(np.concatenate([y[lo:lo + k] for _, _, y in cases]))
    Xd, yd = torch.from_numpy(Xn).cuda(), torch.from_numpy(yn).cuda()
    outs = []
    for models in (inc, full):
        mu_d = torch.empty(B * M, dtype=torch.float64, device="cuda")
        var_d = torch.empty(B * M, dtype=torch.float64, device="cuda")
        vmax = torch.full((B,), -1.0, dtype=torch.float64, device="cuda")
        varg = torch.full((B,), -1, dtype=torch.int64, device="cuda")
        _lib.batch_append_predict(models, Xd.data_ptr(), yd.data_ptr(), [k] * B, mu_d.data_ptr(),
                                  var_d.data_ptr(), vmax_ptr=vmax.data_ptr(), vargmax_ptr=varg.data_ptr())
        outs.append((mu_d.cpu().numpy().reshape(B, M), var_d.cpu().numpy().reshape(B, M),
                     vmax.cpu().numpy(), varg.cpu().numpy()))
    (mu, var, vm, va), (mu_f, var_f, vm_f, va_f) = outs
    for b in range(B):
        assert _err(mu[b], var[b], mu_f[b], var_f[b], HYP_MF) < 1e-8
        assert vm[b] == np.amax(var[b]) and va[b] == int(np.argmax(var[b]))
    Xs0, X0, y0 = cases[0]
    mu_r, var_r = _ref("mf", X0[:lo + k], y0[:lo + k], NL, Xs0, HYP_MF)
    assert _err(mu[0], var[0], mu_r, var_r, HYP_MF) < TOL
    for m in inc:
        st = m.stats()
        assert st["inc_factor"] == 1 and st["lattice"] == 1, st
        assert st["lattice_g2"] == (1 if B == 8 else 0), st


@pytest.mark.parametrize("B,rsplit", [(1, 1), (2, 2), (4, 4), (8, 0), (2, 1), (8, 4)])
def test_headline_vstream_row_splits_vs_full(monkeypatch, full_ctx, B, rsplit):
    """The one-pass predict (k_inc_stream / k_inc_stream_arg) at the headline size with
    the lattice step off, so the V stream's row splits run on the grids it serves
    (non-lattice grids, the LAT_MAXD refresh, one GP): the host's rule (rsplit 0: R = 4 /
    2 / 1 for B = 1-2 / 4 / 8) and forced R = 1 / 2 / 4 (MFGP_RSPLIT). Each must equal
    the full recompute to 1e-8 in the parity metric with the fused max / argmax of its
    variance (the B = 2 / 4 / 8 stream test had moved to the lattice path)."""
    import torch
    from mfgp_coverage_amd import _lib
    G, NL, NH0, k = 128, 1024, 1016, 8
    if rsplit:
        monkeypatch.setenv("MFGP_RSPLIT", str(rsplit))
    ctx = _lib.Context(0)
    ctx.set_lattice(False)
    cases = [_points(G, NL + NH0 + k, seed=330 + b, ongrid=True) for b in range(B)]
    inc = [_model(ctx, "mf", X[:NL + NH0], y[:NL + NH0], NL, Xs)[0] for Xs, X, y in cases]
    full = [_model(full_ctx, "mf", X[:NL + NH0], y[:NL + NH0], NL, Xs)[0] for Xs, X, y in cases]
    for mdl in inc:
        mdl.predict()
    M = G * G
    lo = NL + NH0
    Xn = np.ascontiguousarray(np.vstack([X[lo:lo + k] for _, X, _ in cases]))
    yn = np.ascontiguousarray(np.concatenate([y[lo:lo + k] for _, _, y in cases]))
    Xd, yd = torch.from_numpy(Xn).cuda(), torch.from_numpy(yn).cuda()
    outs = []
    for models in (inc, full):
        mu_d = torch.empty(B * M, dtype=torch.float64, device="cuda")
        var_d = torch.empty(B * M, dtype=torch.float64, device="cuda")
        vmax = torch.full((B,), -1.0, dtype=torch.float64, device="cuda")
        varg = torch.full((B,), -1, dtype=torch.int64, device="cuda")
        _lib.batch_append_predict(models, Xd.data_ptr(), yd.data_ptr(), [k] * B, mu_d.data_ptr(),
                                  var_d.data_ptr(), vmax_ptr=vmax.data_ptr(), vargmax_ptr=varg.data_ptr())
        outs.append((mu_d.cpu().numpy().reshape(B, M), var_d.cpu().numpy().reshape(B, M),
                     vmax.cpu().numpy(), varg.cpu().numpy()))
    (mu, var, vm, va), (mu_f, var_f, vm_f, va_f) = outs
    for b in range(B):
        assert _err(mu[b], var[b], mu_f[b], var_f[b], HYP_MF) < 1e-8, (B, rsplit, b)
        assert vm[b] == np.amax(var[b]) and va[b] == int(np.argmax(var[b]))
    for m in inc:
        st = m.stats()
        assert st["inc_factor"] == 1 and st["lattice"] == 0 and st["vstream"] >= 1, st
    ctx.synchronize()


@pytest.mark.parametrize("kind", ["sf", "mf"])
def test_deferred_appends_vs_oracle(kind):
    """Deferred appends (mfgp_ctx_set_deferred_appends): appends stage their rows and the
    predict runs the bordered append and the one-pass predict as one launch. Sequences of
    single and repeated appends (staged rows up to KINC, then beyond it: a full refactor),
    each predict against the oracle."""
    from mfgp_coverage_amd import _lib
    ctx = _lib.Context(0)
    ctx.set_deferred_appends(True)
    Xs, X, y = _points(40, 400, seed=11, ongrid=True)
    NL = 0 if kind == "sf" else 150
    n = NL + 120
    m, hyp = _model(ctx, kind, X[:n], y[:n], NL, Xs)
    m.predict()
    for ks in ([8], [1], [4, 4], [16], [0], [8, 8], [5, 9, 3], [2]):
        for kk in ks:
            m.append(X[n:n + kk], y[n:n + kk])
            n += kk
        mu, var = m.predict()
        mu_r, var_r = _ref(kind, X[:n], y[:n], NL, Xs, hyp)
        assert _err(mu, var, mu_r, var_r, hyp) < TOL, (ks, _err(mu, var, mu_r, var_r, hyp))
    st = m.stats()
    assert st["inc_factor"] >= 6 and st["full_factor"] >= 2, st   # [5, 9, 3] exceeds KINC: refactor


def test_deferred_append_not_pd_raises_at_predict():
    """Deferred, the non-PD bordered step of test_incremental_not_pd_raises is reported by
    the predict that runs it (the eager default reports it from the append)."""
    from mfgp_coverage_amd import _lib
    ctx = _lib.Context(0)
    ctx.set_deferred_appends(True)
    Xs, X, y = _points(24, 30, seed=2, ongrid=True)
    hyp = np.array([0.0, 0.0, -1.0, 0.0, -3.0, -1.0, -1.0, 2.0, -20.0])
    m = _lib.Model(ctx, _lib.MF, hyp, -1.0)
    m.set_grid(Xs)
    m.set_data(X[:20], y[:20], np.empty((0, 2)), np.empty(0))
    m.predict()
    m.append(X[20:21], y[20:21])
    with pytest.raises(np.linalg.LinAlgError):
        m.predict()


def test_speculative_predict_after_append():
    """An eager append that follows a predict runs the bordered append and the one-pass
    predict in one launch and keeps the result for the next predict. Every change to
    the model in between (more rows, hyperparameters, grid) must drop it; repeated
    predicts return the same bits; a non-PD append still raises at the append."""
    from mfgp_coverage_amd import _lib
    Xs, X, y = _points(36, 400, seed=13, ongrid=True)
    NL, n = 150, 270
    m, hyp = _model(_lib.context(), "mf", X[:n], y[:n], NL, Xs)
    m.predict()
    for step, kk in enumerate((8, 3, 8, 1)):
        m.append(X[n:n + kk], y[n:n + kk])
        n += kk
        if step == 2:                      # a second append before the predict: the first's result is stale
            m.append(X[n:n + 2], y[n:n + 2])
            n += 2
        mu, var = m.predict()
        mu_r, var_r = _ref("mf", X[:n], y[:n], NL, Xs, hyp)
        assert _err(mu, var, mu_r, var_r, hyp) < TOL, step
        mu2, var2 = m.predict()
        np.testing.assert_array_equal(mu2, mu)
        np.testing.assert_array_equal(var2, var)
    # a hyperparameter change after the append: the kept result is not used
    m.append(X[n:n + 4], y[n:n + 4])
    n += 4
    hyp2 = hyp.copy()
    hyp2[2] += 0.1
    m.set_hyp(hyp2, 1e-8)
    mu, var = m.predict()
    mu_r, var_r = _ref("mf", X[:n], y[:n], NL, Xs, hyp2)
    assert _err(mu, var, mu_r, var_r, hyp2) < TOL
    # a grid change after the append
    m.set_hyp(hyp, 1e-8)
    m.predict()
    m.append(X[n:n + 4], y[n:n + 4])
    n += 4
    Xs2 = Xs[::3].copy()
    m.set_grid(Xs2)
    mu, var = m.predict()
    mu_r, var_r = _ref("mf", X[:n], y[:n], NL, Xs2, hyp)
    assert _err(mu, var, mu_r, var_r, hyp) < TOL


def test_speculative_append_not_pd_raises_at_append():
    from mfgp_coverage_amd import _lib
    Xs, X, y = _points(24, 30, seed=2, ongrid=True)
    hyp = np.array([0.0, 0.0, -1.0, 0.0, -3.0, -1.0, -1.0, 2.0, -20.0])
    m = _lib.Model(_lib.context(), _lib.MF, hyp, -1.0)
    m.set_grid(Xs)
    m.set_data(X[:20], y[:20], np.empty((0, 2)), np.empty(0))
    m.predict()
    m.append(X[20:20], y[20:20])           # k = 0
    m.predict()
    with pytest.raises(np.linalg.LinAlgError):
        m.append(X[20:21], y[20:21])       # speculative form (after a predict): raises here


@pytest.mark.parametrize("lattice", [False, True])
def test_early_verdict_append_then_other_calls(lattice):
    """The eager append of one GP returns at the step's L22 verdict (the launch
    publishes it before it computes the posterior): every later call -- factor
    download, clone, truncate, a second append, destroy, a predict -- first waits
    for that launch, so each sees the appended state. Both one-GP launches: the V
    stream (k_inc_stream1) and the lattice step (forced: k_inc_lat_arg)."""
    import gc

    from mfgp_coverage_amd import _lib
    Xs, X, y = _points(36, 420, seed=17, ongrid=True)
    NL, n = 150, 270
    ctx = _lib.Context(0)
    if lattice:
        ctx.set_lattice("force")
    m, hyp = _model(ctx, "mf", X[:n], y[:n], NL, Xs)
    m.predict()
    m.append(X[n:n + 8], y[n:n + 8])
    n += 8
    L = m.factor()                                         # right after the early return
    assert L.shape == (n, n) and np.all(np.isfinite(L))
    m.predict()
    m.append(X[n:n + 8], y[n:n + 8])
    n += 8
    c = m.clone()                                          # clone of a launch still running
    mu_c, var_c = c.predict()
    mu_r, var_r = _ref("mf", X[:n], y[:n], NL, Xs, hyp)
    assert _err(mu_c, var_c, mu_r, var_r, hyp) < TOL
    mu, var = m.predict()
    assert _err(mu, var, mu_r, var_r, hyp) < TOL
    m.append(X[n:n + 4], y[n:n + 4])
    m.truncate(n - NL - 2)                                 # truncate while it runs
    n -= 2
    mu, var = m.predict()
    mu_r, var_r = _ref("mf", X[:n], y[:n], NL, Xs, hyp)
    assert _err(mu, var, mu_r, var_r, hyp) < TOL
    c.append(X[n:n + 8], y[n:n + 8])
    del c                                                  # destroyed while its launch runs
    gc.collect()
    m.append(X[n:n + 8], y[n:n + 8])
    n += 8
    mu, var = m.predict()
    mu_r, var_r = _ref("mf", X[:n], y[:n], NL, Xs, hyp)
    assert _err(mu, var, mu_r, var_r, hyp) < TOL
    assert (m.stats()["lattice"] > 0) == lattice, m.stats()
    # the appends above did return at the published verdict (without it
    # every call here would still pass, each after a full synchronise)
    assert m.stats()["early_pd"] >= 3, m.stats()


def test_dropin_updt_hifi_not_pd_raises_and_stacks(gp_mod):
    """The drop-in updt_hifi sends the rows to the device before it stacks them on
    the host (the append returns at the verdict; the stacking overlaps the launch):
    a non-PD append still raises LinAlgError at updt_hifi and leaves the stacked
    rows, as the reference does (it stacks, then factors: gp:531-542)."""
    Xs, X, y = _points(24, 30, seed=2, ongrid=True)
    m = gp_mod.MFGP(X[:20], y[:20, None], np.empty((0, 2)), np.empty((0, 1)), 1, 1)
    m.hyp = np.array([0.0, 0.0, -1.0, 0.0, -3.0, -1.0, -1.0, 2.0, -20.0])
    m.jitter = -1.0
    m.predict(Xs)
    m.updt_hifi(X[20:20], y[20:20, None])
    m.predict(Xs)
    with pytest.raises(np.linalg.LinAlgError):
        m.updt_hifi(X[20:21], y[20:21, None])
    assert m.X_H.shape == (1, 2) and m.y_H.shape == (1, 1)


def _bad_and_good(ctx, Xs, X, y):
    """A model whose next append is not positive definite (negative jitter, as in
    test_speculative_append_not_pd_raises_at_append) and a well-posed one."""
    from mfgp_coverage_amd import _lib
    hyp = np.array([0.0, 0.0, -1.0, 0.0, -3.0, -1.0, -1.0, 2.0, -20.0])
    bad = _lib.Model(ctx, _lib.MF, hyp, -1.0)
    bad.set_grid(Xs)
    bad.set_data(X[:20], y[:20], np.empty((0, 2)), np.empty(0))
    good, hyp_g = _model(ctx, "mf", X[:20], y[:20], 10, Xs)
    return bad, good, hyp_g


def test_batch_async_not_pd_is_traced_to_its_model():
    """a non-PD factor inside an asynchronous batch is reported at
    mfgp_ctx_synchronize and dropped from ITS model, so that model's next predict
    refactors (and raises again) instead of serving the failed factor; the other
    model of the batch is unaffected."""
    import torch
    from mfgp_coverage_amd import _lib
    ctx = _lib.Context(0)
    Xs, X, y = _points(24, 30, seed=2, ongrid=True)
    bad, good, hyp_g = _bad_and_good(ctx, Xs, X, y)
    M = Xs.shape[0]
    mu = torch.empty(2 * M, dtype=torch.float64, device="cuda")
    var = torch.empty_like(mu)
    _lib.batch_predict([bad, good], mu.data_ptr(), var.data_ptr())
    ctx.synchronize()
    Xn = torch.from_numpy(np.ascontiguousarray(np.concatenate([X[20:21], X[21:22]]))).cuda()
    yn = torch.from_numpy(np.ascontiguousarray(np.concatenate([y[20:21], y[21:22]]))).cuda()
    _lib.batch_append_predict([bad, good], Xn.data_ptr(), yn.data_ptr(), [1, 1], mu.data_ptr(), var.data_ptr(),
                              asynchronous=True)
    with pytest.raises(np.linalg.LinAlgError):
        ctx.synchronize()
    with pytest.raises(np.linalg.LinAlgError):
        bad.predict()
    mu_g, var_g = good.predict()
    Xg = np.concatenate([X[:20], X[21:22]])
    yg = np.concatenate([y[:20], y[21:22]])
    mu_r, var_r = _ref("mf", Xg, yg, 10, Xs, hyp_g)
    assert _err(mu_g, var_g, mu_r, var_r, hyp_g) < TOL


def test_destroy_before_synchronize():
    """a model destroyed (Python GC) while its asynchronous batch is
    pending leaves no dangling status word behind: the context synchronises
    cleanly and the surviving model's result is right."""
    import gc

    import torch
    from mfgp_coverage_amd import _lib
    ctx = _lib.Context(0)
    Xs, X, y = _points(24, 60, seed=5, ongrid=True)
    a, hyp = _model(ctx, "mf", X[:40], y[:40], 20, Xs)
    b, _ = _model(ctx, "mf", X[:40], y[:40], 20, Xs)
    M = Xs.shape[0]
    mu = torch.empty(2 * M, dtype=torch.float64, device="cuda")
    var = torch.empty_like(mu)
    _lib.batch_predict([a, b], mu.data_ptr(), var.data_ptr())
    ctx.synchronize()
    Xn = torch.from_numpy(np.ascontiguousarray(np.concatenate([X[40:44], X[44:48]]))).cuda()
    yn = torch.from_numpy(np.ascontiguousarray(np.concatenate([y[40:44], y[44:48]]))).cuda()
    _lib.batch_append_predict([a, b], Xn.data_ptr(), yn.data_ptr(), [4, 4], mu.data_ptr(), var.data_ptr(),
                              asynchronous=True)
    del b
    gc.collect()
    ctx.synchronize()
    mu_a, var_a = a.predict()
    mu_r, var_r = _ref("mf", X[:44], y[:44], 20, Xs, hyp)
    assert _err(mu_a, var_a, mu_r, var_r, hyp) < TOL


def test_capacity_growth_clamped_to_full_predict_limit():
    """capacity grows by 1.5x on appends; from N ~ 13,000 that would pass
    the full predict's limit (ld <= 16383, include/mfgp_hip.h) and a later full
    predict (here: after a grid change) would fail although N fits. The growth is
    clamped to that limit, so the full predict after the appends runs and agrees
    with a model built from the same rows in one set_data."""
    from mfgp_coverage_amd import _lib
    rng = np.random.default_rng(21)
    N0, k = 13000, 16
    X = rng.random((N0 + 3 * k, 2))
    y = np.sin(4 * X[:, 0]) * np.cos(3 * X[:, 1]) + 0.1 * rng.standard_normal(X.shape[0])
    hyp = HYP_SF
    ctx = _lib.context()
    m = _lib.Model(ctx, _lib.SF, hyp, 1e-8)
    m.set_grid(_grid(16))
    m.set_data(np.empty((0, 2)), np.empty(0), X[:N0], y[:N0])
    m.predict()
    for s in range(3):
        m.append(X[N0 + s * k:N0 + (s + 1) * k], y[N0 + s * k:N0 + (s + 1) * k])
    Xs2 = _grid(12)
    m.set_grid(Xs2)
    mu, var = m.predict()             # full predict at N = 13,048
    ref = _lib.Model(ctx, _lib.SF, hyp, 1e-8)
    ref.set_grid(Xs2)
    ref.set_data(np.empty((0, 2)), np.empty(0), X, y)
    mu_r, var_r = ref.predict()
    assert np.all(np.isfinite(mu)) and np.all(np.isfinite(var))
    assert _err(mu, var, mu_r, var_r, hyp) < 1e-8
