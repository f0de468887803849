"""The lattice-separable incremental step (k_inc_lat).

On a lattice grid with a well-conditioned K the bordered append + predict
(simulator.py:864-892 -> gp:531-542, gp:401-438) runs without a pass over the
resident V: w = K11^-1 K12 from the explicit inverse, the SE kernel's
separability turns L21 V_old into a GEMM over the training terms, and var / mu
are updated from the resident posterior of the old rows. Every step here is
checked against the CPU oracle at every cell (PARITY_TOL) and against the V
stream of the same library (mfgp_ctx_set_lattice(0)); the path counters assert
which kernel ran. Also: ragged batches with the fused var max / argmax, appends
of 1..16 rows (both GEMM row groupings, KA = 8 and 16), points off the grid,
truncate + re-append (the benchmark's step), capacity growth (F and the tables
move), fp32 models, and the conditioning gate (the reference's anti_two_corners
noise stays on the V stream).
"""
import numpy as np
import pytest

from oracle import gp_oracle as O

pytestmark = pytest.mark.gpu

TOL = O.PARITY_TOL


def _grid(G):
    g = np.linspace(0.0, 1.0, G)
    return np.array([(a, b) for a in g for b in g])


def _data(G, n, seed, offgrid_from=None):
    rng = np.random.default_rng(seed)
    Xs = _grid(G)
    X = Xs[rng.choice(Xs.shape[0], n, replace=False)].copy()
    if offgrid_from is not None:
        X[offgrid_from:] += 0.29 / (G - 1)
    c = rng.random((3, 2))
    y = sum(np.exp(-np.sum((X - ci) ** 2, 1) / 0.05) for ci in c)
    y = y / y.max() + 0.1 * rng.standard_normal(n)
    return Xs, X, y


def _hyp(name):
    from mfgp_coverage_amd.synthetic import HYP
    return HYP[name].copy()


def _model(ctx, hyp, X, y, NL, Xs, dtype=None):
    from mfgp_coverage_amd import _lib
    kind = _lib.SF if hyp.shape[0] == 4 else _lib.MF
    m = _lib.Model(ctx, kind, hyp, 1e-8, dtype=_lib.F64 if dtype is None else dtype)
    m.set_grid(Xs)
    if kind == _lib.SF:
        m.set_data(np.empty((0, 2)), np.empty(0), X, y)
    else:
        m.set_data(X[:NL], y[:NL], X[NL:], y[NL:])
    return m


def _ref(hyp, X, y, NL, Xs):
    if hyp.shape[0] == 4:
        return O.sf_diag(X, y, hyp, Xs)
    return O.mf_diag(X[:NL], y[:NL], X[NL:], y[NL:], hyp, Xs)


def _err(hyp, mu, var, mu_r, var_r):
    return max(O.parity_errors(mu, var, mu_r, var_r, O.prior_variance(hyp)))


@pytest.fixture(scope="module", autouse=True)
def lattice_forced():
    """These cases are small (one to three GPs on small grids): force the lattice
    step (the library keeps the V stream for batches that cannot fill the GPU)."""
    from mfgp_coverage_amd import _lib
    _lib.context().set_lattice("force")
    yield
    _lib.context().set_lattice(True)


@pytest.fixture(scope="module")
def vctx():
    """A context without the lattice step: the V stream of the same library."""
    from mfgp_coverage_amd import _lib
    c = _lib.Context(0)
    c.set_lattice(False)
    return c


CASES = [("australia8_mf", 64, 120), ("australia3_sf", 51, 0), ("australia6_mf", 48, 150)]


@pytest.mark.parametrize("hypname,G,NL", CASES)
@pytest.mark.parametrize("ks", [(8, 8, 8, 8, 8), (1, 3, 16, 5, 12, 2)])
def test_lattice_sequence_vs_oracle_and_vstream(hypname, G, NL, ks, vctx):
    from mfgp_coverage_amd import _lib
    hyp = _hyp(hypname)
    N0 = 300
    Xs, X, y = _data(G, N0 + sum(ks), seed=len(ks) + G)
    m = _model(_lib.context(), hyp, X[:N0], y[:N0], NL, Xs)
    v = _model(vctx, hyp, X[:N0], y[:N0], NL, Xs)
    m.predict()
    v.predict()
    n = N0
    for k in ks:
        m.append(X[n:n + k], y[n:n + k])
        v.append(X[n:n + k], y[n:n + k])
        n += k
        mu, var = m.predict()
        mu_v, var_v = v.predict()
        mu_r, var_r = _ref(hyp, X[:n], y[:n], NL, Xs)
        assert _err(hyp, mu, var, mu_r, var_r) < TOL, (n, k)
        assert _err(hyp, mu, var, mu_v, var_v) < 1e-8, (n, k)   # lattice == V stream to rounding
    st, sv = m.stats(), v.stats()
    assert st["lattice"] == len(ks) and st["inc_factor"] == len(ks) and st["full_predict"] == 1, st
    assert sv["lattice"] == 0 and sv["vstream"] == len(ks), sv
    # the factor the lattice step leaves behind equals the V stream's (both bordered)
    np.testing.assert_allclose(m.factor(), v.factor(), rtol=1e-9, atol=1e-12)


def test_lattice_offgrid_points():
    """New points off the grid: the finish solves L21 itself (no V columns); the
    separable GEMM does not care where the training points lie."""
    from mfgp_coverage_amd import _lib
    hyp = _hyp("australia8_mf")
    N0, NL = 260, 100
    Xs, X, y = _data(40, N0 + 24, seed=3, offgrid_from=N0)
    m = _model(_lib.context(), hyp, X[:N0], y[:N0], NL, Xs)
    m.predict()
    n = N0
    for k in (8, 8, 8):
        m.append(X[n:n + k], y[n:n + k])
        n += k
        mu, var = m.predict()
        mu_r, var_r = _ref(hyp, X[:n], y[:n], NL, Xs)
        assert _err(hyp, mu, var, mu_r, var_r) < TOL
    assert m.stats()["lattice"] == 3


def test_lattice_batch_ragged_fused_argmax():
    """Three MF GPs of different sizes in one launch, device outputs, fused
    np.amax / np.argmax (simulator.py:672, 842; sim:352)."""
    import torch
    from mfgp_coverage_amd import _lib
    hyp = _hyp("australia8_mf")
    G = 56
    sizes = [(90, 200), (300, 37), (128, 128)]
    models, data = [], []
    for i, (nl, nh) in enumerate(sizes):
        Xs, X, y = _data(G, nl + nh + 40, seed=40 + i)
        models.append(_model(_lib.context(), hyp, X[:nl + nh], y[:nl + nh], nl, Xs))
        data.append((X, y, nl, nl + nh))
    M = Xs.shape[0]
    B = len(models)
    mu = torch.empty(B * M, dtype=torch.float64, device="cuda")
    var = torch.empty(B * M, dtype=torch.float64, device="cuda")
    vmax = torch.empty(B, dtype=torch.float64, device="cuda")
    vam = torch.empty(B, dtype=torch.int64, device="cuda")
    _lib.batch_predict(models, mu.data_ptr(), var.data_ptr())
    for step, k in enumerate((8, 5, 8, 8)):
        Xn = np.concatenate([d[0][d[3]:d[3] + k] for d in data])
        yn = np.concatenate([d[1][d[3]:d[3] + k] for d in data])
        Xt = torch.from_numpy(np.ascontiguousarray(Xn)).cuda()
        yt = torch.from_numpy(np.ascontiguousarray(yn)).cuda()
        _lib.batch_append_predict(models, Xt.data_ptr(), yt.data_ptr(), [k] * B, mu.data_ptr(), var.data_ptr(),
                                  vmax_ptr=vmax.data_ptr(), vargmax_ptr=vam.data_ptr())
        data = [(X, y, nl, n + k) for (X, y, nl, n) in data]
        mh, vh = mu.cpu().numpy().reshape(B, M), var.cpu().numpy().reshape(B, M)
        for i, (X, y, nl, n) in enumerate(data):
            mu_r, var_r = _ref(hyp, X[:n], y[:n], nl, Xs)
            assert _err(hyp, mh[i], vh[i], mu_r, var_r) < TOL, (step, i)
            assert vmax[i].item() == vh[i].max() and vam[i].item() == int(np.argmax(vh[i])), (step, i)
    for m in models:
        assert m.stats()["lattice"] == 4, m.stats()


def test_lattice_truncate_reappend():
    """The benchmark's step: append k rows, predict, truncate back; every step
    starts from the kept posterior of the same base rows."""
    from mfgp_coverage_amd import _lib
    hyp = _hyp("australia8_mf")
    N0, NL, k = 400, 200, 8
    Xs, X, y = _data(64, N0 + 4 * k, seed=9)
    m = _model(_lib.context(), hyp, X[:N0], y[:N0], NL, Xs)
    m.predict()
    for s in range(4):
        rows = slice(N0 + s * k, N0 + (s + 1) * k)
        m.truncate(N0 - NL)
        m.append(X[rows], y[rows])
        mu, var = m.predict()
        Xr = np.concatenate([X[:N0], X[rows]])
        yr = np.concatenate([y[:N0], y[rows]])
        mu_r, var_r = _ref(hyp, Xr, yr, NL, Xs)
        assert _err(hyp, mu, var, mu_r, var_r) < TOL, s
    assert m.stats()["lattice"] == 4


def test_lattice_f32_model():
    from mfgp_coverage_amd import _lib
    hyp = _hyp("australia9_mf")
    N0, NL = 500, 250
    Xs, X, y = _data(64, N0 + 24, seed=17)
    m = _model(_lib.context(), hyp, X[:N0], y[:N0], NL, Xs, dtype=_lib.F32)
    m.predict()
    n = N0
    for k in (8, 8, 8):
        m.append(X[n:n + k], y[n:n + k])
        n += k
        mu, var = m.predict()
        mu_r, var_r = _ref(hyp, X[:n], y[:n], NL, Xs)
        assert max(O.parity_errors_f32(mu, var, mu_r, var_r, O.prior_variance(hyp))) < O.F32_TOL
    assert m.stats()["lattice"] == 3


def test_conditioning_gate_keeps_v_stream(vctx):
    """anti_two_corners (noise e^-37.8: kss / (noise + jitter) = 6e6 > 1e4) stays
    on the V stream, where the lattice step would lose accuracy (its parity at this
    conditioning is the V stream's own, tests/test_gpu_parity.py replays): the
    same bits as a context without the lattice step."""
    from mfgp_coverage_amd import _lib
    hyp = _hyp("anti_two_corners_sf")
    N0 = 120
    Xs, X, y = _data(51, N0 + 16, seed=2)
    m = _model(_lib.context(), hyp, X[:N0], y[:N0], 0, Xs)
    v = _model(vctx, hyp, X[:N0], y[:N0], 0, Xs)
    m.predict()
    v.predict()
    for s in range(2):
        rows = slice(N0 + 8 * s, N0 + 8 * s + 8)
        m.append(X[rows], y[rows])
        v.append(X[rows], y[rows])
        mu, var = m.predict()
        mu_v, var_v = v.predict()
        assert np.array_equal(mu, mu_v) and np.array_equal(var, var_v)
    st = m.stats()
    assert st["lattice"] == 0 and st["vstream"] == 2, st


def test_lattice_after_hyp_change_rebuilds():
    """New hyperparameters: a full refactor, then the lattice step rebuilds F and
    the tables for the new generation (no stale state)."""
    from mfgp_coverage_amd import _lib
    hyp = _hyp("australia8_mf")
    N0, NL = 300, 120
    Xs, X, y = _data(48, N0 + 16, seed=23)
    m = _model(_lib.context(), hyp, X[:N0], y[:N0], NL, Xs)
    m.predict()
    m.append(X[N0:N0 + 8], y[N0:N0 + 8])
    m.predict()
    hyp2 = hyp.copy()
    hyp2[2] -= 0.3
    m.set_hyp(hyp2, 1e-8)
    m.predict()                       # full refactor + full predict at N0 + 8
    m.append(X[N0 + 8:N0 + 16], y[N0 + 8:N0 + 16])
    mu, var = m.predict()
    mu_r, var_r = _ref(hyp2, X[:N0 + 16], y[:N0 + 16], NL, Xs)
    assert _err(hyp2, mu, var, mu_r, var_r) < TOL
    st = m.stats()
    assert st["lattice"] == 2 and st["full_factor"] == 2, st


@pytest.mark.parametrize("lattice", ["force", False])
def test_lattice_descriptors_by_value_equal_upload(monkeypatch, lattice):
    """A batch step that is one k_inc_lat (or, lattice off, k_inc_stream) launch
    passes its descriptors as the kernel argument (k_inc_lat_arg /
    k_inc_stream_arg, no descriptor upload); MFGP_DESC_ARG=0 makes a context
    upload them instead. Same kernel body, so the same bits; ragged batches of
    1, 3 and 8 GPs (DESC_ARG_MAX) over several steps, fused argmax."""
    import torch
    from mfgp_coverage_amd import _lib
    hyp = _hyp("australia8_mf")
    G = 48

    def run(ctx, B):
        models, data = [], []
        for i in range(B):
            nl, nh = 100 + 17 * i, 150 - 9 * i
            Xs, X, y = _data(G, nl + nh + 40, seed=70 + i)
            models.append(_model(ctx, hyp, X[:nl + nh], y[:nl + nh], nl, Xs))
            data.append((X, y, nl + nh))
        M = Xs.shape[0]
        mu = torch.empty(B * M, dtype=torch.float64, device="cuda")
        var = torch.empty_like(mu)
        vmax = torch.empty(B, dtype=torch.float64, device="cuda")
        vam = torch.empty(B, dtype=torch.int64, device="cuda")
        _lib.batch_predict(models, mu.data_ptr(), var.data_ptr())
        out = []
        for step, k in enumerate((8, 3, 8, 8)):
            Xn = np.concatenate([X[n:n + k] for X, _, n in data])
            yn = np.concatenate([y[n:n + k] for _, y, n in data])
            Xt = torch.from_numpy(np.ascontiguousarray(Xn)).cuda()
            yt = torch.from_numpy(np.ascontiguousarray(yn)).cuda()
            _lib.batch_append_predict(models, Xt.data_ptr(), yt.data_ptr(), [k] * B, mu.data_ptr(), var.data_ptr(),
                                      vmax_ptr=vmax.data_ptr(), vargmax_ptr=vam.data_ptr())
            data = [(X, y, n + k) for X, y, n in data]
            out.append((mu.cpu().numpy(), var.cpu().numpy(), vmax.cpu().numpy(), vam.cpu().numpy()))
        key = "lattice" if lattice else "vstream"
        assert all(m.stats()[key] >= 4 for m in models), [m.stats() for m in models]
        if not lattice:
            assert all(m.stats()["lattice"] == 0 for m in models)
        ctx.synchronize()
        return out

    for B in (1, 3, 8):
        a = _lib.Context(0)
        a.set_lattice(lattice)
        monkeypatch.setenv("MFGP_DESC_ARG", "0")
        b = _lib.Context(0)
        monkeypatch.delenv("MFGP_DESC_ARG")
        b.set_lattice(lattice)
        ra, rb = run(a, B), run(b, B)
        for sa, sb in zip(ra, rb):
            for xa, xb in zip(sa, sb):
                assert np.array_equal(xa, xb), B


@pytest.mark.parametrize("ksplit,wu", [(1, 1), (2, 7), (4, 64), (8, 1024), (8, 2)])
def test_lattice_split_and_w_units_vs_oracle(monkeypatch, ksplit, wu):
    """Every split-K factor of the GEMM tiles (1, 2, 4, 8: the splits share the
    tile's cell passes; 8 = half a pass each) and w-unit count (the launch's total:
    1 = one unit per GP streams all of its F and stores every block alone; 7, 64 =
    blocks shared by several units, partials added in unit order; 1024 = one
    16-row step per unit, clamped to the GP's steps), forced through the context's
    diagnostic switches (MFGP_LAT_KSPLIT / MFGP_LAT_WU): two MF GPs on a 64 x 64
    grid, appends of 8 and 5 rows, against the oracle at every cell."""
    import torch
    from mfgp_coverage_amd import _lib
    monkeypatch.setenv("MFGP_LAT_KSPLIT", str(ksplit))
    monkeypatch.setenv("MFGP_LAT_WU", str(wu))
    ctx = _lib.Context(0)
    ctx.set_lattice("force")
    hyp = _hyp("australia8_mf")
    models, data = [], []
    for i, (nl, nh) in enumerate([(200, 300), (150, 421)]):
        Xs, X, y = _data(64, nl + nh + 20, seed=90 + i)
        models.append(_model(ctx, hyp, X[:nl + nh], y[:nl + nh], nl, Xs))
        data.append((X, y, nl, nl + nh))
    M = Xs.shape[0]
    mu = torch.empty(2 * M, dtype=torch.float64, device="cuda")
    var = torch.empty_like(mu)
    vmax = torch.empty(2, dtype=torch.float64, device="cuda")
    _lib.batch_predict(models, mu.data_ptr(), var.data_ptr())
    for k in (8, 5):
        Xn = np.concatenate([X[n:n + k] for X, _, _, n in data])
        yn = np.concatenate([y[n:n + k] for _, y, _, n in data])
        Xt = torch.from_numpy(np.ascontiguousarray(Xn)).cuda()
        yt = torch.from_numpy(np.ascontiguousarray(yn)).cuda()
        _lib.batch_append_predict(models, Xt.data_ptr(), yt.data_ptr(), [k, k], mu.data_ptr(), var.data_ptr(),
                                  vmax_ptr=vmax.data_ptr())
        data = [(X, y, nl, n + k) for X, y, nl, n in data]
        mh, vh = mu.cpu().numpy().reshape(2, M), var.cpu().numpy().reshape(2, M)
        for i, (X, y, nl, n) in enumerate(data):
            mu_r, var_r = _ref(hyp, X[:n], y[:n], nl, Xs)
            assert _err(hyp, mh[i], vh[i], mu_r, var_r) < TOL, (ksplit, wu, k, i)
        np.testing.assert_array_equal(vmax.cpu().numpy(), vh.max(axis=1))
    for m in models:
        assert m.stats()["lattice"] == 2, m.stats()
    # the factor the steps leave behind (the next V-stream step's L21 comes from V)
    ctx.set_lattice(False)
    for k in (3,):
        Xn = np.concatenate([X[n:n + k] for X, _, _, n in data])
        yn = np.concatenate([y[n:n + k] for _, y, _, n in data])
        _lib.batch_append_predict(models, Xn.ctypes.data, yn.ctypes.data, [k, k], mu.data_ptr(), var.data_ptr())
        data = [(X, y, nl, n + k) for X, y, nl, n in data]
        mh, vh = mu.cpu().numpy().reshape(2, M), var.cpu().numpy().reshape(2, M)
        for i, (X, y, nl, n) in enumerate(data):
            mu_r, var_r = _ref(hyp, X[:n], y[:n], nl, Xs)
            assert _err(hyp, mh[i], vh[i], mu_r, var_r) < TOL, (ksplit, wu, "vstream", i)


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_lattice_gemm2_equals_in_launch_split4(monkeypatch, dtype):
    """The step's GEMM and cells as a second launch (k_lat_gemm2, the default where its
    tiles fill the chip once or twice, forced here with MFGP_LAT_GEMM2=1: four
    K splits inside one 1024-thread workgroup, their sums meeting in LDS) against
    the one-launch form with split-K 4 through memory (MFGP_LAT_GEMM2=0,
    MFGP_LAT_KSPLIT=4): the same stages per split and the same order of the
    splits' sums, so the same bits -- mean, variance, fused max / argmax -- over
    ragged batches (1 and 3 GPs) with off-lattice training rows (the virtual
    stages), appends of 8, 3 and 12 rows (KA = 8 and 16), and the default form
    against the oracle at every cell."""
    import torch
    from mfgp_coverage_amd import _lib
    hyp = _hyp("australia8_mf")
    G = 64
    dt = _lib.F32 if dtype == "f32" else _lib.F64

    def run(ctx, B, check_oracle):
        models, data = [], []
        for i in range(B):
            nl, nh = 120 + 13 * i, 160 - 7 * i
            Xs, X, y = _data(G, nl + nh + 40, seed=90 + i)
            X[5:9] += 0.31 / (G - 1)   # off-lattice lofi rows: virtual K rows
            models.append(_model(ctx, hyp, X[:nl + nh], y[:nl + nh], nl, Xs, dtype=dt))
            data.append((X, y, nl, nl + nh))
        M = Xs.shape[0]
        mu = torch.empty(B * M, dtype=torch.float64, device="cuda")
        var = torch.empty_like(mu)
        vmax = torch.empty(B, dtype=torch.float64, device="cuda")
        vam = torch.empty(B, dtype=torch.int64, device="cuda")
        _lib.batch_predict(models, mu.data_ptr(), var.data_ptr())
        out = []
        for k in (8, 3, 12):
            Xn = np.concatenate([X[n:n + k] for X, _, _, n in data])
            yn = np.concatenate([y[n:n + k] for _, y, _, n in data])
            Xt = torch.from_numpy(np.ascontiguousarray(Xn)).cuda()
            yt = torch.from_numpy(np.ascontiguousarray(yn)).cuda()
            _lib.batch_append_predict(models, Xt.data_ptr(), yt.data_ptr(), [k] * B, mu.data_ptr(), var.data_ptr(),
                                      vmax_ptr=vmax.data_ptr(), vargmax_ptr=vam.data_ptr())
            data = [(X, y, nl, n + k) for X, y, nl, n in data]
            out.append((mu.cpu().numpy(), var.cpu().numpy(), vmax.cpu().numpy(), vam.cpu().numpy()))
        assert all(m.stats()["lattice"] == 3 for m in models), [m.stats() for m in models]
        assert all(m.stats()["lattice_g2"] == (3 if check_oracle else 0) for m in models), [m.stats() for m in models]
        if check_oracle:
            mu_h, var_h = out[-1][0].reshape(B, M), out[-1][1].reshape(B, M)
            for i, (X, y, nl, n) in enumerate(data):
                mu_r, var_r = _ref(hyp, X[:n], y[:n], nl, Xs)
                if dtype == "f64":
                    assert _err(hyp, mu_h[i], var_h[i], mu_r, var_r) < TOL, i
                else:
                    e = O.parity_errors_f32(mu_h[i], var_h[i], mu_r, var_r, O.prior_variance(hyp))
                    assert max(e) < O.F32_TOL, (i, e)
                assert np.isclose(out[-1][2][i], var_h[i].max()) and out[-1][3][i] == int(np.argmax(var_h[i]))
        ctx.synchronize()
        return out

    for B in (1, 3):
        monkeypatch.setenv("MFGP_LAT_GEMM2", "0")
        monkeypatch.setenv("MFGP_LAT_KSPLIT", "4")
        a = _lib.Context(0)
        monkeypatch.setenv("MFGP_LAT_GEMM2", "1")   # (these batches are below the chip's size)
        monkeypatch.delenv("MFGP_LAT_KSPLIT")
        b = _lib.Context(0)
        monkeypatch.delenv("MFGP_LAT_GEMM2")
        a.set_lattice("force")
        b.set_lattice("force")
        ra, rb = run(a, B, False), run(b, B, True)
        for sa, sb in zip(ra, rb):
            for xa, xb in zip(sa, sb):
                assert np.array_equal(xa, xb), B


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_lattice_zcsr_equals_zunits(monkeypatch, dtype):
    """Z units reading the scan units' member lists (MFGP_LAT_ZCSR=1, the default
    where each Z unit would bucket many rows: configs[4]) against Z units that bucket
    the rows themselves (MFGP_LAT_ZCSR=0): the same members in the same row order,
    the same FMAs, so the same bits -- mean, variance, fused max / argmax -- over
    ragged batches with off-lattice rows (virtual Z rows, their padding) and appends
    of 8, 3 and 12 rows (KA = 8 and 16), both GEMM forms."""
    import torch
    from mfgp_coverage_amd import _lib
    hyp = _hyp("australia8_mf")
    G = 64
    dt = _lib.F32 if dtype == "f32" else _lib.F64

    def run(ctx, B):
        models, data = [], []
        for i in range(B):
            nl, nh = 200 + 11 * i, 260 - 5 * i
            Xs, X, y = _data(G, nl + nh + 40, seed=290 + i)
            X[7:12] += 0.27 / (G - 1)   # off-lattice lofi rows
            X[nl + 2] += 0.31 / (G - 1)   # and a hifi one
            models.append(_model(ctx, hyp, X[:nl + nh], y[:nl + nh], nl, Xs, dtype=dt))
            data.append((X, y, nl, nl + nh))
        M = Xs.shape[0]
        mu = torch.empty(B * M, dtype=torch.float64, device="cuda")
        var = torch.empty_like(mu)
        vmax = torch.empty(B, dtype=torch.float64, device="cuda")
        vam = torch.empty(B, dtype=torch.int64, device="cuda")
        _lib.batch_predict(models, mu.data_ptr(), var.data_ptr())
        out = []
        for k in (8, 3, 12):
            Xn = np.concatenate([X[n:n + k] for X, _, _, n in data])
            yn = np.concatenate([y[n:n + k] for _, y, _, n in data])
            Xt = torch.from_numpy(np.ascontiguousarray(Xn)).cuda()
            yt = torch.from_numpy(np.ascontiguousarray(yn)).cuda()
            _lib.batch_append_predict(models, Xt.data_ptr(), yt.data_ptr(), [k] * B, mu.data_ptr(), var.data_ptr(),
                                      vmax_ptr=vmax.data_ptr(), vargmax_ptr=vam.data_ptr())
            data = [(X, y, nl, n + k) for X, y, nl, n in data]
            out.append((mu.cpu().numpy(), var.cpu().numpy(), vmax.cpu().numpy(), vam.cpu().numpy()))
        assert all(m.stats()["lattice"] == 3 for m in models), [m.stats() for m in models]
        assert all(m.stats()["lattice_virtual"] > 0 for m in models), [m.stats() for m in models]
        ctx.synchronize()
        return out

    for B, g2 in ((1, "0"), (3, "0"), (3, "1")):
        monkeypatch.setenv("MFGP_LAT_GEMM2", g2)
        monkeypatch.setenv("MFGP_LAT_ZCSR", "0")
        a = _lib.Context(0)
        monkeypatch.setenv("MFGP_LAT_ZCSR", "1")
        b = _lib.Context(0)
        monkeypatch.delenv("MFGP_LAT_ZCSR")
        monkeypatch.delenv("MFGP_LAT_GEMM2")
        a.set_lattice("force")
        b.set_lattice("force")
        ra, rb = run(a, B), run(b, B)
        for step, (sa, sb) in enumerate(zip(ra, rb)):
            for xa, xb in zip(sa, sb):
                assert np.array_equal(xa, xb), (B, g2, step)


def test_concurrent_contexts_equal_sequential():
    """Two contexts in concurrent mode (mfgp_ctx_set_concurrent: several streams on one
    GPU) step independent lattice batches at the same time -- default gates, member
    lists (lat_zcsr), the GEMM as its own launch -- and must give the bits of the same
    batches stepped one after the other (the dispatch-order argument of the
    hand-offs, every waiter behind the roles it waits on, must hold when another
    context's launch shares the chip; a wait on a later workgroup would hang here,
    bounded, and report MFGP_ERR_DEVICE)."""
    import torch
    from mfgp_coverage_amd import _lib
    hyp = _hyp("australia8_mf")
    G, NL, NH, B, steps, k = 128, 700, 600, 4, 3, 8

    def setup(ctx, seed0):
        ctx.set_concurrent(True)
        ctx.set_lattice("force")
        models, data = [], []
        for i in range(B):
            Xs, X, y = _data(G, NL + NH + steps * k, seed=seed0 + i)
            models.append(_model(ctx, hyp, X[:NL + NH], y[:NL + NH], NL, Xs))
            data.append((X, y))
        M = G * G
        mu = torch.empty(B * M, dtype=torch.float64, device="cuda")
        var = torch.empty_like(mu)
        _lib.batch_predict(models, mu.data_ptr(), var.data_ptr())
        ctx.synchronize()
        pts = []
        for s in range(steps):
            lo = NL + NH + s * k
            Xn = np.ascontiguousarray(np.vstack([X[lo:lo + k] for X, _ in data]))
            yn = np.ascontiguousarray(np.concatenate([y[lo:lo + k] for _, y in data]))
            pts.append((torch.from_numpy(Xn).cuda(), torch.from_numpy(yn).cuda()))
        return models, mu, var, pts

    def step(models, mu, var, pts, s):
        Xd, yd = pts[s]
        _lib.batch_append_predict(models, Xd.data_ptr(), yd.data_ptr(), [k] * B, mu.data_ptr(), var.data_ptr(),
                                  asynchronous=True)

    # sequential
    seq = []
    for seed0 in (510, 520):
        ctx = _lib.Context(0)
        models, mu, var, pts = setup(ctx, seed0)
        outs = []
        for s in range(steps):
            step(models, mu, var, pts, s)
            ctx.synchronize()
            outs.append((mu.cpu().numpy(), var.cpu().numpy()))
        seq.append(outs)
        assert all(m.stats()["lattice"] == steps for m in models)
    # concurrent: both contexts' steps enqueued before either is waited for
    ca, cb = _lib.Context(0), _lib.Context(0)
    A, Bm = setup(ca, 510), setup(cb, 520)
    conc = [[], []]
    for s in range(steps):
        step(*A, s)
        step(*Bm, s)
        ca.synchronize()
        cb.synchronize()
        conc[0].append((A[1].cpu().numpy(), A[2].cpu().numpy()))
        conc[1].append((Bm[1].cpu().numpy(), Bm[2].cpu().numpy()))
    for which in (0, 1):
        for s in range(steps):
            for xa, xb in zip(seq[which][s], conc[which][s]):
                assert np.array_equal(xa, xb), (which, s)
    for m in A[0] + Bm[0]:
        assert m.stats()["lattice"] == steps
