"""The drop-in boundary without a GPU: the C-ABI library loads and exports every
symbol include/mfgp_hip.h declares, the Python mirror has the reference's
surface, DiagCov behaves like the dense covariance for the callers' uses, and
the product path refuses to run without a device (no CPU fallback)."""
import copy
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "mfgp_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mfgp_[a-z_0-9]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__ as ge
    ge.build()
    from mfgp_coverage_amd import _lib
    return _lib


def test_library_exports_every_declared_symbol(lib):
    syms = _header_symbols()
    assert len(syms) >= 20
    h = lib.lib()
    for s in syms:
        assert hasattr(h, s), s
        assert s in lib.SIGNATURES, s
    assert set(lib.SIGNATURES) == set(syms)
    assert b"gfx950" in h.mfgp_version()


def test_library_is_gfx950_code_object(lib):
    data = open(lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    for k in (b"k_predict", b"k_potrf_diag", b"k_panel", b"k_syrk", b"k_assemble"):
        assert k in data


def test_mirror_surface_without_device(lib):
    from mfgp_coverage_amd.gaussian_process import MFGP, SFGP
    e2, e1 = np.empty((0, 2)), np.empty((0, 1))
    sf = SFGP(e2, e1, 1)
    # gp:46-64 defaults
    np.testing.assert_array_equal(sf.hyp, [-4.0, 0.0, 0.0, -4.0])
    assert sf.D == 2 and sf.jitter == 1e-8 and list(sf.idx_theta) == [0, 1, 2]
    mf = MFGP(e2, e1, e2, e1, 1, 1)
    np.testing.assert_array_equal(mf.hyp, [0, 1, 0, 0, 1, 0, -1, 0, 0])   # gp:300-327
    assert list(mf.idx_theta_L) == [0, 1, 2] and list(mf.idx_theta_H) == [3, 4, 5]
    for name in ("updt_info", "updt", "predict"):
        assert callable(getattr(sf, name))
    for name in ("updt_info", "updt_hifi", "predict"):
        assert callable(getattr(mf, name))
    c = copy.deepcopy(sf)   # no device state yet: plain copy
    assert isinstance(c, SFGP) and c is not sf


def test_no_cpu_fallback(lib):
    from mfgp_coverage_amd.gaussian_process import SFGP
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    m = SFGP(np.zeros((1, 2)), np.zeros((1, 1)), 1)
    with pytest.raises(RuntimeError, match="libmfgp_hip"):
        m.predict(np.zeros((4, 2)))


@pytest.mark.gpu
def test_inplace_grid_edit_is_seen(lib):
    """The simulator passes the same x_star array to every predict (sim:671, 884);
    an in-place edit of ONE cell of that same array, anywhere, must move the
    next predict to the edited grid (gp:139 evaluates the kernel on X_star as it
    is at the call) -- and back when the edit is undone."""
    from oracle import gp_oracle as O
    from mfgp_coverage_amd.gaussian_process import SFGP
    from mfgp_coverage_amd.synthetic import HYP, grid
    hyp = HYP["australia3_sf"]
    xs = grid(64)
    rng = np.random.default_rng(4)
    X = xs[rng.choice(xs.shape[0], 150, replace=False)]
    y = rng.standard_normal((150, 1))
    m = SFGP(X.copy(), y.copy(), 1)
    m.hyp = hyp.copy()
    m.updt_info(m.X, m.y)
    mu0, cov0 = m.predict(xs)
    for cell in (1237, 4095, 0):   # cells no strided sample of the array would hit first
        old = xs[cell].copy()
        xs[cell] = (0.123456789, 0.987654321)   # the same array object, edited in place
        mu, cov = m.predict(xs)
        mu_r, var_r = O.sf_diag(X, y, hyp, xs)
        assert max(O.parity_errors(mu[:, 0], np.diag(cov), mu_r, var_r, O.prior_variance(hyp))) < O.PARITY_TOL
        assert mu[cell, 0] != mu0[cell, 0]
        xs[cell] = old
        mu, cov = m.predict(xs)
        np.testing.assert_array_equal(mu, mu0)
        np.testing.assert_array_equal(np.diag(cov), np.diag(cov0))
    # an append between predicts (the simulator's step) still sees an edit
    m.updt(xs[5:7], np.zeros((2, 1)))
    xs[77] = (0.5, 0.55555)
    mu, cov = m.predict(xs)
    mu_r, var_r = O.sf_diag(np.vstack([X, grid(64)[5:7]]), np.vstack([y, np.zeros((2, 1))]), hyp, xs)
    assert max(O.parity_errors(mu[:, 0], np.diag(cov), mu_r, var_r, O.prior_variance(hyp))) < O.PARITY_TOL


def test_diagcov_semantics():
    from mfgp_coverage_amd.gaussian_process import DiagCov
    v = np.array([0.1, 0.5, 0.2])
    c = DiagCov(v)
    np.testing.assert_array_equal(np.diag(c), v)                # simulator.py:301, 341, 685, 855
    assert np.amax(c) == 0.5                                    # simulator.py:672, 842, 1014
    assert np.argmax(c) == 1 * 3 + 1
    assert c.shape == (3, 3) and c[1, 1] == 0.5
    with pytest.raises(TypeError):
        np.asarray(c)
    d = np.diag(c)                                              # as np.diag of a 2-D array: a
    assert not d.flags.writeable and np.shares_memory(d, c.var)  # read-only view, no copy
    f = DiagCov(v, fused=(np.float64(0.5), 1))                  # the launch's fused max / argmax
    assert np.amax(f) == 0.5 and np.argmax(f) == 4 and np.max(f, axis=None) == 0.5
    one = DiagCov(np.array([0.25]))                             # get_neg_var's 1x1 (gp:556-557)
    assert float(2.0 * one[0, 0]) == 0.5
    np.testing.assert_array_equal(np.asarray(one), [[0.25]])
    assert (np.array([[1.0]]) + 2.0 * one)[0, 0] == 1.5


@pytest.mark.gpu
def test_predict_arrays_are_the_callers(lib):
    """predict() returns the model's pinned result buffer itself (mfgp_predict_view,
    no host copy). Each call's arrays are the caller's: a later predict, append or
    in-place edit of one call's arrays changes no other call's; dropped arrays
    return their buffer to the pool and a model keeps working across many calls."""
    import gc
    from mfgp_coverage_amd.gaussian_process import MFGP
    from mfgp_coverage_amd.synthetic import HYP, grid
    hyp = HYP["australia8_mf"]
    xs = grid(48)
    rng = np.random.default_rng(5)
    X = xs[rng.choice(xs.shape[0], 200, replace=False)]
    y = rng.standard_normal((200, 1))
    m = MFGP(X[:80], y[:80], X[80:150], y[80:150], 1, 1)
    m.hyp = hyp.copy()
    m.updt_info(m.X_L, m.y_L, m.X_H, m.y_H)
    mu0, cov0 = m.predict(xs)
    keep_mu, keep_var = mu0.copy(), np.diag(cov0).copy()
    assert mu0.flags.writeable and mu0.dtype == np.float64 and mu0.shape == (xs.shape[0], 1)
    mu1, cov1 = m.predict(xs)   # an unchanged model: the same bits, another buffer
    np.testing.assert_array_equal(mu1, mu0)
    np.testing.assert_array_equal(np.diag(cov1), np.diag(cov0))
    mu1[:] = -1.0               # the caller's own array
    mu2, _ = m.predict(xs)
    np.testing.assert_array_equal(mu2, keep_mu)
    for s in range(12):         # the drop-in step, arrays dropped as the simulator does
        m.updt_hifi(X[150 + 4 * s:154 + 4 * s], y[150 + 4 * s:154 + 4 * s])
        mu, cov = m.predict(xs)
        del mu, cov
        gc.collect()
    np.testing.assert_array_equal(mu0, keep_mu.reshape(-1, 1))   # untouched by later steps
    np.testing.assert_array_equal(np.diag(cov0), keep_var)
    # the drop-in step's consumers (sim:301, 672 / 842 / 1014): after an append the
    # covariance carries its launch's fused max / argmax, equal to the host scan's
    for s in range(3):
        m.updt_hifi(X[190 + 2 * s:192 + 2 * s], y[190 + 2 * s:192 + 2 * s])
        mu, cov = m.predict(xs)
        v = np.diag(cov)
        assert cov.fused is not None
        assert np.amax(cov) == v.max() and np.argmax(cov) == int(np.argmax(v)) * (xs.shape[0] + 1)
        assert not v.flags.writeable and np.shares_memory(v, cov.var)
    mu, cov = m.predict(xs)            # the same model again (no append: a host max)
    assert np.amax(cov) == np.diag(cov).max()
