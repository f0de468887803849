"""likelihood / train (gaussian_process.py:81-119, 344-399) on the device
(mfgp_nlml through SFGP/MFGP.likelihood[_and_grad]) against the reference's own
NLML values and finite-difference gradients (tests/golden/nlml_reference.npz)
and the oracle's analytic gradient."""
import numpy as np
import pytest

from oracle import gp_oracle as O
from tests import _fixtures as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nl():
    return F.load("nlml_reference.npz")


def _mirror(gp, fx, c):
    n = int(fx[c + "_n"])
    X, y = fx["train"][:n, :2].copy(), fx["train"][:n, 2:3].copy()
    if c.startswith("sf"):
        return gp.SFGP(X, y, 1)
    return gp.MFGP(fx["prior"][:, :2].copy(), fx["prior"][:, 2:3].copy(), X, y, 1, 1)


@pytest.mark.parametrize("c", ["sf_n50_h0", "sf_n50_h1", "sf_n130_h0", "sf_n130_h1",
                               "mf_n30_h0", "mf_n30_h1", "mf_n90_h0", "mf_n90_h1"])
def test_nlml_vs_reference(nl, c):
    from mfgp_coverage_amd import gaussian_process as gp
    m = _mirror(gp, nl, c)
    h = nl[c + "_hyp"]
    v = m.likelihood(h)
    np.testing.assert_allclose(v, nl[c + "_nlml"], rtol=O.PARITY_TOL)
    v2, g = m.likelihood_and_grad(h)
    assert v2 == v
    n = int(nl[c + "_n"])
    X, y = nl["train"][:n, :2], nl["train"][:n, 2]
    kw = {} if c.startswith("sf") else {"XL": nl["prior"][:, :2], "yL": nl["prior"][:, 2]}
    _, go = O.nlml(X, y, h, grad=True, **kw)
    fd = nl[c + "_fdgrad"]
    well = c.endswith("h1")      # h0: the trained noise (e^-37.8 SF) leaves K nearly singular
    assert np.all(np.abs(g - go) <= (1e-8 if well else 1e-3) * np.maximum(np.abs(go), 1.0)), (g, go)
    assert np.all(np.abs(g - fd) <= (1e-5 if well else 1e-3) * np.maximum(np.abs(fd), 1.0)), (g, fd)


@pytest.mark.parametrize("kind,N,NL", [("sf", 257, 0), ("mf", 700, 300), ("mf", 1200, 1000)])
def test_nlml_larger_vs_oracle(kind, N, NL):
    """Block boundaries (257) and sizes where the tiled inverse spans many blocks."""
    from mfgp_coverage_amd import _lib, synthetic
    rng = np.random.default_rng(N)
    wl = synthetic.Workload(48, NL, N - NL, 1, 1, seed=N)
    hyp = synthetic.HYP["australia9_mf"] if kind == "mf" else synthetic.HYP["australia3_sf"]
    m = _lib.Model(_lib.context(), _lib.MF if kind == "mf" else _lib.SF, hyp, 1e-8)
    if kind == "sf":
        m.set_data(np.empty((0, 2)), np.empty(0), wl.XH, wl.yH)
        vo, go = O.nlml(wl.XH, wl.yH, hyp, grad=True)
    else:
        m.set_data(wl.XL, wl.yL, wl.XH, wl.yH)
        vo, go = O.nlml(wl.XH, wl.yH, hyp, XL=wl.XL, yL=wl.yL, grad=True)
    h2 = hyp + 0.05 * rng.standard_normal(hyp.shape[0])
    v, g = m.nlml(hyp, grad=True)
    np.testing.assert_allclose(v, vo, rtol=1e-10)
    assert np.all(np.abs(g - go) <= 1e-7 * np.maximum(np.abs(go), 1.0)), (g, go)
    # other hyperparameters than the model's own: the model is unchanged
    kw = {} if kind == "sf" else {"XL": wl.XL, "yL": wl.yL}
    v2, g2 = m.nlml(h2, grad=True)
    vo2, go2 = O.nlml(wl.XH, wl.yH, h2, grad=True, **kw)
    np.testing.assert_allclose(v2, vo2, rtol=1e-10)
    assert np.all(np.abs(g2 - go2) <= 1e-7 * np.maximum(np.abs(go2), 1.0))
    np.testing.assert_allclose(m.nlml(hyp), v, rtol=0)


def test_train_lowers_nlml():
    """train (gp:108-119): L-BFGS-B with the device gradient improves the fit."""
    from mfgp_coverage_amd import gaussian_process as gp, synthetic
    wl = synthetic.Workload(32, 0, 150, 1, 1, seed=1)
    m = gp.SFGP(wl.XH.copy(), wl.yH.reshape(-1, 1).copy(), 0.3)
    before = m.likelihood(m.hyp)
    m.train()
    after = m.likelihood(m.hyp)
    assert after < before - 1.0
    # the oracle agrees on the trained point
    np.testing.assert_allclose(after, O.nlml(wl.XH, wl.yH, m.hyp), rtol=1e-8)
