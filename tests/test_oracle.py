"""Pin the CPU oracle (oracle/gp_oracle.py) against the reference (no GPU).

* golden vectors produced by the reference's own gaussian_process.py
  (tests/golden/make_golden.py, anti_two_corners, SF + MF, 51x51 and 32x32);
* the reference's own logged runs (Data/*_agent.csv VarMax, Var0);
* closed forms (empty GP, single observation).
"""
import numpy as np
import pytest

from oracle import gp_oracle as O
from tests import _fixtures as F


@pytest.fixture(scope="module")
def atc():
    return F.atc()


@pytest.mark.parametrize("grid", F.GRIDS)
@pytest.mark.parametrize("N", F.NS)
def test_sf_oracle_vs_reference(atc, grid, N):
    X, y = atc["train"][:N, :2], atc["train"][:N, 2]
    Xs = atc[f"grid_{grid}"]
    key = f"sf_{grid}_n{N}"
    mu_f, var_f = O.sf_faithful(X, y, atc["hyp_sf"], Xs)
    np.testing.assert_allclose(mu_f, atc[key + "_mu"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(var_f, atc[key + "_var"], rtol=1e-10, atol=1e-20)
    mu_d, var_d = O.sf_diag(X, y, atc["hyp_sf"], Xs)
    e_mu, e_var = O.parity_errors(mu_d, var_d, atc[key + "_mu"], atc[key + "_var"], O.prior_variance(atc["hyp_sf"]))
    assert e_mu < O.PARITY_TOL and e_var < O.PARITY_TOL, (e_mu, e_var)


@pytest.mark.parametrize("grid", F.GRIDS)
@pytest.mark.parametrize("N", F.NS)
def test_mf_oracle_vs_reference(atc, grid, N):
    P = atc["prior"]
    X, y = atc["train"][:N, :2], atc["train"][:N, 2]
    Xs = atc[f"grid_{grid}"]
    key = f"mf_{grid}_n{N}"
    mu_f, var_f = O.mf_faithful(P[:, :2], P[:, 2], X, y, atc["hyp_mf"], Xs)
    np.testing.assert_allclose(mu_f, atc[key + "_mu"], rtol=1e-12, atol=0)
    np.testing.assert_allclose(var_f, atc[key + "_var"], rtol=1e-10, atol=1e-20)
    mu_d, var_d = O.mf_diag(P[:, :2], P[:, 2], X, y, atc["hyp_mf"], Xs)
    e_mu, e_var = O.parity_errors(mu_d, var_d, atc[key + "_mu"], atc[key + "_var"], O.prior_variance(atc["hyp_mf"]))
    assert e_mu < O.PARITY_TOL and e_var < O.PARITY_TOL, (e_mu, e_var)


@pytest.mark.parametrize("grid", F.GRIDS)
def test_empty_gp_closed_form(atc, grid):
    Xs = atc[f"grid_{grid}"]
    e = np.empty((0, 2))
    for hyp, key in ((atc["hyp_sf"], f"sf_{grid}_n0"), (atc["hyp_mf"], f"mfempty_{grid}")):
        mu, var = (O.sf_diag(e, e[:, 0], hyp, Xs) if hyp.shape[0] == 4
                   else O.mf_diag(e, e[:, 0], e, e[:, 0], hyp, Xs))
        assert np.all(mu == O.prior_mean(hyp)) and np.all(var == O.prior_variance(hyp))
        np.testing.assert_allclose(mu, atc[key + "_mu"], rtol=1e-15)
        np.testing.assert_allclose(var, atc[key + "_var"], rtol=1e-15)


def test_single_observation_closed_form(atc):
    hyp = atc["hyp_sf"]
    x0 = np.array([[0.3, 0.7]])
    s = np.exp(hyp[1])
    _, var = O.sf_diag(x0, np.array([0.5]), hyp, x0)
    expect = s - s * s / (s + np.exp(hyp[3]) + O.JITTER)
    np.testing.assert_allclose(var[0], expect, rtol=1e-6)


def test_append_sequence_oracle(atc):
    P, T = atc["prior"], atc["train"]
    Xs = atc["grid_g51"]
    pos = 0
    for s, k in enumerate(atc["seq_chunks"]):
        pos += int(k)
        X = np.vstack([P[:, :2], T[:pos, :2]])
        y = np.concatenate([P[:, 2], T[:pos, 2]])
        mu, var = O.sf_diag(X, y, atc["hyp_sf"], Xs)
        e = O.parity_errors(mu, var, atc[f"sfseq_s{s}_mu"], atc[f"sfseq_s{s}_var"], O.prior_variance(atc["hyp_sf"]))
        assert max(e) < O.PARITY_TOL, e
        mu, var = O.mf_diag(P[:, :2], P[:, 2], T[:pos, :2], T[:pos, 2], atc["hyp_mf"], Xs)
        e = O.parity_errors(mu, var, atc[f"mfseq_s{s}_mu"], atc[f"mfseq_s{s}_var"], O.prior_variance(atc["hyp_mf"]))
        assert max(e) < O.PARITY_TOL, e


class _OracleModel:
    def __init__(self, hyp, prior, grid):
        self.hyp, self.grid = hyp, grid
        self.mf = hyp.shape[0] == 9
        e = np.empty((0, 2))
        self.XL = prior[:, :2] if (prior is not None and self.mf) else e
        self.yL = prior[:, 2] if (prior is not None and self.mf) else np.empty(0)
        self.X = prior[:, :2] if (prior is not None and not self.mf) else e
        self.y = prior[:, 2] if (prior is not None and not self.mf) else np.empty(0)

    def append(self, X, y):
        self.X = np.vstack([self.X, X])
        self.y = np.concatenate([self.y, y.reshape(-1)])

    def var(self):
        if self.mf:
            return O.mf_diag(self.XL, self.yL, self.X, self.y, self.hyp, self.grid)[1]
        return O.sf_diag(self.X, self.y, self.hyp, self.grid)[1]


@pytest.mark.parametrize("run", F.REPLAY_RUNS)
def test_oracle_replays_logged_runs(run):
    fx = F.replay(run)
    for sim in fx["sims"]:
        np.testing.assert_allclose(O.prior_variance(fx["hyp"]), fx[f"s{sim}_var0"], rtol=1e-13)
        logged, got = F.replay_run(
            fx, sim,
            make_model=lambda hyp, prior: _OracleModel(hyp, prior, fx["grid"]),
            append=lambda m, X, y: m.append(X, y),
            predict_var=lambda m: m.var())
        np.testing.assert_allclose(got, logged, rtol=1e-9)


@pytest.mark.parametrize("case", ["sf_n50", "mf_n20", "mf_prior"])
def test_oracle_sample_points_vs_reference(case):
    """The oracle's compute_sample_points loop (simulator.py:326-374: argmax of the
    variance -> append with the posterior mean -> predict) reproduces the
    reference's own output (choi_reference.npz) up to the first near-tie argmax."""
    fx = F.load("choi_reference.npz")
    train, prior, xs = fx["train"], fx["prior"], fx["grid"]
    mf = case.startswith("mf")
    hyp = fx["hyp_mf"] if mf else fx["hyp_sf"]
    n = {"sf_n50": 50, "mf_n20": 20, "mf_prior": 0}[case]
    XL, yL = prior[:, :2], prior[:, 2]
    XH, yH = train[:n, :2].copy(), train[:n, 2].copy()

    def predict():
        if mf:
            return O.mf_diag(XL, yL, XH, yH, hyp, xs)
        return O.sf_diag(XH, yH, hyp, xs)

    thr = float(fx[case + "_threshold"])
    mu, var = predict()
    pts = []
    while var.max() > thr:
        j = int(np.argmax(var))
        pts.append(xs[j])
        XH = np.vstack([XH, xs[j:j + 1]])
        yH = np.concatenate([yH, mu[j:j + 1]])
        mu, var = predict()
    ref, gaps = fx[case + "_points"], fx[case + "_gaps"]
    near = np.flatnonzero(gaps < O.PARITY_TOL * O.prior_variance(hyp))
    upto = int(near[0]) if near.size else ref.shape[0]
    pts = np.asarray(pts).reshape(-1, 2)
    np.testing.assert_array_equal(pts[:upto], ref[:upto])
    if upto == ref.shape[0]:
        assert pts.shape[0] == ref.shape[0]


def _cells_case(fx, i):
    verts, vs = fx[f"c{i}_verts"], fx[f"c{i}_vstart"]
    polys = [verts[vs[j]:vs[j + 1]] for j in range(vs.shape[0] - 1)]
    return polys, fx[f"c{i}_seeds"]


def test_oracle_cell_reductions_vs_reference():
    """in_polygon / compute_loss / compute_centroids / compute_max_var (sim:105-323)
    restated on arrays reproduce the reference's outputs on 12 partitions."""
    fx = F.load("cells_reference.npz")
    truth, mu, var = fx["truth"], fx["mu"], fx["var"]
    xs = truth[:, :2]
    for i in range(int(fx["ncases"])):
        polys, seeds = _cells_case(fx, i)
        res = O.cell_reductions(polys, seeds, xs, w=mu, f=truth[:, 2], var=var)
        np.testing.assert_array_equal([r[0].sum() for r in res], fx[f"c{i}_counts"])
        lo, hi = xs.min(0), xs.max(0)
        cen = np.clip(np.array([r[1] for r in res]), lo, hi)
        np.testing.assert_allclose(cen, fx[f"c{i}_centroids"], rtol=1e-13, atol=1e-15)
        np.testing.assert_allclose(sum(r[2] for r in res), fx[f"c{i}_loss"], rtol=1e-13)
        np.testing.assert_array_equal(np.array([r[3] for r in res]), fx[f"c{i}_maxvar"][:, 0])
        np.testing.assert_array_equal(xs[[r[4] for r in res]], fx[f"c{i}_argmax"])


def _nlml_case(fx, c):
    h, n = fx[c + "_hyp"], int(fx[c + "_n"])
    X, y = fx["train"][:n, :2], fx["train"][:n, 2]
    if c.startswith("sf"):
        return (X, y, h), {}
    return (X, y, h), {"XL": fx["prior"][:, :2], "yL": fx["prior"][:, 2]}


def test_oracle_nlml_vs_reference():
    """likelihood (gp:81-106 / 344-385): the oracle's value equals the reference's, and
    its analytic gradient matches the reference's central finite differences
    (h = 1e-6; looser where K is nearly singular at the trained noise e^-37.8)."""
    fx = F.load("nlml_reference.npz")
    for c in (str(v) for v in fx["cases"]):
        args, kw = _nlml_case(fx, c)
        v, g = O.nlml(*args, grad=True, **kw)
        np.testing.assert_allclose(v, fx[c + "_nlml"], rtol=1e-12)
        fd = fx[c + "_fdgrad"]
        tol = 1e-3 if c.endswith("h0") else 1e-5
        assert np.all(np.abs(g - fd) <= tol * np.maximum(np.abs(fd), 1.0)), (c, g, fd)


def test_parity_errors_f32_degenerate_reference():
    """parity_errors_f32 stays finite for an all-zero reference mean (the 1 % floor
    is then 0; the 1e-300 floor keeps the metric defined) and is an absolute bound
    of 1e-2 * max|mu_ref| below that floor."""
    z = np.zeros(5)
    e = O.parity_errors_f32(z, np.full(5, 0.1), z, np.full(5, 0.1), 0.1)
    assert np.isfinite(e).all() and e == (0.0, 0.0)
    ref = np.array([1.0, 1e-6, -0.5])
    got = ref + np.array([0.0, 1e-6, 0.0])            # |d| = 1e-6 where |ref| is below the 1e-2 floor
    e_mu, _ = O.parity_errors_f32(got, np.ones(3), ref, np.ones(3), 1.0)
    assert abs(e_mu - 1e-6 / 1e-2) < 1e-12
