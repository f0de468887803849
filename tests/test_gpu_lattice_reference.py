"""The lattice-separable step (k_inc_lat) on the reference's
own data: its logged runs, its off-lattice priors, revisited cells, and a horizon
long enough to cross the lattice depth limit (LAT_MAXD = 256 consecutive steps,
then one V-stream step that refreshes the resident posterior).

* Replays of Data/<run>_sample.csv through the drop-in SFGP / MFGP API with the
  lattice step forced (the library's cost gate keeps one GP per process on the V
  stream), checked against the logged per-iteration VarMax (simulator.py:925) and,
  at the last iteration, against the oracle at every cell. The australia runs have
  revisited cells (australia4_todescato_hsf: 40 samples at 13 cells) and priors
  partly off the grid's lattice (australia2: 17 of 81 rows, australia4: 11 of 36);
  the anti_two_corners runs must be refused by the conditioning gate.
* The reference's off-lattice priors (Data/australia{3,9}_prior.csv: 21 of 121 and
  11 of 36 rows 1 ulp off the grid's axis values) as SF data / MF lofi rows, with
  Todescato-style appends that revisit cells; the device's own count of the
  off-lattice rows it ran (the Z units' lidx = -1 rows) is asserted.
* The headline size (128x128, australia8 MF) growing for 300 steps of 8 rows, a
  third of them revisits, across the depth limit: steps 256 (deepest lattice
  step), 257 (the V-stream refresh), 258 and 300 against the oracle.
"""
import numpy as np
import pytest

from oracle import gp_oracle as O
from tests import _fixtures as F

pytestmark = pytest.mark.gpu

TOL = O.PARITY_TOL
RMAX = 1e4   # mfgp_capi.hip LAT_RMAX: the conditioning gate
MAXD = 256   # mfgp_capi.hip LAT_MAXD


@pytest.fixture(scope="module", autouse=True)
def lattice_forced():
    from mfgp_coverage_amd import _lib
    _lib.context().set_lattice("force")
    yield
    _lib.context().set_lattice(True)


def _gate_ok(hyp):
    """The host's conditioning gate (mfgp_capi.hip lat_cond_ok)."""
    h = np.asarray(hyp)
    if h.shape[0] == 4:
        noise = np.exp(h[3])
    else:
        noise = min(np.exp(h[7]), np.exp(h[8]))
    return O.prior_variance(h) / (noise + O.JITTER) <= RMAX


def _off_lattice(X, grid):
    ax, ay = np.unique(grid[:, 0]), np.unique(grid[:, 1])
    return int(np.sum(~(np.isin(X[:, 0], ax) & np.isin(X[:, 1], ay))))


@pytest.mark.parametrize("run", F.REPLAY_RUNS)
def test_lattice_replays_logged_runs(run):
    from mfgp_coverage_amd import gaussian_process as G
    from tests.test_gpu_parity import _replay_append, _replay_model
    fx = F.replay(run)
    grid = fx["grid"]
    hyp = fx["hyp"]
    prior = fx.get("prior")
    for sim in fx["sims"]:
        models = []

        def make(h, p):
            m = _replay_model(G, h, p)
            models.append(m)
            return m

        logged, got = F.replay_run(fx, sim, make_model=make, append=lambda m, X, y: _replay_append(G, m, X, y),
                                   predict_var=lambda m: np.diag(m.predict(grid)[1]))
        np.testing.assert_allclose(got, logged, rtol=TOL)
        m = models[0]
        # the last posterior at every cell against the oracle
        mu, cov = m.predict(grid)
        if hyp.shape[0] == 4:
            mu_r, var_r = O.sf_diag(m.X, m.y, hyp, grid)
        else:
            mu_r, var_r = O.mf_diag(m.X_L, m.y_L, m.X_H, m.y_H, hyp, grid)
        assert max(O.parity_errors(mu[:, 0], np.diag(cov), mu_r, var_r, O.prior_variance(hyp))) < TOL
        st = m._dev().stats()
        ks = np.array([np.sum(fx[f"s{sim}_sample_iter"] == it) for it in fx[f"s{sim}_iters"]])
        # an append of >= 1 row is a lattice step once a predict has run on >= 1
        # training row before it (the resident posterior of its old rows)
        rows = (prior.shape[0] if prior is not None else 0) + np.cumsum(ks)
        eligible = int(np.sum((ks[1:] > 0) & (rows[:-1] >= 1)))
        if _gate_ok(hyp):
            assert st["lattice"] == eligible > 0, (st, ks)
            X_all = m.X if hyp.shape[0] == 4 else np.vstack([m.X_L, m.X_H])
            off = _off_lattice(X_all, grid)
            assert off == (_off_lattice(prior[:, :2], grid) if prior is not None else 0)
            assert st["lattice_virtual"] == off, (st, off)
        else:
            assert st["lattice"] == 0, st   # anti_two_corners: refused, the V stream ran
            assert st["vstream"] >= eligible, st


@pytest.mark.parametrize("name,kind", [("australia3", "sf"), ("australia3", "mf"), ("australia9", "mf")])
def test_lattice_offlattice_prior_with_revisits(name, kind):
    """The reference's priors with rows 1 ulp off the lattice: SF data (simulator.py:
    87-95) or MF lofi rows (sim:59-63); 4 agents per step, a third of the samples at
    cells sampled before; oracle parity at every cell after every step."""
    from mfgp_coverage_amd import gaussian_process as G
    fx = F.load("priors_offlattice.npz")
    P, grid = fx[name + "_prior"], fx[name + "_grid"]
    hyp = fx[f"{name}_hyp_{kind}"]
    assert _gate_ok(hyp)
    off = _off_lattice(P[:, :2], grid)
    assert off > 0
    rng = np.random.default_rng(len(name) + len(kind))
    M, k, steps = grid.shape[0], 4, 24
    truth = np.exp(-np.sum((grid - 0.4) ** 2, 1) / 0.05)
    e2, e1 = np.empty((0, 2)), np.empty((0, 1))
    if kind == "sf":
        m = G.SFGP(P[:, :2].copy(), P[:, 2:3].copy(), 1)
    else:
        m = G.MFGP(P[:, :2].copy(), P[:, 2:3].copy(), e2, e1, 1, 1)
    m.hyp = hyp.copy()
    if kind == "sf":
        m.updt_info(m.X, m.y)
    else:
        m.updt_info(m.X_L, m.y_L, m.X_H, m.y_H)
    m.predict(grid)
    cells = []
    for s in range(steps):
        idx = rng.choice(M, k, replace=False)
        if cells:
            idx[: k // 3 + 1] = rng.choice(np.array(cells), k // 3 + 1)   # revisits
        cells.extend(idx.tolist())
        Xn, yn = grid[idx].copy(), (truth[idx] + 0.1 * rng.standard_normal(k)).reshape(-1, 1)
        (m.updt if kind == "sf" else m.updt_hifi)(Xn, yn)
        mu, cov = m.predict(grid)
        if kind == "sf":
            mu_r, var_r = O.sf_diag(m.X, m.y, hyp, grid)
        else:
            mu_r, var_r = O.mf_diag(m.X_L, m.y_L, m.X_H, m.y_H, hyp, grid)
        e = O.parity_errors(mu[:, 0], np.diag(cov), mu_r, var_r, O.prior_variance(hyp))
        assert max(e) < TOL, (s, e)
    assert len(set(cells)) < len(cells)
    st = m._dev().stats()
    assert st["lattice"] == steps and st["lattice_virtual"] == off, (st, off)


def test_lattice_depth_refresh_headline_revisits():
    """300 steps of the simulator's pattern at the headline size (2 GPs through the
    batched ABI, 8 rows per step, a third of them revisits): steps 1..256 are
    lattice steps (each from the previous step's posterior), step 257 refreshes
    the posterior from V on the V stream, steps 258.. are lattice steps again."""
    import torch
    from mfgp_coverage_amd import _lib
    from mfgp_coverage_amd.synthetic import HYP, Workload
    hyp = HYP["australia8_mf"]
    B, K, NL0, STEPS = 2, 8, 1024, 300
    wls = [Workload(128, NL0, 0, K, STEPS, seed=60 + i, revisit=1 / 3) for i in range(B)]
    xs = wls[0].xs
    M = xs.shape[0]
    models = []
    for w in wls:
        m = _lib.Model(_lib.context(), _lib.MF, hyp, 1e-8)
        m.set_grid(w.xs)
        m.set_data(w.XL, w.yL, np.empty((0, 2)), np.empty(0))
        models.append(m)
    mu = torch.empty(B * M, dtype=torch.float64, device="cuda")
    var = torch.empty(B * M, dtype=torch.float64, device="cuda")
    vmax = torch.empty(B, dtype=torch.float64, device="cuda")
    _lib.batch_predict(models, mu.data_ptr(), var.data_ptr())
    X = torch.from_numpy(np.ascontiguousarray(np.stack([w.Xnew for w in wls], 1))).cuda()   # [S, B, K, 2]
    Y = torch.from_numpy(np.ascontiguousarray(np.stack([w.ynew for w in wls], 1))).cuda()
    rng = np.random.default_rng(1)
    lat_prev, s_prev = 0, 0
    for s in range(1, STEPS + 1):
        _lib.batch_append_predict(models, X[s - 1].data_ptr(), Y[s - 1].data_ptr(), [K] * B, mu.data_ptr(),
                                  var.data_ptr(), asynchronous=True, vmax_ptr=vmax.data_ptr())
        if s in (MAXD - 1, MAXD, MAXD + 1, MAXD + 2, STEPS):
            lat = models[0].stats()["lattice"]   # synchronises (the virtual-row read-back)
            # step 257 (depth 256 reached) is the V-stream refresh, every other a lattice step
            expect = (s - s_prev) - (1 if s_prev < MAXD + 1 <= s else 0)
            assert lat - lat_prev == expect, (s, lat, lat_prev)
            lat_prev, s_prev = lat, s
        if s in (MAXD, MAXD + 1, MAXD + 2, STEPS):
            _lib.context().synchronize()
            mu_h, var_h = mu.cpu().numpy().reshape(B, M), var.cpu().numpy().reshape(B, M)
            np.testing.assert_array_equal(vmax.cpu().numpy(), var_h.max(axis=1))
            for i in ((0,) if s < STEPS else range(B)):
                w = wls[i]
                XH, yH = w.Xnew[:s].reshape(-1, 2), w.ynew[:s].reshape(-1)
                if s == STEPS and i == 0:
                    pick = np.arange(M)   # every cell once
                else:
                    pick = np.unique(np.concatenate([rng.choice(M, 4096, replace=False),
                                                     [int(np.argmax(var_h[i]))]]))
                mu_r, var_r = O.mf_diag(w.XL, w.yL, XH, yH, hyp, xs[pick])
                e = O.parity_errors(mu_h[i, pick], var_h[i, pick], mu_r, var_r, O.prior_variance(hyp))
                assert max(e) < TOL, (s, i, e)
    XH0 = wls[0].Xnew.reshape(-1, 2)
    assert np.unique(XH0, axis=0).shape[0] < XH0.shape[0] * 0.8   # revisits are in the data
    for m in models:
        st = m.stats()
        assert st["inc_factor"] == STEPS and st["full_predict"] == 1, st
        assert st["lattice"] == STEPS - 1 and st["vstream"] == STEPS, st
