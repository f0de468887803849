"""A Todescato-style coverage loop driven through the drop-in API, against the same
loop on the CPU oracle.

Each step follows simulator.py:840-892 in miniature: predict the posterior on the
grid, partition the domain among the agents (bounded Voronoi cells), move every
agent to its cell's mean-weighted centroid (compute_centroids, sim:231-283),
sample the field there (grid cells, sim:875) and append the samples to the hifi
set (updt_hifi, sim:888-892). On the device the loop runs MFGP.predict /
updt_hifi (bordered appends) and geometry.compute_centroids (mfgp_cell_reduce);
on the CPU it runs oracle.mf_diag and oracle.cell_reductions. The agents'
trajectories must be identical and the last posterior within the parity
tolerance.
"""
import types

import numpy as np
import pytest

from oracle import gp_oracle as O

pytestmark = pytest.mark.gpu

EPS = 1e-9


def _bounded_voronoi(points, box):
    """Voronoi cells of `points` clipped to `box` by mirroring the seeds across its
    four sides (the construction of simulator.py:154-191); the object carries the
    fields the planners read: vertices, filtered_regions, filtered_points."""
    from scipy.spatial import Voronoi
    x0, x1, y0, y1 = box
    c = np.asarray(points, dtype=np.float64)
    left, right, down, up = c.copy(), c.copy(), c.copy(), c.copy()
    left[:, 0] = x0 - (c[:, 0] - x0 + EPS)
    right[:, 0] = x1 + (x1 - c[:, 0] + EPS)
    down[:, 1] = y0 - (c[:, 1] - y0 + EPS)
    up[:, 1] = y1 + (y1 - c[:, 1] + EPS)
    vor = Voronoi(np.vstack([c, left, right, down, up]))
    regions = [vor.regions[vor.point_region[i]] for i in range(c.shape[0])]
    return types.SimpleNamespace(vertices=vor.vertices, filtered_regions=regions, filtered_points=c)


def _cpu_centroids(vor, xs, mu):
    polys = [vor.vertices[r, :] for r in vor.filtered_regions]
    cen = np.array([r[1] for r in O.cell_reductions(polys, vor.filtered_points, xs, w=mu)])
    lo, hi = xs.min(0), xs.max(0)
    return np.clip(cen, lo, hi)   # the reference's snapping into the domain (sim:272-280)


def _nearest_cells(xs, pts):
    return np.array([int(np.argmin(((xs - p) ** 2).sum(1))) for p in pts])


def test_todescato_loop_matches_cpu():
    from mfgp_coverage_amd import geometry
    from mfgp_coverage_amd.gaussian_process import MFGP
    from mfgp_coverage_amd.synthetic import HYP, Workload, field
    hyp = HYP["australia8_mf"]
    G, agents, steps = 40, 4, 10
    w = Workload(G, 120, 24, 1, 1, seed=41)
    xs = w.xs
    rng = np.random.default_rng(4)
    truth = field(xs, rng.random((4, 2)))
    noise = 0.1 * rng.standard_normal((steps, agents))
    start = rng.choice(xs.shape[0], agents, replace=False)
    box = (0.0, 1.0, 0.0, 1.0)

    gp = MFGP(w.XL.copy(), w.yL.reshape(-1, 1).copy(), w.XH.copy(), w.yH.reshape(-1, 1).copy(), 1, 1)
    gp.hyp = hyp.copy()
    gp.updt_info(gp.X_L, gp.y_L, gp.X_H, gp.y_H)
    XH_cpu, yH_cpu = w.XH.copy(), w.yH.copy()

    pos_gpu, pos_cpu = xs[start].copy(), xs[start].copy()
    for t in range(steps):
        mu, cov = gp.predict(xs)
        mu_c, var_c = O.mf_diag(w.XL, w.yL, XH_cpu, yH_cpu, hyp, xs)
        e = O.parity_errors(mu[:, 0], np.diag(cov), mu_c, var_c, O.prior_variance(hyp))
        assert max(e) < O.PARITY_TOL, (t, e)
        cen_g = geometry.compute_centroids(_bounded_voronoi(pos_gpu, box), xs, mu)
        cen_c = _cpu_centroids(_bounded_voronoi(pos_cpu, box), xs, mu_c)
        np.testing.assert_allclose(cen_g, cen_c, rtol=1e-9, atol=1e-12)
        cells_g, cells_c = _nearest_cells(xs, cen_g), _nearest_cells(xs, cen_c)
        np.testing.assert_array_equal(cells_g, cells_c)
        pos_gpu, pos_cpu = xs[cells_g], xs[cells_c]
        y_new = truth[cells_g] + noise[t]
        gp.updt_hifi(pos_gpu, y_new.reshape(-1, 1))
        XH_cpu = np.vstack([XH_cpu, pos_cpu])
        yH_cpu = np.concatenate([yH_cpu, y_new])
    mu, cov = gp.predict(xs)
    mu_c, var_c = O.mf_diag(w.XL, w.yL, XH_cpu, yH_cpu, hyp, xs)
    assert max(O.parity_errors(mu[:, 0], np.diag(cov), mu_c, var_c, O.prior_variance(hyp))) < O.PARITY_TOL
    st = gp._dev().stats()
    assert st["inc_factor"] >= steps, st   # the appends took the bordered path
