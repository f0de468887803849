"""Voronoi-cell reductions on the device (mfgp_cells.hip through
mfgp_coverage_amd.geometry) against the reference's own compute_loss,
compute_centroids and compute_max_var (simulator.py:194-323) on 12 bounded
Voronoi partitions of the native anti_two_corners grid
(tests/golden/cells_reference.npz, made by make_golden.py from /root/reference).

Membership must be exact: half of the partitions have grid points on cell
boundaries, where the reference's in_polygon counts a point in two cells or in
none, and the device reproduces that. Same inputs, so max var and its argmax are
bit-exact; the sums differ from NumPy's pairwise means by rounding only.
"""
import types

import numpy as np
import pytest

from oracle import gp_oracle as O
from tests import _fixtures as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cells():
    return F.load("cells_reference.npz")


def _vor(fx, i):
    """A voronoi_bounded-like object (vertices, filtered_regions, filtered_points)."""
    verts, vs = fx[f"c{i}_verts"], fx[f"c{i}_vstart"]
    regions = [list(range(vs[j], vs[j + 1])) for j in range(vs.shape[0] - 1)]
    return types.SimpleNamespace(vertices=verts, filtered_regions=regions, filtered_points=fx[f"c{i}_seeds"])


@pytest.mark.parametrize("i", range(12))
def test_cell_reductions_vs_reference(cells, i):
    from mfgp_coverage_amd import _lib, geometry
    truth, mu, var = cells["truth"], cells["mu"], cells["var"]
    xs = truth[:, :2]
    vor = _vor(cells, i)
    # membership counts (in_polygon), straight from the kernel
    vs = cells[f"c{i}_vstart"]
    out, am = _lib.cell_reduce(xs, cells[f"c{i}_verts"], vs, cells[f"c{i}_seeds"], w=mu, f=truth[:, 2], var=var)
    np.testing.assert_array_equal(out[:, 0].astype(np.int64), cells[f"c{i}_counts"])
    np.testing.assert_allclose(geometry.compute_loss(vor, truth), cells[f"c{i}_loss"], rtol=1e-13)
    np.testing.assert_allclose(geometry.compute_centroids(vor, xs, mu.reshape(-1, 1)), cells[f"c{i}_centroids"],
                               rtol=1e-13, atol=1e-15)
    # the predict output form (DiagCov) and a dense matrix both work
    from mfgp_coverage_amd.gaussian_process import DiagCov
    am_pts, mv = geometry.compute_max_var(vor, truth, DiagCov(var))
    np.testing.assert_array_equal(mv, cells[f"c{i}_maxvar"])
    np.testing.assert_array_equal(am_pts, cells[f"c{i}_argmax"])


def test_cell_reductions_random_vs_oracle():
    """Random polygons (convex and not) and weights on a 128x128 grid against the
    oracle's restatement; device-resident inputs and outputs."""
    import torch
    from mfgp_coverage_amd import _lib
    rng = np.random.default_rng(3)
    g = np.linspace(0, 1, 128)
    xs = np.array([(a, b) for a in g for b in g])
    polys = []
    for n in (3, 5, 8, 12):
        ang = np.sort(rng.random(n)) * 2 * np.pi
        rad = 0.2 + 0.3 * rng.random(n)
        c = rng.random(2)
        polys.append(np.column_stack([c[0] + rad * np.cos(ang), c[1] + rad * np.sin(ang)]))
    polys.append(np.array([[0.0, 0.0], [1.0, 0.0], [1.0, 1.0], [0.0, 1.0]]))   # the whole box: edges on grid lines
    seeds = rng.random((len(polys), 2))
    w, f, var = rng.random(xs.shape[0]), rng.random(xs.shape[0]), rng.random(xs.shape[0])
    verts = np.vstack(polys)
    vs = np.concatenate([[0], np.cumsum([p.shape[0] for p in polys])]).astype(np.int32)
    dev = {k: torch.from_numpy(np.ascontiguousarray(a)).cuda() for k, a in
           (("xs", xs), ("verts", verts), ("seeds", seeds), ("w", w), ("f", f), ("var", var))}
    out_d = torch.empty((len(polys), 6), dtype=torch.float64, device="cuda")
    am_d = torch.empty(len(polys), dtype=torch.int64, device="cuda")
    import ctypes
    _lib.check(_lib.lib().mfgp_cell_reduce(
        _lib.context().handle, ctypes.c_void_p(dev["xs"].data_ptr()), xs.shape[0], len(polys),
        ctypes.c_void_p(vs.ctypes.data), ctypes.c_void_p(dev["verts"].data_ptr()),
        ctypes.c_void_p(dev["seeds"].data_ptr()), ctypes.c_void_p(dev["w"].data_ptr()),
        ctypes.c_void_p(dev["f"].data_ptr()), ctypes.c_void_p(dev["var"].data_ptr()),
        ctypes.c_void_p(out_d.data_ptr()), ctypes.c_void_p(am_d.data_ptr())))
    out, am = out_d.cpu().numpy(), am_d.cpu().numpy()
    ref = O.cell_reductions(polys, seeds, xs, w=w, f=f, var=var)
    for j, (m, _, _, vmax, amax) in enumerate(ref):
        assert out[j, 0] == m.sum()
        np.testing.assert_allclose(out[j, 1], w[m].sum(), rtol=1e-12)
        np.testing.assert_allclose(out[j, 2], (w[m] * xs[m, 0]).sum(), rtol=1e-12)
        np.testing.assert_allclose(out[j, 4], (np.sum((xs[m] - seeds[j]) ** 2, 1) * f[m]).sum(), rtol=1e-12)
        assert out[j, 5] == vmax and am[j] == amax
