"""Voronoi-cell reductions of the planners, with the grid work on the GPU.

Mirrors of simulator.py's per-cell reductions over a bounded Voronoi partition
(the ``vor`` objects of ``voronoi_bounded``, sim:154-191: ``vertices``,
``filtered_regions``, ``filtered_points``):

* ``compute_loss(vor, truth_arr)``              -- sim:194-228
* ``compute_centroids(vor, x_star, mu_star)``   -- sim:231-283
* ``compute_max_var(vor, truth_arr, var_star)`` -- sim:286-323

Which grid points fall in which cell is decided on the device by the
reference's own rule (in_polygon, sim:105-124 = matplotlib's crossing test,
reproduced exactly in mfgp_cells.hip), and the per-cell sums, maxima and
argmaxima are reduced there too (mfgp_cell_reduce). The host keeps what is
O(cells): the polygon areas (Shoelace, sim:127-136) and the final divisions.
Same signatures and return values as the reference; ``var_star`` may be the
``DiagCov`` of ``predict`` or a dense matrix (only its diagonal is read,
sim:302).
"""
from __future__ import annotations

import numpy as np

from . import _lib


def _polygons(vor):
    regions = [list(r) for r in vor.filtered_regions]
    verts = [np.asarray(vor.vertices, dtype=np.float64)[r, :] for r in regions]
    vstart = np.zeros(len(regions) + 1, dtype=np.int32)
    vstart[1:] = np.cumsum([v.shape[0] for v in verts])
    flat = np.vstack(verts) if verts else np.empty((0, 2))
    return flat, vstart, verts, np.asarray(vor.filtered_points, dtype=np.float64)


def _area(v):
    """Shoelace area of a polygon given as [n, 2] vertices (sim:127-136)."""
    x, y = v[:, 0], v[:, 1]
    # (np.roll(a, 1) of these 1-D arrays, built without np.roll's overhead: the same arrays)
    return 0.5 * np.abs(np.dot(x, np.concatenate((y[-1:], y[:-1]))) - np.dot(y, np.concatenate((x[-1:], x[:-1]))))


def compute_loss(vor, truth_arr):
    """sim:194-228: sum over cells of mean(|x - seed|^2 * f) * cell area."""
    truth_arr = np.asarray(truth_arr, dtype=np.float64)
    flat, vstart, verts, seeds = _polygons(vor)
    out, _ = _lib.cell_reduce(truth_arr[:, :2], flat, vstart, seeds, f=truth_arr[:, 2])
    loss = 0
    with np.errstate(invalid="ignore", divide="ignore"):   # an empty cell gives NaN, as np.mean([]) does
        for i, v in enumerate(verts):
            loss += (out[i, 4] / out[i, 0]) * _area(v)
    return loss


def compute_centroids(vor, x_star, mu_star):
    """sim:231-283: mu-weighted centroid of every cell, snapped into the domain."""
    x_star = np.asarray(x_star, dtype=np.float64)
    mu = np.asarray(mu_star, dtype=np.float64).reshape(x_star.shape[0], -1)[:, 0]
    flat, vstart, verts, seeds = _polygons(vor)
    out, _ = _lib.cell_reduce(x_star[:, :2], flat, vstart, seeds, w=mu)
    # (per column: the same values as x_star[:, :2].min(0) / .max(0), ~15x faster)
    lo = np.array([x_star[:, 0].min(), x_star[:, 1].min()])
    hi = np.array([x_star[:, 0].max(), x_star[:, 1].max()])
    centroids = np.empty((len(verts), 2))
    with np.errstate(invalid="ignore", divide="ignore"):
        for i, v in enumerate(verts):
            area = _area(v)
            n = out[i, 0]
            f_integral = (out[i, 1] / n) * area
            weighted = np.array([out[i, 2] / n, out[i, 3] / n]) * area
            centroids[i] = np.minimum(np.maximum(weighted / f_integral, lo), hi)
    return centroids


def compute_max_var(vor, truth_arr, var_star):
    """sim:286-323 -> (argmax (x, y) per cell [n, 2], max var per cell [n, 1])."""
    truth_arr = np.asarray(truth_arr, dtype=np.float64)
    var = np.ascontiguousarray(np.diag(var_star), dtype=np.float64)
    flat, vstart, _, seeds = _polygons(vor)
    out, am = _lib.cell_reduce(truth_arr[:, :2], flat, vstart, seeds, var=var)
    if np.any(am < 0):
        raise ValueError("zero-size array to reduction operation maximum which has no identity")
    return truth_arr[am][:, [0, 1]].reshape(-1, 2), out[:, 5].reshape(-1, 1)
