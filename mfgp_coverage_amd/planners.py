"""GPU versions of the planner helpers that sit on the GP hot path.

``compute_sample_points`` mirrors simulator.py:326-374 (the Choi doubling
planner's sample-set selection, called once per period at sim:1031): on a copy
of the model, append the grid cell of maximal posterior variance with its
posterior mean as the observation until the maximal variance is at or below
the threshold, and return the chosen cells in order. Here the whole loop runs
on the device (libmfgp_hip's mfgp_sample_points): every iteration is a 1-row
bordered Cholesky append plus one pass over the resident V with a fused argmax,
and the host synchronises once per 32 iterations. Same signature, same return
value, same model-unchanged contract: the reference works on ``copy.deepcopy``;
here the rows go past the model's own and are dropped at the end (the leading
rows' factor, V and F do not depend on them), and what the loop overwrites
besides -- the resident posterior, the kept result, the path counters -- is saved
and restored, so no copy of the model's device state is made.

``compute_sample_points_batch`` runs the same loop for many models at once (the
Choi planner of a rank's Monte-Carlo seeds: one seed's sample set each): every
iteration is one decision launch for all of them and one batched 1-row append +
predict (libmfgp_hip's mfgp_batch_sample_points, the lattice step where the batch
takes it); each model stops at its own threshold.
"""
from __future__ import annotations

import numpy as np

from .gaussian_process import MFGP, SFGP


def compute_sample_points(model, x_star, threshold, console):
    """simulator.py:326-374 -> [n, 2] ndarray of the cells to sample, in order."""
    if not isinstance(model, (SFGP, MFGP)):
        raise TypeError("Invalid model type: must be SFGP or MFGP")
    xs = np.ascontiguousarray(np.asarray(x_star, dtype=np.float64).reshape(-1, 2))
    model._sync_data()
    model._push_hyp()
    model._grid_to_device(xs)
    # the reference loops until the threshold is met; bound the output buffer
    # generously and refuse to return a truncated answer
    cap = 4 * xs.shape[0] + 1
    pts = model._dev().sample_points(float(threshold), cap)
    if pts.shape[0] >= cap:
        raise RuntimeError("compute_sample_points: no convergence within %d points" % cap)
    if console:
        print("Sample points to reduce max var below " + str(threshold) + ": " + str(pts.shape[0]))
    return pts


def compute_sample_points_batch(models, x_star, thresholds, console=False):
    """compute_sample_points (simulator.py:326-374) for every model of ``models``
    (one context, one dtype, the same grid ``x_star``), stepped together ->
    list of [n_b, 2] arrays, each model's cells in order. ``thresholds``: one value
    or one per model."""
    from . import _lib
    if not models:
        return []
    for m in models:
        if not isinstance(m, (SFGP, MFGP)):
            raise TypeError("Invalid model type: must be SFGP or MFGP")
    xs = np.ascontiguousarray(np.asarray(x_star, dtype=np.float64).reshape(-1, 2))
    for m in models:
        m._sync_data()
        m._push_hyp()
        m._grid_to_device(xs)
    cap = 4 * xs.shape[0] + 1
    thr = np.broadcast_to(np.asarray(thresholds, dtype=np.float64), (len(models),))
    pts = _lib.batch_sample_points([m._dev() for m in models], thr, cap)
    for b, p in enumerate(pts):
        if p.shape[0] >= cap:
            raise RuntimeError("compute_sample_points: no convergence within %d points" % cap)
        if console:
            print("Sample points to reduce max var below " + str(thr[b]) + ": " + str(p.shape[0]))
    return pts
