"""GPU versions of the planner helpers that sit on the GP hot path.

``compute_sample_points`` mirrors simulator.py:326-374 (the Choi doubling
planner's sample-set selection, called once per period at sim:1031): on a copy
of the model, append the grid cell of maximal posterior variance with its
posterior mean as the observation until the maximal variance is at or below
the threshold, and return the chosen cells in order. Here the whole loop runs
on the device (libmfgp_hip's mfgp_sample_points): every iteration is a 1-row
bordered Cholesky append plus one pass over the resident V with a fused argmax,
and the host synchronises once per 32 iterations. Same signature, same return
value, same model-unchanged contract (the reference works on ``copy.deepcopy``).
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
