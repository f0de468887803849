"""Synthetic inputs of the benchmark workloads.

* grid: ``linspace(0,1,G)`` in the reference's x-outer row-major order
  (distribution.py:86-88; every Data/*_hifi.csv is this order at G = 51);
* training points are grid cells (the reference samples only at grid points,
  simulator.py:705, 875), distinct within a fidelity, drawn with
  ``default_rng(seed)``;
* values come from a sum-of-exponentials field in the style of
  ``distribution.exponential`` (distribution.py:22-71), normalised to [0,1],
  plus N(0, 0.1) noise on hifi samples and N(0, 0.01) on lofi samples
  (runner.py:86, distribution.py:305-306);
* hyperparameters are the reference's trained values (Data/*_hyp.csv), embedded
  here so nothing reads the reference at run time.
"""
from __future__ import annotations

import numpy as np

# Data/australia8_mf_hyp.csv (config 4, the headline) and others used by the configs
HYP = {
    "australia8_mf": np.array([-1.700903132, -1.947362545, -0.309197345, -14.9598621, -3.655273338,
                               -1.317607182, -0.721748367, -5.926942955, -1.371689752]),
    "australia9_mf": np.array([-2.451095562, -2.338000887, -0.640857957, -15.98930639, -3.643963754,
                               -2.281232319, -1.551102826, -4.605170186, -2.302585093]),
    "australia6_mf": np.array([-0.8460513962053721, -2.5372906071161143, -0.5420349584953533,
                               -18.003211372750144, -3.0873278390400363, -1.6010169416738749,
                               -0.6486247923907078, -4.616714381668361, -1.4266316993802974]),
    "australia3_sf": np.array([0.001, -2.368468757, -1.353149618, -4.596652374]),
    "anti_two_corners_sf": np.array([0.0001, -2.797478161, -1.500619305, -37.82682938]),
}


def grid(G):
    g = np.linspace(0.0, 1.0, G)
    return np.array([(a, b) for a in g for b in g], dtype=np.float64)


def field(xy, centres, width=0.05):
    f = np.zeros(xy.shape[0])
    for c in centres:
        f += np.exp(-np.sum((xy - c) ** 2, axis=1) / width)
    return f / f.max()


class Workload:
    """One Monte-Carlo seed: a grid, a lofi prior set, a hifi set and a stream of
    per-step agent samples (k new hifi points per update)."""

    def __init__(self, G, NL, NH, k, steps, seed, revisit=0.0):
        """revisit: the fraction of each step's k samples taken at cells sampled
        before (the base hifi set or earlier steps, the same cell twice in one step
        allowed), with fresh noise -- the reference's Todescato loop re-samples an
        explorer's current cell (simulator.py:872-891), so its training sets hold
        repeated rows. 0 (default) keeps every hifi cell distinct."""
        rng = np.random.default_rng(seed)
        self.xs = grid(G)
        M = self.xs.shape[0]
        centres = rng.random((4, 2))
        truth = field(self.xs, centres)
        lofi = field(self.xs, centres + 0.05 * rng.standard_normal((4, 2)), width=0.08)
        il = rng.choice(M, NL, replace=False) if NL else np.empty(0, dtype=np.int64)
        ih = rng.choice(M, NH + k * steps, replace=False)
        self.XL = self.xs[il]
        self.yL = lofi[il] + 0.01 * rng.standard_normal(il.shape[0])
        self.XH = self.xs[ih[:NH]]
        self.yH = truth[ih[:NH]] + 0.1 * rng.standard_normal(NH)
        inew = ih[NH:]
        if revisit > 0 and steps * k:
            # a separate stream, so that revisit = 0 draws exactly the data above
            rr = np.random.default_rng(seed + 7919)
            inew = inew.reshape(steps, k).copy()
            nrep = int(round(revisit * k))
            for s in range(steps):
                seen = np.concatenate([ih[:NH], inew[:s].reshape(-1)])
                if seen.size == 0:
                    continue
                slots = rr.choice(k, nrep, replace=False)
                inew[s, slots] = seen[rr.integers(0, seen.size, nrep)]
                if nrep >= 2 and s % 3 == 0:
                    inew[s, slots[1]] = inew[s, slots[0]]   # two agents in one cell
            inew = inew.reshape(-1)
        self.Xnew = self.xs[inew].reshape(steps, k, 2)
        self.ynew = (truth[inew] + 0.1 * rng.standard_normal(inew.shape[0])).reshape(steps, k)
