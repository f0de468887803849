"""Shared fixture readers and the log-replay driver (test infrastructure)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NS = (0, 9, 50, 130, 260)
GRIDS = ("g51", "g32")
REPLAY_RUNS = (
    "atc24_todescato_nsf", "atc24_todescato_hsf", "atc24_todescato_hmf",
    "atc24_choi_hmf", "atc248_todescato_hmf",
    "australia6_todescato_nsf", "australia6_todescato_hmf",
    # priors partly off the grid's lattice, revisited cells (make_golden.py REPLAYS)
    "australia2_todescato_hsf", "australia2_todescato_hmf",
    "australia4_todescato_hsf", "australia4_todescato_hmf",
)


def load(name):
    # plain arrays only: allow_pickle stays False
    with np.load(os.path.join(GOLDEN, name)) as z:
        return {k: z[k] for k in z.files}


def atc():
    return load("atc_reference.npz")


def replay(run):
    return load(f"replay_{run}.npz")


def replay_run(fx, sim, make_model, append, predict_var):
    """Replay a logged run (simulator.py:864-892 / 1056-1084).

    make_model(hyp, prior_or_None) -> model conditioned on the prior
    append(model, X[k,2], y[k,1])  -> updt / updt_hifi (k may be 0)
    predict_var(model) -> diag posterior variance over fx['grid']
    Returns (logged max VarMax per iteration, replayed max var per iteration).
    """
    hyp = fx["hyp"]
    prior = fx.get("prior")
    model = make_model(hyp, prior)
    its = fx[f"s{sim}_iters"]
    s_it = fx[f"s{sim}_sample_iter"]
    s_xy = fx[f"s{sim}_sample_xy"]
    s_y = fx[f"s{sim}_sample_y"]
    got = np.empty(its.shape[0])
    for n, it in enumerate(its):
        sel = s_it == it
        append(model, s_xy[sel].reshape(-1, 2), s_y[sel].reshape(-1, 1))
        got[n] = np.max(predict_var(model))
    return fx[f"s{sim}_varmax"], got
