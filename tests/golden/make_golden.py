"""Generate the golden fixtures under tests/golden/ -- BUILD CONTAINER ONLY.

Two kinds of fixtures, both plain data (.npz, no pickles):

1. ``atc_reference.npz``: outputs of the reference's OWN ``gaussian_process.py``
   (``/root/reference``, imported here with a pass-through ``autograd`` shim:
   ``autograd.numpy`` is NumPy for non-traced calls, gp:16-17; ``value_and_grad``
   is only used by ``train``, gp:117/397, which is never called) on the
   ``anti_two_corners`` data (``Data/anti_two_corners_*``): SF and MF, the native
   51x51 grid and a 32x32 grid, N in {0, 9, 50, 130, 260}, plus append sequences
   (``updt`` / ``updt_hifi`` in chunks of 4, and an empty append).
   Stored: inputs (hyp, training data, grids) and ``mu``, ``diag(cov)``,
   ``amax(cov)``.

2. ``replay_*.npz``: the reference's own logged runs (``Data/<run>_sample.csv``
   and ``Data/<run>_agent.csv``), reduced to what the GP path determines: the
   sample sequence per iteration and the per-iteration max of the logged
   ``VarMax`` (max posterior variance per Voronoi cell, simulator.py:286-323; the
   max over cells is the max over the grid) plus ``Var0`` (simulator.py:841-842).
   No reference code is involved in (2): it is a CSV extraction.

Run: ``python tests/golden/make_golden.py`` (needs /root/reference; the GPU box
never runs this -- it only reads the committed .npz files).
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import pandas as pd

REF = "/root/reference"
DATA = os.path.join(REF, "Data")
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    shim = types.ModuleType("autograd")
    shim.numpy = np
    shim.value_and_grad = None
    sys.modules.setdefault("autograd", shim)
    sys.modules.setdefault("autograd.numpy", np)
    sys.path.insert(0, REF)
    import gaussian_process as gp  # noqa: E402  (the reference module)
    return gp


def _csv(name):
    return pd.read_csv(os.path.join(DATA, name)).values.astype(np.float64)


def grid32():
    g = np.linspace(0.0, 1.0, 32)
    # x-outer row-major order, distribution.py:86-88
    return np.array([(a, b) for a in g for b in g], dtype=np.float64)


def make_reference_fixture(gp):
    hyp_sf = _csv("anti_two_corners_sf_hyp.csv")[0]
    hyp_mf = _csv("anti_two_corners_mf_hyp.csv")[0]
    truth = _csv("anti_two_corners_hifi.csv")
    train = _csv("anti_two_corners_hifi_train.csv")
    prior = _csv("anti_two_corners_prior.csv")
    grids = {"g51": truth[:, :2].copy(), "g32": grid32()}
    out = {"hyp_sf": hyp_sf, "hyp_mf": hyp_mf, "train": train, "prior": prior,
           "grid_g51": grids["g51"], "grid_g32": grids["g32"]}
    e2, e1 = np.empty((0, 2)), np.empty((0, 1))

    def pred(model, gname):
        mu, cov = model.predict(grids[gname])
        return mu[:, 0].copy(), np.diag(cov).copy(), float(np.amax(cov))

    for gname in grids:
        for N in (0, 9, 50, 130, 260):
            X, y = train[:N, :2].copy(), train[:N, 2:3].copy()
            # SF: SFGP(X, y, len) then .hyp = ... then updt_info (simulator.py:78-102, 676-678)
            m = gp.SFGP(X, y, 1)
            m.hyp = hyp_sf.copy()
            if N > 0:
                m.updt_info(m.X, m.y)
            mu, var, vmax = pred(m, gname)
            key = f"sf_{gname}_n{N}"
            out[key + "_mu"], out[key + "_var"], out[key + "_amax"] = mu, var, np.array(vmax)
            # MF: lofi = prior (simulator.py:59-63), hifi = first N training rows
            m = gp.MFGP(prior[:, :2].copy(), prior[:, 2:3].copy(), X, y, 1, 1)
            m.hyp = hyp_mf.copy()
            m.updt_info(m.X_L, m.y_L, m.X_H, m.y_H)
            mu, var, vmax = pred(m, gname)
            key = f"mf_{gname}_n{N}"
            out[key + "_mu"], out[key + "_var"], out[key + "_amax"] = mu, var, np.array(vmax)
        # fully empty MF (null prior): the Var0 path (simulator.py:829-842)
        m = gp.MFGP(e2.copy(), e1.copy(), e2.copy(), e1.copy(), 1, 1)
        m.hyp = hyp_mf.copy()
        mu, var, vmax = pred(m, gname)
        key = f"mfempty_{gname}"
        out[key + "_mu"], out[key + "_var"], out[key + "_amax"] = mu, var, np.array(vmax)

    # append sequences on the native grid: updt / updt_hifi (gp:257-268, 531-542)
    chunks = [4, 4, 0, 4, 4, 1]
    sf = gp.SFGP(prior[:, :2].copy(), prior[:, 2:3].copy(), 1)
    sf.hyp = hyp_sf.copy()
    sf.updt_info(sf.X, sf.y)
    mf = gp.MFGP(prior[:, :2].copy(), prior[:, 2:3].copy(), e2.copy(), e1.copy(), 1, 1)
    mf.hyp = hyp_mf.copy()
    mf.updt_info(mf.X_L, mf.y_L, mf.X_H, mf.y_H)
    pos = 0
    for s, k in enumerate(chunks):
        xa, ya = train[pos:pos + k, :2].copy(), train[pos:pos + k, 2:3].copy()
        pos += k
        sf.updt(xa, ya)
        mf.updt_hifi(xa, ya)
        for name, model in (("sfseq", sf), ("mfseq", mf)):
            mu, var, vmax = pred(model, "g51")
            key = f"{name}_s{s}"
            out[key + "_mu"], out[key + "_var"], out[key + "_amax"] = mu, var, np.array(vmax)
    out["seq_chunks"] = np.array(chunks, dtype=np.int64)
    np.savez_compressed(os.path.join(OUT, "atc_reference.npz"), **out)
    print("wrote atc_reference.npz with", len(out), "arrays")


# run name -> (truth/grid data prefix, hyp file, prior file or None)
REPLAYS = {
    "atc24_todescato_nsf": ("anti_two_corners", "anti_two_corners_sf_hyp.csv", None, (0, 1)),
    "atc24_todescato_hsf": ("anti_two_corners", "anti_two_corners_sf_hyp.csv", "anti_two_corners_prior.csv", (0, 1)),
    "atc24_todescato_hmf": ("anti_two_corners", "anti_two_corners_mf_hyp.csv", "anti_two_corners_prior.csv", (0, 1)),
    "atc24_choi_hmf": ("anti_two_corners", "anti_two_corners_mf_hyp.csv", "anti_two_corners_prior.csv", (0,)),
    "atc248_todescato_hmf": ("anti_two_corners", "anti_two_corners_mf_hyp.csv", "anti_two_corners_prior.csv", (3,)),
    "australia6_todescato_nsf": ("australia6", "australia6_sf_hyp.csv", None, (0,)),
    "australia6_todescato_hmf": ("australia6", "australia6_mf_hyp.csv", "australia6_prior.csv", (0,)),
    # priors partly off the grid's lattice (distribution.py:112-113 builds them by
    # float steps: australia2 has 17 of 81 rows 1 ulp off the grid's axis values,
    # australia4 11 of 36) and revisited cells (australia4_todescato_hsf: 40 samples
    # at 13 distinct cells; simulator.py:872-891 re-samples an explorer's cell)
    "australia2_todescato_hsf": ("australia2", "australia2_sf_hyp.csv", "australia2_prior.csv", (0, 1)),
    "australia2_todescato_hmf": ("australia2", "australia2_mf_hyp.csv", "australia2_prior.csv", (0, 1)),
    "australia4_todescato_hsf": ("australia4", "australia4_sf_hyp.csv", "australia4_prior.csv", (0,)),
    "australia4_todescato_hmf": ("australia4", "australia4_mf_hyp.csv", "australia4_prior.csv", (0,)),
}


def make_replay_fixtures():
    for run, (data, hypf, priorf, sims) in REPLAYS.items():
        agent = pd.read_csv(os.path.join(DATA, run + "_agent.csv"))
        sample = pd.read_csv(os.path.join(DATA, run + "_sample.csv"))
        out = {"hyp": _csv(hypf)[0], "grid": _csv(data + "_hifi.csv")[:, :2].copy(),
               "sims": np.array(sims, dtype=np.int64)}
        if priorf is not None:
            out["prior"] = _csv(priorf)
        for sim in sims:
            a = agent[agent.SimNum == sim]
            s = sample[sample.SimNum == sim]
            its = np.sort(a.Iteration.unique())
            out[f"s{sim}_iters"] = its.astype(np.int64)
            out[f"s{sim}_varmax"] = a.groupby("Iteration").VarMax.max().loc[its].values.astype(np.float64)
            out[f"s{sim}_var0"] = np.array(a.Var0.iloc[0], dtype=np.float64)
            out[f"s{sim}_sample_iter"] = s.Iteration.values.astype(np.int64)
            out[f"s{sim}_sample_xy"] = s[["X", "Y"]].values.astype(np.float64)
            out[f"s{sim}_sample_y"] = s.Sample.values.astype(np.float64)
        np.savez_compressed(os.path.join(OUT, f"replay_{run}.npz"), **out)
        print("wrote replay", run)


def make_prior_fixtures():
    """7. ``priors_offlattice.npz``: the reference's priors that lie partly off the
    grid's lattice (distribution.py:112-113 steps the prior positions by float
    additions, so some coordinates end 1 ulp away from the grid's axis values,
    e.g. 0.6000000000000001 against 0.6), with the native 51x51 grid they come
    with (``<name>_hifi.csv``) and the trained hyperparameters. CSV extraction."""
    out = {}
    for name in ("australia2", "australia3", "australia4", "australia9"):
        out[name + "_prior"] = _csv(name + "_prior.csv")
        out[name + "_grid"] = _csv(name + "_hifi.csv")[:, :2].copy()
        out[name + "_hyp_sf"] = _csv(name + "_sf_hyp.csv")[0]
        out[name + "_hyp_mf"] = _csv(name + "_mf_hyp.csv")[0]
        g = out[name + "_grid"]
        ax, ay = np.unique(g[:, 0]), np.unique(g[:, 1])
        P = out[name + "_prior"]
        off = ~(np.isin(P[:, 0], ax) & np.isin(P[:, 1], ay))
        print(name, "prior rows", P.shape[0], "off the lattice", int(off.sum()))
    np.savez_compressed(os.path.join(OUT, "priors_offlattice.npz"), **out)


def _import_simulator():
    """simulator.py needs `mlrose` at import (sim:29, used only by the TSP step);
    a stub module stands in for it. compute_sample_points itself runs unchanged."""
    sys.modules.setdefault("mlrose", types.ModuleType("mlrose"))
    import simulator as sim  # noqa: E402  (the reference module)
    return sim


def make_choi_fixture(gp, sim):
    """3. ``choi_reference.npz``: the reference's own ``compute_sample_points``
    (simulator.py:326-374, the Choi planner's sample-set selection) on
    anti_two_corners models and the 32x32 grid. Stored per case: the chosen
    points in order, and for every step the gap between the largest and the
    second largest posterior variance the loop's argmax saw (an argmax whose gap is
    below the parity tolerance is decided by rounding, so the tests compare the
    sequence only up to the first such step)."""
    import copy
    hyp_sf = _csv("anti_two_corners_sf_hyp.csv")[0]
    hyp_mf = _csv("anti_two_corners_mf_hyp.csv")[0]
    train = _csv("anti_two_corners_hifi_train.csv")
    prior = _csv("anti_two_corners_prior.csv")
    xs = grid32()
    e2, e1 = np.empty((0, 2)), np.empty((0, 1))
    out = {"grid": xs, "hyp_sf": hyp_sf, "hyp_mf": hyp_mf, "train": train, "prior": prior}
    cases = {
        # name: (builder, threshold as a fraction of the model's current max variance)
        "sf_n50": (lambda: gp.SFGP(train[:50, :2].copy(), train[:50, 2:3].copy(), 1), hyp_sf, 0.08),
        "mf_n20": (lambda: gp.MFGP(prior[:, :2].copy(), prior[:, 2:3].copy(), train[:20, :2].copy(),
                                   train[:20, 2:3].copy(), 1, 1), hyp_mf, 0.08),
        "mf_prior": (lambda: gp.MFGP(prior[:, :2].copy(), prior[:, 2:3].copy(), e2.copy(), e1.copy(), 1, 1),
                     hyp_mf, 0.15),
    }
    for name, (build, hyp, frac) in cases.items():
        m = build()
        m.hyp = hyp.copy()
        if isinstance(m, gp.SFGP):
            m.updt_info(m.X, m.y)
        else:
            m.updt_info(m.X_L, m.y_L, m.X_H, m.y_H)
        _, cov = m.predict(xs)
        thr = frac * float(np.amax(cov))
        pts = sim.compute_sample_points(m, xs, thr, False)
        # the same loop again, recording the argmax margins (and checking the points)
        t = copy.deepcopy(m)
        mu, cov = t.predict(xs)
        var = np.diag(cov)
        gaps = []
        for p in pts:
            j = int(np.argmax(var))
            assert np.array_equal(xs[j], p)
            srt = np.sort(var)
            gaps.append(srt[-1] - srt[-2])
            (t.updt if isinstance(t, gp.SFGP) else t.updt_hifi)(xs[j:j + 1], mu[j:j + 1])
            mu, cov = t.predict(xs)
            var = np.diag(cov)
        out[name + "_threshold"] = np.array(thr)
        out[name + "_points"] = np.asarray(pts, dtype=np.float64).reshape(-1, 2)
        out[name + "_gaps"] = np.array(gaps, dtype=np.float64)
        print(name, "points", len(pts), "min gap", min(gaps) if gaps else None)
    np.savez_compressed(os.path.join(OUT, "choi_reference.npz"), **out)


def _voronoi_bounded(sim, seeds, bb):
    """The reference's voronoi_bounded (sim:154-191). Its np.array(vor.regions)
    (sim:190) fails on NumPy >= 1.24 for ragged regions; the same call with an
    object array is what older NumPy did."""
    real = sim.np.array

    def arr(x, *a, **k):
        try:
            return real(x, *a, **k)
        except ValueError:
            return real(x, dtype=object)
    sim.np.array = arr
    try:
        return sim.voronoi_bounded(seeds, bb)
    finally:
        sim.np.array = real


def make_cells_fixture(sim):
    """4. ``cells_reference.npz``: the reference's own compute_loss,
    compute_centroids and compute_max_var (sim:194-323) over voronoi_bounded
    partitions (sim:154-191) of random agent sets on the native 51x51
    anti_two_corners grid (half of them on grid points, so that grid points lie
    on cell boundaries), with the reference GP's posterior mean / variance
    (mf_g51_n50 of atc_reference.npz) as the weights. Stored per case: the
    seeds, the cell polygons (flattened + offsets), the per-cell point counts of
    in_polygon, and the three functions' outputs."""
    truth = _csv("anti_two_corners_hifi.csv")
    xs = truth[:, :2].copy()
    ref = np.load(os.path.join(OUT, "atc_reference.npz"))
    mu, var = ref["mf_g51_n50_mu"], ref["mf_g51_n50_var"]
    bb = np.array([xs[:, 0].min(), xs[:, 0].max(), xs[:, 1].min(), xs[:, 1].max()])
    rng = np.random.default_rng(2020)
    out = {"truth": truth, "mu": mu, "var": var}
    ncase = 0
    dense_var = np.diag(var)
    while ncase < 12:
        n = int(rng.integers(2, 9))
        seeds = rng.random((n, 2))
        if ncase % 2 == 0:
            seeds = np.round(seeds * 50) / 50
        vor = _voronoi_bounded(sim, seeds, bb)
        polys = [vor.vertices[list(c), :] for c in vor.filtered_regions]
        counts = np.array([sim.in_polygon(xs[:, 0], xs[:, 1], v[:, 0], v[:, 1]).sum() for v in polys])
        if np.any(counts == 0):
            continue
        key = f"c{ncase}"
        out[key + "_seeds"] = np.asarray(vor.filtered_points, dtype=np.float64)
        out[key + "_verts"] = np.vstack(polys).astype(np.float64)
        out[key + "_vstart"] = np.concatenate([[0], np.cumsum([v.shape[0] for v in polys])]).astype(np.int32)
        out[key + "_counts"] = counts.astype(np.int64)
        out[key + "_loss"] = np.array(sim.compute_loss(vor, truth))
        out[key + "_centroids"] = sim.compute_centroids(vor, xs, mu.reshape(-1, 1))
        am, mv = sim.compute_max_var(vor, truth, dense_var)
        out[key + "_argmax"], out[key + "_maxvar"] = am, mv
        ncase += 1
    out["ncases"] = np.array(ncase)
    np.savez_compressed(os.path.join(OUT, "cells_reference.npz"), **out)
    print("wrote cells_reference.npz,", ncase, "partitions")


def make_nlml_fixture(gp):
    """5. ``nlml_reference.npz``: the reference's own likelihood (gp:81-106 SF,
    gp:344-385 MF) on anti_two_corners data at the trained hyperparameters and at
    moved ones, with its central finite-difference gradient (h = 1e-6; the
    reference differentiates with autograd, which is absent here)."""
    train = _csv("anti_two_corners_hifi_train.csv")
    prior = _csv("anti_two_corners_prior.csv")
    hyp_sf = _csv("anti_two_corners_sf_hyp.csv")[0]
    hyp_mf = _csv("anti_two_corners_mf_hyp.csv")[0]
    rng = np.random.default_rng(7)
    out = {"train": train, "prior": prior}
    cases = []
    for n in (50, 130):
        for j, h in enumerate((hyp_sf, hyp_sf + np.array([0.0, 0.3, -0.2, 30.0]))):
            cases.append((f"sf_n{n}_h{j}", "sf", n, h))
    for n in (30, 90):
        for j, h in enumerate((hyp_mf, hyp_mf + 0.2 * rng.standard_normal(9) + np.array([0, 0, 0, 0, 0, 0, 0, 0, 20]))):
            cases.append((f"mf_n{n}_h{j}", "mf", n, h))
    for name, kind, n, h in cases:
        X, y = train[:n, :2].copy(), train[:n, 2:3].copy()
        if kind == "sf":
            m = gp.SFGP(X, y, 1)
        else:
            m = gp.MFGP(prior[:, :2].copy(), prior[:, 2:3].copy(), X, y, 1, 1)
        val = m.likelihood(h.copy())
        fd = np.zeros(h.shape[0])
        for p in range(h.shape[0]):
            e = np.zeros(h.shape[0])
            e[p] = 1e-6
            fd[p] = (m.likelihood(h + e) - m.likelihood(h - e)) / 2e-6
        out[name + "_hyp"] = h
        out[name + "_n"] = np.array(n)
        out[name + "_nlml"] = np.array(val)
        out[name + "_fdgrad"] = fd
    out["cases"] = np.array([c[0] for c in cases])
    np.savez_compressed(os.path.join(OUT, "nlml_reference.npz"), **out)
    print("wrote nlml_reference.npz,", len(cases), "cases")


SIM_CASES = {
    # name: (algorithm, data set, fidelity (hyp file), prior file or None, agents, iterations, seeds)
    "a6_todescato_hmf": ("todescato", "australia6", "mf", "australia6_prior.csv", 4, 14, (0, 1, 2)),
    "a6_todescato_hsf": ("todescato", "australia6", "sf", "australia6_prior.csv", 4, 14, (0, 1)),
    "a6_periodic_nmf": ("periodic", "australia6", "mf", None, 4, 14, (0, 1)),
    "a6_todescato_nsf": ("todescato", "australia6", "sf", None, 3, 12, (3,)),
}


def make_sim_fixture(sim):
    """7. ``sim_reference.npz``: the reference's own ``todescato`` / ``periodic``
    (simulator.py:788-954 / 618-785) on its australia6 data (51x51 grid), with its
    process-global generators replaced by the counter-based per-seed streams of
    ``mfgp_coverage_amd.coverage.SeedStreams`` (``random.random`` -> the explore
    stream, sim:943; ``np.random.default_rng()`` -> the noise stream, sim:877; the
    start positions of run_sim, runner.py:41-43, from the start stream), so the
    device drivers can replay the same draws. Stored per case and seed: the three
    logs encoded as float64 columns in the reference's key order
    (``runner.encode``), and per iteration and agent the gap between the largest
    and the second largest posterior variance inside the agent's Lloyd cell (the
    argmax that decides the next explore target: where the gap is below the parity
    tolerance the choice is decided by rounding, so the tests compare a
    trajectory only up to the first such iteration)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from mfgp_coverage_amd import runner
    from mfgp_coverage_amd.coverage import SeedStreams
    out = {}
    real_cmv, real_random, real_rng = sim.compute_max_var, sim.random, sim.np.random.default_rng
    real_arr = sim.np.array

    def arr(x, *a, **k):
        try:
            return real_arr(x, *a, **k)
        except ValueError:
            return real_arr(x, dtype=object)
    for name, (algo, data, fid, prior_file, agents, iterations, seeds) in SIM_CASES.items():
        truth = pd.read_csv(os.path.join(DATA, f"{data}_hifi.csv"))
        hyp = pd.read_csv(os.path.join(DATA, f"{data}_{fid}_hyp.csv"))
        prior = pd.read_csv(os.path.join(DATA, prior_file or "null_prior.csv"))
        out[name + "_truth"] = truth.values.astype(np.float64)
        out[name + "_hyp"] = hyp.values.astype(np.float64)[0]
        out[name + "_prior"] = prior.values.astype(np.float64).reshape(-1, 3)
        out[name + "_meta"] = np.array([agents, iterations, len(seeds)], dtype=np.int64)
        out[name + "_seeds"] = np.array(seeds, dtype=np.int64)
        for s in seeds:
            st = SeedStreams(s)
            gaps = []

            def cmv(vor, truth_arr, var_star):
                var = np.diag(var_star)
                g = []
                for cell in vor.filtered_regions:
                    v = vor.vertices[cell, :]
                    inside = sim.in_polygon(truth_arr[:, 0], truth_arr[:, 1], v[:, 0], v[:, 1])
                    iv = np.sort(var[inside])
                    g.append(iv[-1] - iv[-2] if iv.size > 1 else np.inf)
                gaps.append(g)
                return real_cmv(vor, truth_arr, var_star)
            sim.compute_max_var = cmv
            sim.random = types.SimpleNamespace(random=lambda: float(st.explore.random()))
            sim.np.random.default_rng = lambda *a, **k: st.noise
            sim.np.array = arr
            try:
                fn = sim.todescato if algo == "todescato" else sim.periodic
                logs = fn(name, s, iterations, agents, st.start_positions(agents), truth, 0.1, prior, hyp,
                          False, None, True)
            finally:
                sim.compute_max_var, sim.random, sim.np.random.default_rng = real_cmv, real_random, real_rng
                sim.np.array = real_arr
            for recs, cols, kind in zip(logs, runner.SCHEMAS, ("loss", "agent", "sample")):
                out[f"{name}_s{s}_{kind}"] = runner.encode(recs, cols)
            out[f"{name}_s{s}_gaps"] = np.array(gaps, dtype=np.float64)
            print(name, "seed", s, "samples", len(logs[2]), "min gap", np.min(gaps))
    out["cases"] = np.array(list(SIM_CASES))
    np.savez_compressed(os.path.join(OUT, "sim_reference.npz"), **out)


def make_log_headers():
    """6. ``log_headers.json``: the column headers of the reference's own logs
    (Data/atc24_choi_hmf_{loss,agent,sample}.csv), for the runner's CSV schemas."""
    import json
    out = {}
    for kind in ("loss", "agent", "sample"):
        out[kind] = list(pd.read_csv(os.path.join(DATA, f"atc24_choi_hmf_{kind}.csv"), nrows=2).columns)
    with open(os.path.join(OUT, "log_headers.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    if sys.argv[1:] == ["replays"]:   # CSV extraction only (no reference code)
        make_replay_fixtures()
        make_prior_fixtures()
        sys.exit(0)
    if sys.argv[1:] == ["sims"]:      # only the planner runs (sim_reference.npz)
        _import_reference()
        make_sim_fixture(_import_simulator())
        sys.exit(0)
    gp = _import_reference()
    make_reference_fixture(gp)
    make_replay_fixtures()
    sim = _import_simulator()
    make_choi_fixture(gp, sim)
    make_cells_fixture(sim)
    make_nlml_fixture(gp)
    make_log_headers()
    make_sim_fixture(sim)
