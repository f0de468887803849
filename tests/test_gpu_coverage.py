"""The coverage simulations on the device (mfgp_coverage_amd/coverage.py): the
drop-in driver (one seed through SFGP / MFGP, as the reference runs it) and the
lockstep driver (B seeds, one batched GP step and one batched cell reduction per
iteration) against

* the reference's OWN todescato / periodic runs (tests/golden/sim_reference.npz:
  simulator.py:788-954 / 618-785 on its australia6 data, made with the same
  per-seed random streams), log for log;
* each other, at the headline size (128x128, australia8 MF, 1024 lofi prior
  points, 8 agents) and on a 64x64 SF case;
* the same seeds sharded over two gloo ranks (byte-identical CSVs, uneven shards).

A trajectory is compared iteration by iteration up to the first place where the
two runs may legitimately part: an explorer's target is the argmax of the
posterior variance in its cell, and where the largest and second-largest variance
in that cell are closer than the parity tolerance the choice is decided by
rounding (tests/golden/make_golden.py records those gaps for the reference; for
two device runs the oracle recomputes them). A divergence anywhere else fails.
"""
import os
import socket

import numpy as np
import pytest

from mfgp_coverage_amd import runner
from oracle import gp_oracle as O
from tests import _fixtures as F

pytestmark = pytest.mark.gpu

TOL = O.PARITY_TOL
A, S = runner.AGENT_COLUMNS, runner.SAMPLE_COLUMNS
IT, AG, X, Y, XMAX, VMAX, V0, XC, YC, PE, EX = (A.index(c) for c in ("Iteration", "Agent", "X", "Y", "XMax", "VarMax",
                                                                       "Var0", "XCentroid", "YCentroid", "ProbExplore",
                                                                       "Explore"))


def _enc(logs):
    return tuple(runner.encode(recs, cols) for recs, cols in zip(logs, runner.SCHEMAS))


def _partition_flips(xs, seeds_r, seeds_g):
    """Do the bounded Voronoi partitions of two seed sets that agree to ~1e-9 (the
    two runs' positions or centroids) put some grid point into different cells?
    Only a grid point within rounding of a cell edge can move: in_polygon (sim:105-124)
    decides it, and the rounding of the runs' means decides the edge."""
    from mfgp_coverage_amd import coverage
    bb = np.array([xs[:, 0].min(), xs[:, 0].max(), xs[:, 1].min(), xs[:, 1].max()])
    vr, vg = coverage.voronoi_bounded(seeds_r, bb), coverage.voronoi_bounded(seeds_g, bb)
    for cr, cg in zip(vr.filtered_regions, vg.filtered_regions):
        if not np.array_equal(O.in_polygon(xs, vr.vertices[cr, :]), O.in_polygon(xs, vg.vertices[cg, :])):
            return True
    return False


STOPS = []
LOSS_FLIPS = []


def compare_runs(ref, got, kss, near_tie, xs):
    """ref, got: encoded (loss, agent, sample) logs of one seed; xs the grid.
    near_tie(t, a) -> True when agent a's cell argmax at iteration t is decided by
    rounding. Two runs may part only where rounding decides a discrete choice: an
    explorer's argmax (a near tie), or a grid point's cell when it lies on an edge
    of the partition of the centroids (the Lloyd step, sim:900-904) -- checked by
    recomputing both runs' partitions. An edge of the agents' partition through a
    grid point changes only that iteration's logged loss (sim:895-896; nothing
    feeds back), so the comparison goes on past it.
    Returns the number of iterations compared in full (before such a place); the
    reason it stopped is appended to STOPS."""
    lr, ar, sr = ref
    lg, ag, sg = got
    its = int(ar[:, IT].max()) + 1
    for t in range(its):
        r, g = ar[ar[:, IT] == t], ag[ag[:, IT] == t]
        assert r.shape == g.shape, t
        dpos = np.abs(r[:, [X, Y]] - g[:, [X, Y]]).max(axis=1)
        if np.any(dpos > 1e-9):
            # positions at t are the decisions of t - 1: an explorer's target may
            # differ only through a near tie of its cell's argmax
            for a in np.flatnonzero(dpos > 1e-9):
                assert t > 0 and r[a, EX] == 1 and g[a, EX] == 1, (t, a, r[a], g[a])
                assert near_tie(t - 1, a), (t, a, "diverged without a near tie")
            STOPS.append((t, "explorer's target: near tie"))
            return t
        srt, sgt = sr[sr[:, 1] == t], sg[sg[:, 1] == t]
        np.testing.assert_array_equal(srt, sgt, err_msg=f"samples at iteration {t}")
        np.testing.assert_allclose(g[:, V0], r[:, V0], rtol=1e-12)
        prev_r = ar[ar[:, IT] == t - 1][:, [XC, YC]] if t > 0 else r[:, [X, Y]]
        prev_g = ag[ag[:, IT] == t - 1][:, [XC, YC]] if t > 0 else g[:, [X, Y]]
        loss_ok = np.allclose(lg[lg[:, 1] == t, 4], lr[lr[:, 1] == t, 4], rtol=1e-9, atol=0)
        if not loss_ok:
            # (the loss is only logged, nothing feeds back: the comparison goes on)
            assert _partition_flips(xs, r[:, [X, Y]], g[:, [X, Y]]), (t, "loss differs without a partition flip")
            LOSS_FLIPS.append(t)
        err = np.abs(g[:, VMAX] - r[:, VMAX]) / np.maximum(np.abs(r[:, VMAX]), 1e-6 * kss)
        cen_ok = np.allclose(g[:, [XC, YC]], r[:, [XC, YC]], rtol=0, atol=1e-9)
        if err.max() >= TOL or not cen_ok:
            assert _partition_flips(xs, prev_r, prev_g), (t, err, "VarMax / centroids differ without a flip")
            STOPS.append((t, "Lloyd partition: grid point on an edge"))
            return t
        for a in np.flatnonzero(g[:, XMAX] != r[:, XMAX]):
            if not near_tie(t, a):
                assert _partition_flips(xs, prev_r, prev_g), (t, a, "argmax differs without a near tie")
                STOPS.append((t, "argmax: grid point on an edge"))
                return t
        np.testing.assert_allclose(g[:, PE], r[:, PE], rtol=1e-6, err_msg=f"ProbExplore {t}")
        np.testing.assert_array_equal(g[:, EX], r[:, EX], err_msg=f"Explore {t}")
    return its


# ---------------------------------------------------------------------------
# against the reference's own runs
# ---------------------------------------------------------------------------
SIM = F.load("sim_reference.npz")
CASES = [str(c) for c in SIM["cases"]]


def _case(case):
    agents, iterations, _ = (int(v) for v in SIM[case + "_meta"])
    prior = SIM[case + "_prior"]
    algo = "todescato" if "todescato" in case else "periodic"
    return algo, agents, iterations, SIM[case + "_truth"], (prior if prior.shape[0] else None), SIM[case + "_hyp"]


def _ref(case, s):
    return tuple(SIM[f"{case}_s{s}_{k}"] for k in ("loss", "agent", "sample"))


# per case: the mean number of iterations a natural (unforced) run of the seeds must
# be compared over. compare_runs stops at a rounding-decided choice that parts a run
# from the reference's; none did in round 5 (`pytest -s` prints RECORD: every seed of
# every case, both drivers, compared over all of its logged iterations -- 14, and 12
# for a6_todescato_nsf seed 3), so the floor is the whole run. RECORD keeps each
# seed's count and the reason its comparison stopped.
FLOOR = {"a6_todescato_hmf": 14, "a6_todescato_hsf": 14, "a6_periodic_nmf": 14, "a6_todescato_nsf": 12}
RECORD = {}


def _golden_tie(case, s, kss):
    gaps = SIM[f"{case}_s{s}_gaps"]
    return lambda t, a: gaps[t, a] < TOL * kss


@pytest.mark.parametrize("case", CASES)
def test_dropin_simulation_matches_reference_run(case):
    from mfgp_coverage_amd import coverage
    algo, agents, iterations, truth, prior, hyp = _case(case)
    kss = O.prior_variance(hyp)
    done = []
    for s in SIM[case + "_seeds"]:
        got = _enc(coverage.simulate(algo, int(s), iterations, agents, truth, 0.1, prior, hyp))
        n0 = len(STOPS)
        done.append(compare_runs(_ref(case, s), got, kss, _golden_tie(case, s, kss), truth[:, :2]))
        RECORD[("dropin", case, int(s))] = (done[-1], STOPS[-1][1] if len(STOPS) > n0 else "all iterations")
    print("compared (iterations, stop):", {k: v for k, v in RECORD.items() if k[:2] == ("dropin", case)})
    assert sum(done) >= FLOOR[case] * len(done), (done, STOPS[-len(done):])


@pytest.mark.parametrize("case", CASES)
def test_lockstep_simulation_matches_reference_run(case):
    from mfgp_coverage_amd import _lib, coverage
    algo, agents, iterations, truth, prior, hyp = _case(case)
    kss = O.prior_variance(hyp)
    seeds = [int(s) for s in SIM[case + "_seeds"]]
    stats = coverage.LockstepStats()
    logs = coverage.run_lockstep(algo, seeds, iterations, agents, truth, 0.1, prior, hyp, stats=stats)
    done = []
    for s, lg in zip(seeds, logs):
        n0 = len(STOPS)
        done.append(compare_runs(_ref(case, s), _enc(lg), kss, _golden_tie(case, s, kss), truth[:, :2]))
        RECORD[("lockstep", case, s)] = (done[-1], STOPS[-1][1] if len(STOPS) > n0 else "all iterations")
    print("compared (iterations, stop):", {k: v for k, v in RECORD.items() if k[:2] == ("lockstep", case)})
    assert sum(done) >= FLOOR[case] * len(done), (done, STOPS[-len(done):])
    assert stats.iterations == iterations and stats.seeds == len(seeds)


# ---------------------------------------------------------------------------
# forced replay of the reference's runs: every iteration compared
# ---------------------------------------------------------------------------
REPLAY = {}


def compare_replay(ref, got, kss, near_tie):
    """ref, got: encoded logs of one seed, got replayed from ref (coverage.Replay: the
    same positions, samples and Lloyd seeds at every iteration, so the partitions and
    the GP's data are the reference's). Every iteration must match: VarMax in the
    parity metric, the argmax cell (or a near tie of the reference's own top two
    variances in that cell, tests/golden), the centroids to 1e-9, the loss to 1e-9
    relative, Var0. Returns the iterations compared (all of them)."""
    lr, ar, sr = ref
    lg, ag, sg = got
    its = int(ar[:, IT].max()) + 1
    ties = 0
    for t in range(its):
        r, g = ar[ar[:, IT] == t], ag[ag[:, IT] == t]
        assert r.shape == g.shape, t
        np.testing.assert_array_equal(g[:, [X, Y]], r[:, [X, Y]], err_msg=f"positions {t}")
        np.testing.assert_array_equal(sg[sg[:, 1] == t], sr[sr[:, 1] == t], err_msg=f"samples {t}")
        np.testing.assert_allclose(g[:, V0], r[:, V0], rtol=1e-12)
        err = np.abs(g[:, VMAX] - r[:, VMAX]) / np.maximum(np.abs(r[:, VMAX]), 1e-6 * kss)
        assert err.max() < TOL, (t, err)
        np.testing.assert_allclose(g[:, [XC, YC]], r[:, [XC, YC]], rtol=0, atol=1e-9, err_msg=f"centroids {t}")
        np.testing.assert_allclose(lg[lg[:, 1] == t, 4], lr[lr[:, 1] == t, 4], rtol=1e-9, err_msg=f"loss {t}")
        for a in np.flatnonzero(g[:, XMAX] != r[:, XMAX]):
            assert near_tie(t, a), (t, a, "argmax differs without a near tie")
            ties += 1
    return its, ties


def _replays(case, seeds):
    from mfgp_coverage_amd import coverage
    return [coverage.Replay(SIM[f"{case}_s{s}_agent"], SIM[f"{case}_s{s}_sample"]) for s in seeds]


@pytest.mark.parametrize("case", CASES)
def test_dropin_replay_matches_reference_every_iteration(case):
    """the drop-in driver replaying the reference's own runs
    (positions, samples and Lloyd seeds forced from the logs) matches VarMax, argmax,
    centroids and loss at EVERY iteration of every seed."""
    from mfgp_coverage_amd import coverage
    algo, agents, iterations, truth, prior, hyp = _case(case)
    kss = O.prior_variance(hyp)
    seeds = [int(s) for s in SIM[case + "_seeds"]]
    for s, rp in zip(seeds, _replays(case, seeds)):
        got = _enc(coverage.simulate(algo, s, iterations, agents, truth, 0.1, prior, hyp, forced=rp))
        n, ties = compare_replay(_ref(case, s), got, kss, _golden_tie(case, s, kss))
        assert n == iterations, (case, s, n)
        REPLAY[("dropin", case, s)] = (n, ties)
    print("replay (iterations compared, argmax near ties):", {k: v for k, v in REPLAY.items() if k[1] == case})


@pytest.mark.parametrize("case", CASES)
def test_lockstep_replay_matches_reference_every_iteration(case):
    """The lockstep driver (one batched GP step and one batched cell reduction per
    iteration for all seeds) replaying the reference's runs: every iteration of every
    seed, as the drop-in replay above."""
    from mfgp_coverage_amd import coverage
    algo, agents, iterations, truth, prior, hyp = _case(case)
    kss = O.prior_variance(hyp)
    seeds = [int(s) for s in SIM[case + "_seeds"]]
    logs = coverage.run_lockstep(algo, seeds, iterations, agents, truth, 0.1, prior, hyp,
                                 forced=_replays(case, seeds))
    for s, lg in zip(seeds, logs):
        n, ties = compare_replay(_ref(case, s), _enc(lg), kss, _golden_tie(case, s, kss))
        assert n == iterations, (case, s, n)
        REPLAY[("lockstep", case, s)] = (n, ties)
    print("replay (iterations compared, argmax near ties):", {k: v for k, v in REPLAY.items() if k[1] == case})


# ---------------------------------------------------------------------------
# lockstep against the drop-in driver, seed by seed
# ---------------------------------------------------------------------------
def _oracle_tie(truth, prior, hyp, sample, agent_log, kss):
    """near_tie for two device runs: the oracle's posterior variance given the samples
    logged up to iteration t, in agent a's Lloyd cell at t (seeded by the centroids
    of t - 1, or the start positions at t = 0): largest minus second largest."""
    from mfgp_coverage_amd import coverage
    xs = truth[:, :2]
    bb = np.array([xs[:, 0].min(), xs[:, 0].max(), xs[:, 1].min(), xs[:, 1].max()])
    P = np.empty((0, 3)) if prior is None else prior

    def tie(t, a):
        sel = sample[sample[:, 1] <= t]
        Xn, yn = sel[:, [S.index("X"), S.index("Y")]], sel[:, S.index("Sample")]
        if hyp.shape[0] == 4:
            _, var = O.sf_diag(np.vstack([P[:, :2], Xn]), np.concatenate([P[:, 2], yn]), hyp, xs)
        else:
            _, var = O.mf_diag(P[:, :2], P[:, 2], Xn, yn, hyp, xs)
        prev = agent_log[agent_log[:, IT] == max(t - 1, 0)]
        seeds = prev[:, [XC, YC]] if t > 0 else prev[:, [X, Y]]
        vor = coverage.voronoi_bounded(seeds, bb)
        v = vor.vertices[vor.filtered_regions[a], :]
        iv = np.sort(var[O.in_polygon(xs, v)])
        return iv.size > 1 and iv[-1] - iv[-2] < TOL * kss
    return tie


@pytest.mark.parametrize("algo,kind", [("todescato", "mf"), ("periodic", "sf")])
def test_lockstep_equals_dropin_headline(algo, kind):
    """B = 4 seeds in lockstep vs the same seeds one at a time through the drop-in API:
    MF at the headline size (128x128, australia8, 1024 lofi prior points, 8 agents;
    the batch takes the lattice step) and SF at 64x64 (australia3, 121 prior points)."""
    from mfgp_coverage_amd import coverage
    from mfgp_coverage_amd.synthetic import HYP, Workload, field
    if kind == "mf":
        G, NL, agents, hyp = 128, 1024, 8, HYP["australia8_mf"]
    else:
        G, NL, agents, hyp = 64, 121, 4, HYP["australia3_sf"]
    iterations, seeds = 12, [10, 11, 12, 13]
    w = Workload(G, NL, 0, 1, 1, seed=7)
    rng = np.random.default_rng(3)
    truth = np.column_stack([w.xs, field(w.xs, rng.random((4, 2)))])
    prior = np.column_stack([w.XL, w.yL])
    kss = O.prior_variance(hyp)
    stats = coverage.LockstepStats()
    logs = coverage.run_lockstep(algo, seeds, iterations, agents, truth, 0.1, prior, hyp, stats=stats)
    done = []
    for s, lg in zip(seeds, logs):
        one = _enc(coverage.simulate(algo, s, iterations, agents, truth, 0.1, prior, hyp))
        tie = _oracle_tie(truth, prior, hyp, one[2], one[1], kss)
        done.append(compare_runs(one, _enc(lg), kss, tie, truth[:, :2]))
    assert sum(done) >= 0.6 * iterations * len(seeds), (done, STOPS[-len(done):])
    assert stats.rows > 0


# ---------------------------------------------------------------------------
# the runner: lockstep seeds sharded over ranks, logs gathered on rank 0
# ---------------------------------------------------------------------------
SHARD = dict(G=32, NL=60, agents=3, iterations=6, sims=5)


def _shard_inputs():
    from mfgp_coverage_amd.synthetic import HYP, Workload, field
    w = Workload(SHARD["G"], SHARD["NL"], 0, 1, 1, seed=5)
    truth = np.column_stack([w.xs, field(w.xs, np.random.default_rng(8).random((4, 2)))])
    return truth, np.column_stack([w.XL, w.yL]), HYP["australia8_mf"]


def _shard_worker(rank, world, port, out_dir, q):
    import torch.distributed as dist
    from mfgp_coverage_amd import coverage
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    truth, prior, hyp = _shard_inputs()
    coverage.run("todescato", SHARD["sims"], SHARD["iterations"], SHARD["agents"], truth, 0.1, prior, hyp,
                 world=world, rank=rank, out_name=os.path.join(out_dir, "dist"))
    dist.barrier()
    dist.destroy_process_group()
    q.put(rank)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_lockstep_runner_two_ranks_byte_identical(tmp_path):
    """5 seeds over two gloo ranks sharing the GPU (3 + 2: uneven) give the same CSV
    bytes as one process stepping the same two batches; the seeds are all there, in
    order, and each rank's batch took the lockstep path."""
    import torch.multiprocessing as mp
    from mfgp_coverage_amd import coverage
    truth, prior, hyp = _shard_inputs()
    single = coverage.run("todescato", SHARD["sims"], SHARD["iterations"], SHARD["agents"], truth, 0.1, prior, hyp,
                          blocks=2, out_name=str(tmp_path / "single"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == [0, 1]
    for kind in ("loss", "agent", "sample"):
        a = (tmp_path / f"single_{kind}.csv").read_bytes()
        b = (tmp_path / f"dist_{kind}.csv").read_bytes()
        assert a == b, kind
    loss = single[0]
    assert list(loss.SimNum.unique()) == list(range(SHARD["sims"]))
    assert (loss.groupby("SimNum").size() == SHARD["iterations"]).all()


# ---------------------------------------------------------------------------
# the two batched entry points the lockstep driver added
# ---------------------------------------------------------------------------
def test_batch_cell_reduce_equals_per_partition():
    """mfgp_batch_cell_reduce over three seeds' partitions (fields read in place from
    device buffers) equals mfgp_cell_reduce of each partition, bit for bit."""
    import torch
    from mfgp_coverage_amd import _lib, coverage
    from mfgp_coverage_amd.synthetic import grid
    xs = grid(40)
    M = xs.shape[0]
    rng = np.random.default_rng(2)
    B = 3
    w = rng.random((B, M))
    var = rng.random((B, M))
    f = rng.random(M)
    parts = [coverage.voronoi_bounded(rng.random((int(rng.integers(2, 7)), 2)), np.array([0, 1, 0, 1.0]))
             for _ in range(2 * B)]
    cells, seeds, field = [], [], []
    for j, vor in enumerate(parts):
        for r in vor.filtered_regions:
            cells.append(vor.vertices[r, :])
        seeds.append(vor.filtered_points)
        field.extend([j // 2] * len(vor.filtered_regions))
    vstart = np.concatenate([[0], np.cumsum([c.shape[0] for c in cells])]).astype(np.int32)
    wd = torch.from_numpy(w.reshape(-1)).cuda()
    vd = torch.from_numpy(var.reshape(-1)).cuda()
    out, am = _lib.batch_cell_reduce(xs, np.vstack(cells), vstart, np.vstack(seeds), field, B, w=wd.data_ptr(),
                                     f=f, var=vd.data_ptr())
    c0 = 0
    for j, vor in enumerate(parts):
        n = len(vor.filtered_regions)
        b = j // 2
        flat = np.vstack([vor.vertices[r, :] for r in vor.filtered_regions])
        vs = np.concatenate([[0], np.cumsum([len(r) for r in vor.filtered_regions])]).astype(np.int32)
        o1, a1 = _lib.cell_reduce(xs, flat, vs, vor.filtered_points, w=w[b], f=f, var=var[b])
        np.testing.assert_array_equal(out[c0:c0 + n], o1)
        np.testing.assert_array_equal(am[c0:c0 + n], a1)
        c0 += n


def test_unchanged_batch_members_take_the_resident_posterior():
    """A batch step in which some GPs append nothing: those return their previous
    posterior bit for bit (k_post_copy, with the fused max / argmax), the others still
    take one lattice launch, and both agree with the oracle."""
    import torch
    from mfgp_coverage_amd import _lib
    from mfgp_coverage_amd.synthetic import HYP, Workload
    hyp = HYP["australia8_mf"]
    B, K, G = 4, 8, 64
    wls = [Workload(G, 300, 0, K, 3, seed=90 + i) for i in range(B)]
    M = G * G
    ctx = _lib.context()
    ctx.set_lattice("force")
    try:
        models = []
        for w in wls:
            m = _lib.Model(ctx, _lib.MF, hyp, 1e-8)
            m.set_grid(w.xs)
            m.set_data(w.XL, w.yL, np.empty((0, 2)), np.empty(0))
            models.append(m)
        mu = torch.empty(B * M, dtype=torch.float64, device="cuda")
        var = torch.empty(B * M, dtype=torch.float64, device="cuda")
        vmax = torch.zeros(B, dtype=torch.float64, device="cuda")
        varg = torch.zeros(B, dtype=torch.int64, device="cuda")
        _lib.batch_append_predict(models, 0, 0, [0] * B, mu.data_ptr(), var.data_ptr())
        rows = [[] for _ in range(B)]
        prev = None
        for s in range(3):
            ks = [K if (b + s) % 2 == 0 else 0 for b in range(B)]
            Xn = np.vstack([wls[b].Xnew[s] for b in range(B) if ks[b]])
            yn = np.concatenate([wls[b].ynew[s] for b in range(B) if ks[b]])
            for b in range(B):
                if ks[b]:
                    rows[b].append(s)
            _lib.batch_append_predict(models, Xn.ctypes.data, yn.ctypes.data, ks, mu.data_ptr(), var.data_ptr(),
                                      vmax_ptr=vmax.data_ptr(), vargmax_ptr=varg.data_ptr())
            mu_h, var_h = mu.cpu().numpy().reshape(B, M), var.cpu().numpy().reshape(B, M)
            np.testing.assert_array_equal(vmax.cpu().numpy(), var_h.max(axis=1))
            np.testing.assert_array_equal(varg.cpu().numpy(), var_h.argmax(axis=1))
            for b in range(B):
                if prev is not None and ks[b] == 0:
                    np.testing.assert_array_equal(mu_h[b], prev[0][b])
                    np.testing.assert_array_equal(var_h[b], prev[1][b])
                w = wls[b]
                XH = w.Xnew[rows[b]].reshape(-1, 2)
                yH = w.ynew[rows[b]].reshape(-1)
                mu_r, var_r = O.mf_diag(w.XL, w.yL, XH, yH, hyp, w.xs)
                assert max(O.parity_errors(mu_h[b], var_h[b], mu_r, var_r, O.prior_variance(hyp))) < TOL, (s, b)
            prev = (mu_h, var_h)
        st = [m.stats() for m in models]
        # (the first batch predict wrote every member's resident posterior, so every
        # k = 0 member-step is a copy)
        assert [x["post_copy"] for x in st] == [1, 2, 1, 2], st
        assert [x["lattice"] for x in st] == [2, 1, 2, 1], st
    finally:
        ctx.set_lattice(True)
