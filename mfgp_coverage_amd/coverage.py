"""Coverage simulations on the device: the reference's Todescato and periodic
planners driving this package's GPs, one seed at a time or many in lockstep.

Reference (MSU-dcypherlab/mfgp-coverage): ``todescato`` (simulator.py:788-954),
``periodic`` (sim:618-785), ``run_sim`` (runner.py:33-69) and the helpers they
call -- ``voronoi_bounded`` (sim:154-191), ``todescato_prob`` (sim:457-467),
``periodic_decision`` (sim:492-500) and the Voronoi-cell reductions
(sim:194-323, here ``geometry`` / ``mfgp_batch_cell_reduce``).

Two drivers with the same per-seed semantics and log schemas (sim:918-931):

* ``simulate`` runs ONE seed through the drop-in API (``SFGP``/``MFGP``
  ``updt``/``updt_hifi``/``predict`` and ``geometry.compute_*``), statement for
  statement as the reference does -- its own process model (one simulation per
  process, runner.py:136).
* ``run_lockstep`` steps B seeds together ("each rank runs
  its seeds and batches their GPs per step"). Per iteration it issues ONE batched
  append + predict for all seeds (``mfgp_batch_append_predict``: the lattice step
  or the V stream over the whole batch in one launch; seeds whose agents all
  exploited append nothing and take their resident posterior, ``k_post_copy``),
  computes every seed's two bounded Voronoi partitions on the host while the GPU
  runs, and reduces all of their cells in ONE launch (``mfgp_batch_cell_reduce``:
  loss over the agents' partition with the truth, centroids and max variance over
  the Lloyd partition with the seed's own mean / variance, read in place from the
  batch's device outputs).

Randomness. The reference draws from process-global generators: ``random.random()``
for the start positions (runner.py:41-42) and the explore Bernoulli (sim:943), an
unseeded ``np.random.default_rng()`` for the sample noise (sim:877) -- its runs do
not repeat. Here every seed owns counter-based streams (Philox keyed by the seed
and the purpose), so a seed draws the same numbers in either driver, in any batch,
on any rank: the lockstep driver can be checked against the sequential one, a
sharded run produces the same logs as one process, and the reference itself can
be replayed with the same draws (tests/golden/make_golden.py patches its
generators with these streams).

Out of scope here: ``choi`` (its period plan is compute_sample_points, which the
device runs per seed -- planners.py -- followed by an mlrose TSP tour) and
``lloyd`` (no GP).
"""
from __future__ import annotations

import numpy as np

EPS = 0.1                      # simulator.py:33, the bounding-box cushion
ALGOS = ("todescato", "periodic")


# ---------------------------------------------------------------------------
# host geometry and decisions (the reference's helpers, restated)
# ---------------------------------------------------------------------------
class BoundedVoronoi:
    """What the planners read of the reference's ``vor``: ``vertices``,
    ``filtered_regions`` (vertex index lists, one per point inside the box) and
    ``filtered_points`` (sim:188-190)."""

    __slots__ = ("vertices", "filtered_regions", "filtered_points")

    def __init__(self, vertices, filtered_regions, filtered_points):
        self.vertices = vertices
        self.filtered_regions = filtered_regions
        self.filtered_points = filtered_points


def in_box(points, bounding_box):
    """sim:139-151: points within the box widened by EPS on every side."""
    return np.logical_and(np.logical_and(bounding_box[0] - EPS <= points[:, 0], points[:, 0] <= bounding_box[1] + EPS),
                          np.logical_and(bounding_box[2] - EPS <= points[:, 1], points[:, 1] <= bounding_box[3] + EPS))


def voronoi_bounded(points, bounding_box):
    """sim:154-191: the Voronoi partition of the points inside the box, bounded by
    mirroring them across the box's four sides (each mirror EPS further out), so
    that every inside point's region is closed. Qhull (scipy) on the host."""
    from scipy.spatial import Voronoi
    points = np.asarray(points, dtype=np.float64)
    bb = np.asarray(bounding_box, dtype=np.float64)
    c = points[in_box(points, bb), :]
    left, right, down, up = c.copy(), c.copy(), c.copy(), c.copy()
    left[:, 0] = bb[0] - (left[:, 0] - bb[0] + EPS)
    right[:, 0] = bb[1] + (bb[1] - right[:, 0] + EPS)
    down[:, 1] = bb[2] - (down[:, 1] - bb[2] + EPS)
    up[:, 1] = bb[3] + (bb[3] - up[:, 1] + EPS)
    vor = Voronoi(np.vstack([c, left, right, down, up]))
    # (sim:190: the regions of the first fifth of the points, the centre ones)
    regions = [vor.regions[r] for r in vor.point_region[:vor.npoints // 5]]
    return BoundedVoronoi(vor.vertices, regions, c)


def _roll1(a):
    """np.roll(a, 1) of a 1-D array (the same array, built without np.roll's overhead)."""
    return np.concatenate((a[-1:], a[:-1]))


def poly_area(x, y):
    """sim:127-136 (Shoelace)."""
    return 0.5 * np.abs(np.dot(x, _roll1(y)) - np.dot(y, _roll1(x)))


def todescato_prob(max_var_t, max_var_0):
    """sim:457-467: probability of exploring, per agent."""
    num_agents = max_var_t.shape[0]
    return np.sqrt(max_var_t / (max_var_0 * num_agents))


def periodic_decision(iteration):
    """sim:492-500: every agent explores for 5 iterations, then exploits for 5."""
    return (iteration // 5) % 2 == 0


def fidelity_of(hyp):
    """sim:647-652 / 817-822."""
    n = np.asarray(hyp).reshape(-1).shape[0]
    if n == 4:
        return "S"
    if n == 9:
        return "M"
    raise TypeError("Hyperparameters must be of length 4 (single-fidelity) or 9 (multi-fidelity)")


class SeedStreams:
    """The random draws of one simulation, as counter-based streams (numpy Philox
    keyed by (seed, purpose)): ``start`` for the agents' start positions
    (runner.py:41-43: all x, then all y), ``noise`` for the sample noise (sim:877,
    one normal per exploring agent in agent order), ``explore`` for the Bernoulli
    explore decisions (sim:943, one uniform per agent in agent order)."""

    def __init__(self, sim_num, key=0):
        base = (int(key) << 48) + 4 * int(sim_num)
        self.start = np.random.Generator(np.random.Philox(key=base))
        self.noise = np.random.Generator(np.random.Philox(key=base + 1))
        self.explore = np.random.Generator(np.random.Philox(key=base + 2))

    def start_positions(self, agents):
        x = self.start.random(agents)
        y = self.start.random(agents)
        return np.column_stack((x, y))

    def sample_noise(self, sigma_n):
        return self.noise.normal(loc=0, scale=sigma_n)

    def explore_draws(self, agents):
        return self.explore.random(agents)


def _prior_arrays(prior):
    """init_SFGP / init_MFGP (sim:47-102): the prior's (x, y) and value columns, or empty."""
    if prior is not None and len(prior) > 0:
        p = np.asarray(prior, dtype=np.float64).reshape(-1, 3)
        return np.reshape(p[:, [0, 1]], (-1, 2)), np.reshape(p[:, 2], (-1, 1))
    return np.empty([0, 2]), np.empty([0, 1])


class TruthIndex:
    """The rows of ``truth_arr`` by exact (x, y): the selection sim:874-877 makes
    with ``(truth_arr[:, 0] == x) & (truth_arr[:, 1] == y)`` over every row (the
    same rows in the same order: float keys compare as ``==`` does, 0.0 and -0.0
    alike), looked up instead of scanned."""

    def __init__(self, truth_arr):
        self.rows = {}
        for i, (x, y) in enumerate(zip(truth_arr[:, 0].tolist(), truth_arr[:, 1].tolist())):
            self.rows.setdefault((x, y), []).append(i)
        self.none = np.empty(0, dtype=np.int64)

    def __call__(self, x, y):
        r = self.rows.get((float(x), float(y)))
        return self.none if r is None else np.asarray(r, dtype=np.int64)


def _sample(truth_arr, x_sample, streams, sigma_n, index=None):
    """sim:874-877: the truth at the agent's grid cell plus noise."""
    if index is None:
        sample_idx = np.logical_and(truth_arr[:, 0] == x_sample[0], truth_arr[:, 1] == x_sample[1])
    else:
        sample_idx = index(x_sample[0], x_sample[1])
    return truth_arr[sample_idx, 2] + streams.sample_noise(sigma_n)


def _log_iteration(logs, sim_num, iteration, period, fidelity, loss_t, positions, argmax_var_t, max_var_t,
                   max_var_0, centroids_t, prob_explore_t, explore_t, distance, x_new, y_new, id_new):
    """sim:917-931 (the dict schemas, key order included; "YMax" logs the agent's
    own y as the reference does)."""
    loss_log, agent_log, sample_log = logs
    loss_log.append({"SimNum": sim_num, "Iteration": iteration, "Period": period,
                     "Fidelity": fidelity, "Loss": loss_t})
    for i in range(positions.shape[0]):
        agent_log.append({"SimNum": sim_num, "Iteration": iteration, "Period": period,
                          "Fidelity": fidelity, "Agent": i,
                          "X": positions[i, 0], "Y": positions[i, 1],
                          "XMax": argmax_var_t[i, 0], "YMax": positions[i, 1],
                          "VarMax": max_var_t[i, 0], "Var0": max_var_0,
                          "XCentroid": centroids_t[i, 0], "YCentroid": centroids_t[i, 1],
                          "ProbExplore": prob_explore_t[i, 0], "Explore": explore_t[i, 0],
                          "Distance": distance[i, 0]})
    for i in range(id_new.size):
        sample_log.append({"SimNum": sim_num, "Iteration": iteration, "Period": period, "Fidelity": fidelity,
                           "Agent": id_new[i, 0], "X": x_new[i, 0], "Y": x_new[i, 1], "Sample": y_new[i, 0]})


def _decide(algo, iteration, max_var_t, max_var_0, streams, agents):
    """sim:941-943 (todescato) / sim:771-774 (periodic): next iteration's explore decisions."""
    if algo == "todescato":
        prob_explore_t = todescato_prob(max_var_t, max_var_0)
        draws = streams.explore_draws(agents)
        explore_t = np.array([int(u < cutoff[0]) for u, cutoff in zip(draws, prob_explore_t)]).reshape(-1, 1)
    else:
        explore_bool = periodic_decision(iteration)
        prob_explore_t = np.array([int(explore_bool) for _ in range(agents)]).reshape(-1, 1)
        explore_t = np.array([int(explore_bool) for _ in range(agents)]).reshape(-1, 1)
    return prob_explore_t, explore_t


class Replay:
    """A logged run to replay (the reference's own, tests/golden/sim_reference.npz):
    at every iteration the drivers take the agents' positions, the samples and the
    Lloyd partition's seeds from the log instead of their own decisions, so each
    iteration's GP step, cell reduction and logged values (VarMax, XMax, centroids,
    loss) can be compared with the logged ones wherever rounding would otherwise
    have decided a discrete choice (an explorer's near-tie argmax, a grid point on a
    cell edge) and parted the runs. ``agent_log`` / ``sample_log``: the encoded logs
    (runner.encode, runner.AGENT_COLUMNS / SAMPLE_COLUMNS) of one seed."""

    def __init__(self, agent_log, sample_log):
        from . import runner
        A, S = runner.AGENT_COLUMNS, runner.SAMPLE_COLUMNS
        self._a, self._s = np.asarray(agent_log, dtype=np.float64), np.asarray(sample_log, dtype=np.float64)
        self._ai = {c: A.index(c) for c in ("Iteration", "Agent", "X", "Y", "XCentroid", "YCentroid",
                                            "ProbExplore", "Explore")}
        self._si = {c: S.index(c) for c in ("Iteration", "Agent", "X", "Y", "Sample")}

    def _rows(self, t):
        r = self._a[self._a[:, self._ai["Iteration"]] == t]
        return r[np.argsort(r[:, self._ai["Agent"]], kind="stable")]

    def positions(self, t):
        """the agents' positions logged at iteration t [agents, 2]"""
        r = self._rows(t)
        return r[:, [self._ai["X"], self._ai["Y"]]].copy()

    def lloyd_seeds(self, t):
        """the Lloyd partition's seeds at t: the centroids logged at t - 1 (at t = 0
        the start positions, as sim:862-863 initialises centroids_t)"""
        if t == 0:
            return self.positions(0)
        r = self._rows(t - 1)
        return r[:, [self._ai["XCentroid"], self._ai["YCentroid"]]].copy()

    def decisions(self, t):
        """(prob_explore_t, explore_t) logged at t (decided at t - 1) [agents, 1] each"""
        r = self._rows(t)
        return (r[:, [self._ai["ProbExplore"]]].copy(), r[:, [self._ai["Explore"]]].copy())

    def samples(self, t):
        """(x_new [k, 2], y_new [k, 1], id_new [k, 1]) logged at t, in log order"""
        s = self._s[self._s[:, self._si["Iteration"]] == t]
        return (s[:, [self._si["X"], self._si["Y"]]].copy(), s[:, [self._si["Sample"]]].copy(),
                s[:, [self._si["Agent"]]].copy())


def _algo(name):
    for a in ALGOS:
        if a in name:
            return a
    raise ValueError(f"lockstep / device simulations cover {ALGOS}, not {name!r}")


# ---------------------------------------------------------------------------
# one seed through the drop-in API (the reference's process model)
# ---------------------------------------------------------------------------
def simulate(algo, sim_num, iterations, agents, truth_arr, sigma_n, prior, hyp, positions=None, streams=None,
             log=True, forced=None):
    """todescato() / periodic() (sim:788-954 / 618-785) of one seed, with this
    package's SFGP / MFGP and device cell reductions. ``truth_arr`` [M, 3] (x, y,
    f) as in sim:833, ``prior`` [P, 3] or None, ``hyp`` the 4 / 9 log-scaled
    hyperparameters. ``forced``: a ``Replay`` whose positions, samples, Lloyd seeds
    and decisions replace the run's own at every iteration. Returns (loss_log,
    agent_log, sample_log)."""
    from . import geometry
    from .gaussian_process import MFGP, SFGP
    algo = _algo(algo)
    streams = streams or SeedStreams(sim_num)
    positions = np.array(streams.start_positions(agents) if positions is None else positions, dtype=np.float64)
    hyp = np.asarray(hyp, dtype=np.float64).reshape(-1)
    fidelity = fidelity_of(hyp)
    logs = ([], [], [])

    def init(prior_):
        X, y = _prior_arrays(prior_)
        if fidelity == "S":
            m = SFGP(X, y, 1)
        else:
            m = MFGP(X, y, np.empty([0, 2]), np.empty([0, 1]), 1, 1)
        m.hyp = hyp.copy()
        return m

    # 1-3) the empty model's max variance: the normalising constant (sim:827-843)
    truth_arr = np.asarray(truth_arr, dtype=np.float64)
    tindex = TruthIndex(truth_arr)
    model = init(None)
    x_star = truth_arr[:, [0, 1]]
    bounding_box = np.array([np.amin(x_star[:, 0]), np.amax(x_star[:, 0]),
                             np.amin(x_star[:, 1]), np.amax(x_star[:, 1])])
    mu_star, var_star = model.predict(x_star)
    max_var_0 = np.amax(var_star)
    # 4-5) the model conditioned on the prior (sim:845-861)
    model = init(prior)
    if fidelity == "S":
        model.updt_info(model.X, model.y)
    else:
        model.updt_info(model.X_L, model.y_L, model.X_H, model.y_H)
    mu_star, var_star = model.predict(x_star)
    var = np.diag(var_star)
    max_var_t = np.amax(var) * np.ones((agents, 1))
    prob_explore_t = todescato_prob(max_var_t, max_var_0) if algo == "todescato" else np.zeros((agents, 1))
    explore_t = np.zeros((agents, 1))
    prev_positions = np.copy(positions)
    centroids_t = np.copy(positions)
    period = 0
    for iteration in range(iterations):
        if forced is not None:
            positions = forced.positions(iteration)
            centroids_t = forced.lloyd_seeds(iteration)
            prev_positions = forced.positions(iteration - 1) if iteration > 0 else positions
            prob_explore_t, explore_t = forced.decisions(iteration)
        # 7) samples of the exploring agents (sim:868-885)
        x_new, y_new, id_new = np.empty([0, 2]), np.empty([0, 1]), np.empty([0, 1])
        for i in range(agents):
            if forced is None and explore_t[i] == 1:
                x_sample = positions[i, :]
                y_sample = _sample(truth_arr, x_sample, streams, sigma_n, tindex)
                x_new = np.vstack((x_new, x_sample))
                y_new = np.vstack((y_new, y_sample))
                id_new = np.vstack((id_new, i))
        if forced is not None:
            x_new, y_new, id_new = forced.samples(iteration)
        distance = np.sqrt(np.sum((positions - prev_positions) ** 2, axis=1)).reshape(-1, 1)
        # 8) update and predict (sim:887-892)
        if fidelity == "S":
            model.updt(x_new, y_new)
        else:
            model.updt_hifi(x_new, y_new)
        mu_star, var_star = model.predict(x_star)
        # 9-11) loss, centroids, max variance (sim:894-904)
        loss_vor = voronoi_bounded(positions, bounding_box)
        loss_t = geometry.compute_loss(loss_vor, truth_arr)
        # (every agent exploited: it stands on its centroid, so the two partitions are
        # of the same points -- the same partition, computed once)
        lloyd_vor = loss_vor if np.array_equal(positions, centroids_t) else voronoi_bounded(centroids_t, bounding_box)
        centroids_t = geometry.compute_centroids(lloyd_vor, x_star, mu_star)
        argmax_var_t, max_var_t = geometry.compute_max_var(lloyd_vor, truth_arr, var_star)
        if log:
            _log_iteration(logs, sim_num, iteration, period, fidelity, loss_t, positions, argmax_var_t, max_var_t,
                           max_var_0, centroids_t, prob_explore_t, explore_t, distance, x_new, y_new, id_new)
        # 13-14) decisions and moves (sim:941-951)
        prob_explore_t, explore_t = _decide(algo, iteration, max_var_t, max_var_0, streams, agents)
        prev_positions = np.copy(positions)
        for i in range(agents):
            if explore_t[i, 0]:
                positions[i, :] = argmax_var_t[i, :]
            else:
                positions[i, :] = centroids_t[i, :]
    return logs


# ---------------------------------------------------------------------------
# B seeds in lockstep (one batched GP step and one cell reduction per iteration)
# ---------------------------------------------------------------------------
def _cells_of(vor):
    regions = [list(r) for r in vor.filtered_regions]
    verts = [np.asarray(vor.vertices, dtype=np.float64)[r, :] for r in regions]
    return verts, np.asarray(vor.filtered_points, dtype=np.float64)


class LockstepStats:
    """Where the lockstep driver's wall time went (seconds, summed over iterations)."""

    def __init__(self):
        self.gp = 0.0          # enqueue of the batched append + predict
        self.voronoi = 0.0     # host Qhull (overlaps the GP step on the device)
        self.cells = 0.0       # the batched cell reduction (waits for the GP step)
        self.host = 0.0        # samples, logs, decisions
        self.iterations = 0
        self.seeds = 0
        self.rows = 0          # hifi rows appended, all seeds
        self.post_copy = 0     # seed-steps that appended nothing (resident posterior)

    def as_dict(self):
        return dict(self.__dict__)


def run_lockstep(algo, sim_nums, iterations, agents, truth_arr, sigma_n, prior, hyp, log=True, ctx=None,
                 stats=None, key=0, forced=None):
    """todescato() / periodic() (sim:788-954 / 618-785) for the seeds ``sim_nums``
    stepped together on the device. Same arguments as ``simulate`` (one truth,
    prior and hyperparameter set for all seeds, as runner.py:131-132 passes them;
    ``forced``: one ``Replay`` per seed, as in ``simulate``).
    Returns one (loss_log, agent_log, sample_log) per seed, in ``sim_nums`` order;
    each equals ``simulate`` of that seed up to the rounding of the batched kernels.
    """
    import time

    import torch

    from . import _lib
    algo = _algo(algo)
    sims = [int(s) for s in sim_nums]
    B = len(sims)
    if B == 0:
        return []
    ctx = ctx or _lib.context()
    dev = torch.device("cuda", int(ctx.device))
    hyp = np.asarray(hyp, dtype=np.float64).reshape(-1)
    fidelity = fidelity_of(hyp)
    kind = _lib.SF if fidelity == "S" else _lib.MF
    truth_arr = np.ascontiguousarray(truth_arr, dtype=np.float64)
    x_star = np.ascontiguousarray(truth_arr[:, [0, 1]])
    M = x_star.shape[0]
    bounding_box = np.array([np.amin(x_star[:, 0]), np.amax(x_star[:, 0]),
                             np.amin(x_star[:, 1]), np.amax(x_star[:, 1])])
    streams = [SeedStreams(s, key) for s in sims]
    positions = [st.start_positions(agents) for st in streams]
    tindex = TruthIndex(truth_arr)
    grid_lo = np.array([x_star[:, 0].min(), x_star[:, 1].min()])   # (the centroids' clamp, sim:276-281)
    grid_hi = np.array([x_star[:, 0].max(), x_star[:, 1].max()])
    e2, e1 = np.empty((0, 2)), np.empty(0)
    st_ = stats if stats is not None else LockstepStats()
    st_.seeds += B

    # 1-3) the empty model's max variance (sim:827-843): the prior variance
    # everywhere; the same for every seed (one hyperparameter set)
    empty = _lib.Model(ctx, kind, hyp, 1e-8)
    empty.set_grid(x_star)
    empty.set_data(e2, e1, e2, e1)
    _, var0 = empty.predict()
    max_var_0 = np.amax(var0)
    del empty
    # 4-5) the models conditioned on the prior (sim:845-861), predicted as one batch
    Xp, yp = _prior_arrays(prior)
    models = []
    for _ in range(B):
        m = _lib.Model(ctx, kind, hyp, 1e-8)
        m.set_grid(x_star)
        if fidelity == "S":
            m.set_data(e2, e1, Xp, yp.reshape(-1))
        else:
            m.set_data(Xp, yp.reshape(-1), e2, e1)
        models.append(m)
    mu = torch.empty(B * M, dtype=torch.float64, device=dev)
    var = torch.empty(B * M, dtype=torch.float64, device=dev)
    # the grid and the truth stay on the device for the cell reductions
    truth_f = torch.from_numpy(np.ascontiguousarray(truth_arr[:, 2])).to(dev)
    grid_d = torch.from_numpy(x_star).to(dev)
    mu_p, var_p, f_p, g_p = mu.data_ptr(), var.data_ptr(), truth_f.data_ptr(), grid_d.data_ptr()
    torch.cuda.synchronize(dev)
    _lib.batch_append_predict(models, 0, 0, [0] * B, mu_p, var_p)
    var_h = var.cpu().numpy().reshape(B, M)
    max_var_t = [np.amax(var_h[b]) * np.ones((agents, 1)) for b in range(B)]
    prob_explore_t = [todescato_prob(mv, max_var_0) if algo == "todescato" else np.zeros((agents, 1))
                      for mv in max_var_t]
    explore_t = [np.zeros((agents, 1)) for _ in range(B)]
    prev_positions = [np.copy(p) for p in positions]
    centroids_t = [np.copy(p) for p in positions]
    period = 0
    logs = [([], [], []) for _ in range(B)]
    for iteration in range(iterations):
        t0 = time.perf_counter()
        if forced is not None:
            for b in range(B):
                positions[b] = forced[b].positions(iteration)
                centroids_t[b] = forced[b].lloyd_seeds(iteration)
                prev_positions[b] = forced[b].positions(iteration - 1) if iteration > 0 else positions[b]
                prob_explore_t[b], explore_t[b] = forced[b].decisions(iteration)
        # 7) every seed's samples (sim:868-885)
        x_new, y_new, id_new, dist = [], [], [], []
        for b in range(B):
            xb, yb, ib = np.empty([0, 2]), np.empty([0, 1]), np.empty([0, 1])
            if forced is not None:
                xb, yb, ib = forced[b].samples(iteration)
            for i in range(agents):
                if forced is None and explore_t[b][i] == 1:
                    x_sample = positions[b][i, :]
                    y_sample = _sample(truth_arr, x_sample, streams[b], sigma_n, tindex)
                    xb = np.vstack((xb, x_sample))
                    yb = np.vstack((yb, y_sample))
                    ib = np.vstack((ib, i))
            x_new.append(xb)
            y_new.append(yb)
            id_new.append(ib)
            dist.append(np.sqrt(np.sum((positions[b] - prev_positions[b]) ** 2, axis=1)).reshape(-1, 1))
        ks = [xb.shape[0] for xb in x_new]
        Xc = np.ascontiguousarray(np.vstack(x_new), dtype=np.float64)
        Yc = np.ascontiguousarray(np.vstack(y_new).reshape(-1), dtype=np.float64)
        t1 = time.perf_counter()
        # 8) one batched append + predict for all seeds, left running (sim:887-892)
        _lib.batch_append_predict(models, Xc.ctypes.data if Xc.size else 0, Yc.ctypes.data if Yc.size else 0,
                                  ks, mu_p, var_p, asynchronous=True)
        t2 = time.perf_counter()
        # 9-10) every seed's two partitions, on the host while the GPU runs (sim:895, 900)
        cells, seeds, field, nloss = [], [], [], []
        for b in range(B):
            lv, lp = _cells_of(voronoi_bounded(positions[b], bounding_box))
            # (a seed whose agents all exploited stands on its centroids: one partition)
            same = np.array_equal(positions[b], centroids_t[b])
            gv, gp = (lv, lp) if same else _cells_of(voronoi_bounded(centroids_t[b], bounding_box))
            nloss.append(len(lv))
            cells.extend(lv + gv)
            seeds.append(np.vstack([lp, gp]))
            field.extend([b] * (len(lv) + len(gv)))
        vstart = np.zeros(len(cells) + 1, dtype=np.int32)
        vstart[1:] = np.cumsum([v.shape[0] for v in cells])
        t3 = time.perf_counter()
        # 9-11) all cells of all seeds in one launch, reading each seed's posterior in
        # place (after the GP step on the same stream); then the step's status
        out, am = _lib.batch_cell_reduce(g_p, np.vstack(cells), vstart, np.vstack(seeds), field, B,
                                         w=mu_p, f=f_p, var=var_p, ctx=ctx, M=M)
        ctx.synchronize()   # LinAlgError here if a seed's factor was not positive definite
        t4 = time.perf_counter()
        c0 = 0
        lo, hi = grid_lo, grid_hi
        for b in range(B):
            nl = nloss[b]
            ng = len(seeds[b]) - nl
            # compute_loss (sim:194-228)
            loss_t = 0
            with np.errstate(invalid="ignore", divide="ignore"):
                for i in range(nl):
                    v = cells[c0 + i]
                    loss_t += (out[c0 + i, 4] / out[c0 + i, 0]) * poly_area(v[:, 0], v[:, 1])
            # compute_centroids (sim:231-283) and compute_max_var (sim:286-323)
            cen = np.empty((ng, 2))
            amax = np.empty((ng, 2))
            vmax = np.empty((ng, 1))
            with np.errstate(invalid="ignore", divide="ignore"):
                for i in range(ng):
                    j = c0 + nl + i
                    v = cells[j]
                    area = poly_area(v[:, 0], v[:, 1])
                    n = out[j, 0]
                    f_integral = (out[j, 1] / n) * area
                    weighted = np.array([out[j, 2] / n, out[j, 3] / n]) * area
                    cen[i] = np.minimum(np.maximum(weighted / f_integral, lo), hi)
                    if am[j] < 0:
                        raise ValueError("zero-size array to reduction operation maximum which has no identity")
                    amax[i] = truth_arr[am[j], [0, 1]]
                    vmax[i, 0] = out[j, 5]
            c0 += nl + ng
            centroids_t[b] = cen
            max_var_t[b] = vmax
            if log:
                _log_iteration(logs[b], sims[b], iteration, period, fidelity, loss_t, positions[b], amax, vmax,
                               max_var_0, cen, prob_explore_t[b], explore_t[b], dist[b], x_new[b], y_new[b],
                               id_new[b])
            # 13-14) decisions and moves (sim:941-951)
            prob_explore_t[b], explore_t[b] = _decide(algo, iteration, vmax, max_var_0, streams[b], agents)
            prev_positions[b] = np.copy(positions[b])
            for i in range(agents):
                positions[b][i, :] = amax[i, :] if explore_t[b][i, 0] else cen[i, :]
        t5 = time.perf_counter()
        st_.gp += t2 - t1
        st_.voronoi += t3 - t2
        st_.cells += t4 - t3
        st_.host += (t1 - t0) + (t5 - t4)
        st_.iterations += 1
        st_.rows += int(sum(ks))
        st_.post_copy += int(sum(1 for k in ks if k == 0))
    return logs


def run(algo, simulations, iterations, agents, truth_arr, sigma_n, prior, hyp, world=1, rank=0, group=None,
        device=None, out_name=None, lockstep=True, blocks=None, key=0, stats=None):
    """runner.run (runner.py:72-161) of the device simulations: this rank's
    contiguous block of seeds (``ensemble.shard_seeds``) stepped in lockstep (or one
    at a time through the drop-in API with ``lockstep=False``), the three logs
    gathered on rank 0 in two collectives and written as ``<out_name>_{loss,agent,
    sample}.csv``. ``blocks`` (one process only): run the seeds as that many
    lockstep batches one after the other -- the batches a ``world = blocks`` run
    would form, so its logs are the same bits (a seed's numbers depend on the batch
    it is stepped in through the kernels' rounding only)."""
    from . import runner
    from .ensemble import shard_seeds
    if blocks is not None and world != 1:
        raise ValueError("blocks is for one process (it replays a world = blocks sharding)")
    nblk = blocks or 1

    def sims_of(r, w):
        return shard_seeds(simulations, w, r)

    def sim_logs():
        out = []
        groups = [sims_of(r, nblk) for r in range(nblk)] if blocks else [sims_of(rank, world)]
        for g in groups:
            if lockstep:
                out.extend(run_lockstep(algo, g, iterations, agents, truth_arr, sigma_n, prior, hyp, key=key,
                                        stats=stats))
            else:
                out.extend(simulate(algo, s, iterations, agents, truth_arr, sigma_n, prior, hyp,
                                    streams=SeedStreams(s, key)) for s in g)
        return out

    per_seed = sim_logs()
    logs = ([], [], [])
    for part in per_seed:
        for acc, recs in zip(logs, part):
            acc.extend(recs)
    tables = runner.gather_tables([runner.encode(recs, cols) for recs, cols in zip(logs, runner.SCHEMAS)], world,
                                  group, device)
    if rank != 0:
        return None
    dfs = [runner.decode(t, cols) for t, cols in zip(tables, runner.SCHEMAS)]
    if out_name:
        for df, kind in zip(dfs, ("loss", "agent", "sample")):
            df.to_csv(f"{out_name}_{kind}.csv")
    return tuple(dfs)
