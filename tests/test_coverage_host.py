"""Host side of the device coverage simulations (mfgp_coverage_amd/coverage.py), on
the CPU: the restated voronoi_bounded against the reference's own partitions, and
the per-seed random streams against the reference's runs that were made with them
(tests/golden/sim_reference.npz: simulator.py's todescato / periodic with their
process-global generators replaced by SeedStreams, make_golden.make_sim_fixture).
The GP and cell reductions of those runs are checked on the GPU
(tests/test_gpu_coverage.py)."""
import numpy as np
import pytest

from mfgp_coverage_amd import coverage as C
from mfgp_coverage_amd import runner
from tests import _fixtures as F

SIM = F.load("sim_reference.npz")


def _col(arr, cols, name):
    return arr[:, cols.index(name)]


def test_voronoi_bounded_equals_reference_partitions():
    """The cells of the reference's voronoi_bounded (sim:154-191) on the 12 partitions
    of cells_reference.npz: same polygons, vertex for vertex, cell for cell."""
    fx = F.load("cells_reference.npz")
    truth = fx["truth"]
    xs = truth[:, :2]
    bb = np.array([xs[:, 0].min(), xs[:, 0].max(), xs[:, 1].min(), xs[:, 1].max()])
    for c in range(int(fx["ncases"])):
        seeds = fx[f"c{c}_seeds"]
        vor = C.voronoi_bounded(seeds, bb)
        np.testing.assert_array_equal(vor.filtered_points, seeds)
        vs, verts = fx[f"c{c}_vstart"], fx[f"c{c}_verts"]
        assert len(vor.filtered_regions) == vs.shape[0] - 1
        for i, r in enumerate(vor.filtered_regions):
            np.testing.assert_array_equal(vor.vertices[r, :], verts[vs[i]:vs[i + 1]])


def test_voronoi_bounded_filters_points_outside_the_box():
    """sim:165-167: only points within the box (widened by EPS) seed cells."""
    pts = np.array([[0.2, 0.3], [0.7, 0.8], [1.5, 0.5], [0.5, -0.05]])
    vor = C.voronoi_bounded(pts, np.array([0.0, 1.0, 0.0, 1.0]))
    np.testing.assert_array_equal(vor.filtered_points, pts[[0, 1, 3]])
    assert len(vor.filtered_regions) == 3


def test_decisions_and_fidelity():
    mv = np.array([[0.04], [0.01]])
    np.testing.assert_allclose(C.todescato_prob(mv, 0.08), np.sqrt(mv / 0.16))
    assert [C.periodic_decision(i) for i in (0, 4, 5, 9, 10)] == [True, True, False, False, True]
    assert C.fidelity_of(np.zeros(4)) == "S" and C.fidelity_of(np.zeros(9)) == "M"
    with pytest.raises(TypeError):
        C.fidelity_of(np.zeros(5))


def test_seed_streams_are_per_seed():
    """A seed's draws do not depend on which other seeds exist or in what order they draw."""
    a = C.SeedStreams(5)
    b = C.SeedStreams(5)
    other = C.SeedStreams(6)
    other.explore_draws(3)
    np.testing.assert_array_equal(a.start_positions(4), b.start_positions(4))
    np.testing.assert_array_equal(a.explore_draws(4), np.array([b.explore.random() for _ in range(4)]))
    assert a.sample_noise(0.1) == b.sample_noise(0.1)
    assert not np.array_equal(C.SeedStreams(5).start_positions(4), C.SeedStreams(6).start_positions(4))
    assert not np.array_equal(C.SeedStreams(5, key=1).start_positions(4), C.SeedStreams(5).start_positions(4))


@pytest.mark.parametrize("case", [str(c) for c in SIM["cases"]])
def test_reference_runs_used_the_seed_streams(case):
    """The golden runs draw exactly what SeedStreams gives: start positions (runner.py:
    41-43), one noise draw per sample in log order (sim:877), and the explore decisions
    of todescato (sim:942-943: int(u < sqrt(VarMax / (Var0 agents))) per agent, u from
    the explore stream) -- the protocol both device drivers follow."""
    agents, iterations, _ = (int(v) for v in SIM[case + "_meta"])
    truth = SIM[case + "_truth"]
    A, S = runner.AGENT_COLUMNS, runner.SAMPLE_COLUMNS
    for s in SIM[case + "_seeds"]:
        st = C.SeedStreams(int(s))
        ag, sa = SIM[f"{case}_s{s}_agent"], SIM[f"{case}_s{s}_sample"]
        it0 = _col(ag, A, "Iteration") == 0
        np.testing.assert_array_equal(np.column_stack([_col(ag, A, "X"), _col(ag, A, "Y")])[it0],
                                      st.start_positions(agents))
        for row in sa:
            x, y = row[S.index("X")], row[S.index("Y")]
            cell = (truth[:, 0] == x) & (truth[:, 1] == y)
            assert cell.sum() == 1
            assert row[S.index("Sample")] == truth[cell, 2][0] + st.sample_noise(0.1)
        if "todescato" in case:
            for t in range(iterations - 1):
                cur, nxt = ag[_col(ag, A, "Iteration") == t], ag[_col(ag, A, "Iteration") == t + 1]
                prob = C.todescato_prob(_col(cur, A, "VarMax").reshape(-1, 1), _col(cur, A, "Var0")[0])
                np.testing.assert_allclose(_col(nxt, A, "ProbExplore"), prob[:, 0], rtol=1e-15)
                u = st.explore_draws(agents)
                np.testing.assert_array_equal(_col(nxt, A, "Explore"), (u < prob[:, 0]).astype(float))


def test_truth_index_selects_the_mask_rows():
    """TruthIndex picks the rows sim:874-877's exact-equality mask picks: the same
    rows in the same order, duplicates and a signed zero included, none for a
    point off the grid."""
    from mfgp_coverage_amd import coverage as C
    g = np.linspace(0.0, 1.0, 17)
    xs = np.array([(a, b) for a in g for b in g])
    truth = np.column_stack([xs, np.arange(xs.shape[0], dtype=np.float64)])
    truth = np.vstack([truth, [[0.5, 0.25, -1.0]], [[-0.0, 0.0, -2.0]]])   # a duplicate, a signed zero
    ti = C.TruthIndex(truth)
    probes = [xs[i] for i in range(0, xs.shape[0], 7)] + [np.array([0.5, 0.25]), np.array([0.0, -0.0]),
                                                       np.array([0.5, 0.2500000001])]
    for p in probes:
        mask = np.logical_and(truth[:, 0] == p[0], truth[:, 1] == p[1])
        assert np.array_equal(truth[mask, 2], truth[ti(p[0], p[1]), 2]), p
        a = C._sample(truth, p, C.SeedStreams(3), 0.1)
        b = C._sample(truth, p, C.SeedStreams(3), 0.1, ti)
        assert a.shape == b.shape and np.array_equal(a, b), p


@pytest.mark.parametrize("case", [str(c) for c in SIM["cases"]])
def test_replay_reads_the_reference_logs(case):
    """coverage.Replay (the forced replay of tests/test_gpu_coverage.py) hands the
    drivers the reference's own state: positions at t are the moves of t - 1 (an
    explorer to its logged argmax XMax -- the reference logs the agent's own y as
    "YMax", so the y is checked against the position -- an exploiter to its logged
    centroid, sim:945-951); the Lloyd seeds at t are the centroids of t - 1 (the
    start positions at t = 0); the samples at t sit at the explorers' positions."""
    agents, iterations, _ = (int(v) for v in SIM[case + "_meta"])
    A = runner.AGENT_COLUMNS
    for s in SIM[case + "_seeds"]:
        ag, sa = SIM[f"{case}_s{s}_agent"], SIM[f"{case}_s{s}_sample"]
        rp = C.Replay(ag, sa)
        np.testing.assert_array_equal(rp.lloyd_seeds(0), rp.positions(0))
        for t in range(iterations):
            pos = rp.positions(t)
            assert pos.shape == (agents, 2)
            _, explore = rp.decisions(t)
            xn, yn, idn = rp.samples(t)
            assert xn.shape[0] == yn.shape[0] == idn.shape[0] == int(explore.sum())
            np.testing.assert_array_equal(xn, pos[idn[:, 0].astype(int)])
            if t == 0:
                continue
            prev = ag[_col(ag, A, "Iteration") == t - 1]
            prev = prev[np.argsort(_col(prev, A, "Agent"), kind="stable")]
            cen = np.column_stack([_col(prev, A, "XCentroid"), _col(prev, A, "YCentroid")])
            np.testing.assert_array_equal(rp.lloyd_seeds(t), cen)
            for i in range(agents):
                if explore[i, 0]:
                    assert pos[i, 0] == _col(prev, A, "XMax")[i]
                else:
                    np.testing.assert_array_equal(pos[i], cen[i])
