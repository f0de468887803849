"""The seed-sharded runner (runner.py:72-161, log schemas simulator.py:918-931)
driving device GPs: each simulation is a miniature Todescato loop (as in
tests/test_gpu_loop.py: predict, VarMax = np.amax(cov) (sim:1014), bounded
Voronoi cells, compute_loss / compute_centroids on the device, move, sample,
MFGP.updt_hifi on the bordered path) logging the reference's loss / agent /
sample records. Two gloo ranks sharing the GPU must produce the same logs as
one process, and every logged VarMax must equal the oracle's max posterior
variance given the samples logged before it."""
import os
import socket

import numpy as np
import pandas as pd
import pytest

from oracle import gp_oracle as O

pytestmark = pytest.mark.gpu

SIMS, G, AGENTS, STEPS, NL, NH = 4, 32, 3, 10, 60, 12


def _device_sim(sim_num):
    from mfgp_coverage_amd import geometry
    from mfgp_coverage_amd.gaussian_process import MFGP
    from mfgp_coverage_amd.synthetic import HYP, Workload, field
    from tests.test_gpu_loop import _bounded_voronoi, _nearest_cells
    hyp = HYP["australia8_mf"]
    w = Workload(G, NL, NH, 1, 1, seed=sim_num)
    xs = w.xs
    rng = np.random.default_rng(100 + sim_num)
    truth = field(xs, rng.random((4, 2)))
    truth_arr = np.column_stack([xs, truth])
    noise = 0.1 * rng.standard_normal((STEPS, AGENTS))
    pos = xs[rng.choice(xs.shape[0], AGENTS, replace=False)]
    gp = MFGP(w.XL.copy(), w.yL.reshape(-1, 1).copy(), w.XH.copy(), w.yH.reshape(-1, 1).copy(), 1, 1)
    gp.hyp = hyp.copy()
    gp.updt_info(gp.X_L, gp.y_L, gp.X_H, gp.y_H)
    var0 = O.prior_variance(hyp)
    loss_log, agent_log, sample_log = [], [], []
    for t in range(STEPS):
        mu, cov = gp.predict(xs)
        var_max = float(np.amax(cov))
        jmax = int(np.argmax(np.diag(cov)))
        vor = _bounded_voronoi(pos, (0.0, 1.0, 0.0, 1.0))
        loss = geometry.compute_loss(vor, truth_arr)
        cen = geometry.compute_centroids(vor, xs, mu)
        cells = _nearest_cells(xs, cen)
        rec = {"SimNum": sim_num, "Iteration": t, "Period": 0, "Fidelity": "M"}
        loss_log.append(dict(rec, Loss=loss))
        new = xs[cells]
        for a in range(AGENTS):
            agent_log.append(dict(rec, Agent=a, X=pos[a, 0], Y=pos[a, 1], XMax=xs[jmax, 0], YMax=xs[jmax, 1],
                                  VarMax=var_max, Var0=var0, XCentroid=cen[a, 0], YCentroid=cen[a, 1],
                                  ProbExplore=0.0, Explore=0.0, Distance=float(np.hypot(*(new[a] - pos[a])))))
        y_new = truth[cells] + noise[t]
        gp.updt_hifi(new, y_new.reshape(-1, 1))
        for a in range(AGENTS):
            sample_log.append(dict(rec, Agent=float(a), X=new[a, 0], Y=new[a, 1], Sample=y_new[a]))
        pos = new
    assert gp._dev().stats()["inc_factor"] >= STEPS
    return loss_log, agent_log, sample_log


def _worker(rank, world, port, out_dir, q):
    import torch.distributed as dist
    from mfgp_coverage_amd import runner
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = runner.run(_device_sim, SIMS, world=world, rank=rank, out_name=os.path.join(out_dir, "dist"))
    if rank == 0:
        q.put(tuple(df.to_json() for df in res))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_runner_device_sims_two_ranks_match_one(tmp_path):
    import io

    import torch.multiprocessing as mp
    from mfgp_coverage_amd import runner
    single = runner.run(_device_sim, SIMS, out_name=str(tmp_path / "single"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for df, js in zip(single, got):
        pd.testing.assert_frame_equal(df, pd.read_json(io.StringIO(js)), check_dtype=False, rtol=1e-12)
    for kind in ("loss", "agent", "sample"):
        assert (tmp_path / f"dist_{kind}.csv").exists()

    # VarMax against the oracle, iteration by iteration, from the logged samples
    from mfgp_coverage_amd.synthetic import HYP, Workload
    hyp = HYP["australia8_mf"]
    loss, agent, sample = single
    assert sorted(loss.SimNum.unique()) == list(range(SIMS))
    for s in range(SIMS):
        w = Workload(G, NL, NH, 1, 1, seed=s)
        for t in range(STEPS):
            prev = sample[(sample.SimNum == s) & (sample.Iteration < t)]
            XH = np.vstack([w.XH, prev[["X", "Y"]].to_numpy()])
            yH = np.concatenate([w.yH, prev["Sample"].to_numpy()])
            _, var_r = O.mf_diag(w.XL, w.yL, XH, yH, hyp, w.xs)
            vm = agent[(agent.SimNum == s) & (agent.Iteration == t)]["VarMax"].to_numpy()
            kss = O.prior_variance(hyp)
            assert np.all(np.abs(vm - var_r.max()) <= O.PARITY_TOL * max(var_r.max(), 1e-6 * kss)), (s, t)
