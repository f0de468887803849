"""The seed-sharded runner (runner.py:72-161 with the log schemas of
simulator.py:918-931): gloo world 2 on CPU gives the same logs, in seed order,
as one process, and the CSVs have the reference's headers
(tests/golden/log_headers.json, from the reference's own Data/*.csv)."""
import io
import json
import os
import socket

import numpy as np
import pandas as pd
import torch.distributed as dist
import torch.multiprocessing as mp

from mfgp_coverage_amd import runner

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _sim(sim_num):
    """A stand-in simulation with the reference's log records (a varying number of
    samples per iteration, two fidelities)."""
    rng = np.random.default_rng(sim_num)
    fid = "M" if sim_num % 2 else "S"
    loss, agent, sample = [], [], []
    for it in range(4):
        loss.append({"SimNum": sim_num, "Iteration": it, "Period": it // 2, "Fidelity": fid, "Loss": rng.random()})
        for a in range(3):
            x, y = rng.random(2)
            agent.append({"SimNum": sim_num, "Iteration": it, "Period": it // 2, "Fidelity": fid, "Agent": a,
                          "X": x, "Y": y, "XMax": rng.random(), "YMax": y, "VarMax": rng.random(), "Var0": 0.08,
                          "XCentroid": rng.random(), "YCentroid": rng.random(), "ProbExplore": rng.random(),
                          "Explore": float(rng.random() > 0.5), "Distance": rng.random()})
        for _ in range(int(rng.integers(0, 3))):
            sample.append({"SimNum": sim_num, "Iteration": it, "Period": it // 2, "Fidelity": fid,
                           "Agent": float(rng.integers(0, 3)), "X": rng.random(), "Y": rng.random(),
                           "Sample": rng.random()})
    return loss, agent, sample


def _worker(rank, world, port, sims, out_dir, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = runner.run(_sim, sims, world=world, rank=rank, out_name=os.path.join(out_dir, "dist"))
    if rank == 0:
        q.put(tuple(df.to_json() for df in res))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_runner_gloo_matches_single_process(tmp_path):
    sims, world = 5, 2
    single = runner.run(_sim, sims, out_name=str(tmp_path / "single"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sims, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for df, js in zip(single, got):
        pd.testing.assert_frame_equal(df, pd.read_json(io.StringIO(js)), check_dtype=False)
    # same CSVs from one process and from two
    for kind in ("loss", "agent", "sample"):
        a = (tmp_path / f"single_{kind}.csv").read_text()
        b = (tmp_path / f"dist_{kind}.csv").read_text()
        assert a == b


def test_runner_headers_and_summary(tmp_path):
    with open(os.path.join(GOLDEN, "log_headers.json")) as f:
        ref = json.load(f)
    runner.run(_sim, 3, out_name=str(tmp_path / "r"))
    for kind in ("loss", "sample"):
        assert list(pd.read_csv(tmp_path / f"r_{kind}.csv", nrows=1).columns) == ref[kind]
    # the code's agent record (sim:926-929) adds Distance after the logged files' columns
    assert list(pd.read_csv(tmp_path / "r_agent.csv", nrows=1).columns) == ref["agent"] + ["Distance"]
    loss = pd.read_csv(tmp_path / "r_loss.csv", index_col=0)
    mean, std = runner.loss_summary(loss, "t")
    np.testing.assert_allclose(mean["t"].values, loss.groupby("Iteration")["Loss"].mean().values)
    np.testing.assert_allclose(std["t"].values, loss.groupby("Iteration")["Loss"].std().values)
