"""Grid-sharded predict of one GP (SURVEY.md 8e secondary mode; the X*-row split of
gaussian_process_numba.py:478-503): block bounds, and the all_gather of the blocks
over gloo world 2. The CPU tests give each rank an oracle-backed stand-in model.
The GPU test runs the real SFGP / MFGP on cuda:0 in two gloo ranks and compares
them with an unsharded predict, through an append whose new points lie in only one
rank's block."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from mfgp_coverage_amd.sharded import lattice_row, shard_cells
from oracle import gp_oracle as O

HYP_SF = np.array([0.0001, -2.797478161, -1.500619305, -4.6])
HYP_MF = np.array([0.16, -2.03, -0.63, 0.0001, -3.1, -1.52, -0.65, -5.0, -2.0])


def _grid(G):
    g = np.linspace(0.0, 1.0, G)
    return np.array([(a, b) for a in g for b in g])


def test_shard_cells_partition():
    for M, row in ((0, 1), (7, 1), (1024, 32), (1000, 32), (16384, 128), (51 * 51, 51)):
        for world in (1, 2, 3, 8):
            b = [shard_cells(M, world, r, row) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == M
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
            if M % row == 0:
                assert all(lo % row == 0 and hi % row == 0 for lo, hi in b)
                sizes = [(hi - lo) // row for lo, hi in b]
                assert max(sizes) - min(sizes) <= 1


def test_lattice_row():
    assert lattice_row(_grid(32)) == 32
    assert lattice_row(_grid(51)) == 51
    xs = _grid(16)
    assert lattice_row(xs[::-1]) == 16
    assert lattice_row(xs[:, ::-1]) == 1          # y-outer order: not the reference's layout
    rng = np.random.default_rng(0)
    assert lattice_row(rng.random((64, 2))) == 1
    assert lattice_row(np.empty((0, 2))) == 1


class _OracleSF:
    """Stand-in with the SFGP.predict contract, computed by the CPU oracle."""

    def __init__(self, X, y, hyp):
        self.X, self.y, self.hyp = X, y, hyp

    def predict(self, Xs):
        from mfgp_coverage_amd.gaussian_process import DiagCov
        mu, var = O.sf_diag(self.X, self.y, self.hyp, Xs)
        return mu.reshape(-1, 1), DiagCov(var)


def _data(G, N, seed):
    rng = np.random.default_rng(seed)
    Xs = _grid(G)
    X = Xs[rng.choice(Xs.shape[0], N, replace=False)]
    y = np.sin(3 * X[:, :1]) + 0.1 * rng.standard_normal((N, 1))
    return Xs, X, y


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return sorted(res, key=lambda t: t[0])


def _cpu_worker(rank, world, port, q, G, N):
    import torch.distributed as dist

    from mfgp_coverage_amd.sharded import predict_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    Xs, X, y = _data(G, N, 1)
    mu, cov = predict_sharded(_OracleSF(X, y, HYP_SF), Xs)
    q.put((rank, mu, np.diag(cov)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,G", [(2, 20), (3, 17)])
def test_predict_sharded_gloo_oracle(world, G):
    res = _run(_cpu_worker, world, G, 40)
    Xs, X, y = _data(G, 40, 1)
    mu_r, var_r = O.sf_diag(X, y, HYP_SF, Xs)
    for _, mu, var in res:
        assert mu.shape == (G * G, 1)
        np.testing.assert_allclose(mu[:, 0], mu_r, rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(var, var_r, rtol=1e-10, atol=1e-15)


def _gpu_worker(rank, world, port, q, kind):
    import torch
    import torch.distributed as dist

    from mfgp_coverage_amd.gaussian_process import MFGP, SFGP
    from mfgp_coverage_amd.sharded import predict_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)                     # both ranks share the box's one GPU
    dist.init_process_group("gloo", rank=rank, world_size=world)
    Xs, X, y = _data(48, 180, 2)
    if kind == "sf":
        gp = SFGP(X[:170], y[:170], 1)
        gp.hyp = HYP_SF
        gp.updt_info(gp.X, gp.y)
    else:
        gp = MFGP(X[:90], y[:90], X[90:170], y[90:170], 1, 1)
        gp.hyp = HYP_MF
        gp.updt_info(gp.X_L, gp.y_L, gp.X_H, gp.y_H)
    out = []
    mu, cov = predict_sharded(gp, Xs)
    out.append((mu[:, 0], np.diag(cov)))
    # new samples on cells of the first rows only: rank 1's block does not hold them
    new = np.array([i * 48 + j for i, j in ((0, 3), (1, 40), (2, 7), (3, 20))])
    Xn, yn = Xs[new], np.cos(2 * Xs[new, :1])
    if kind == "sf":
        gp.updt(Xn, yn)
    else:
        gp.updt_hifi(Xn, yn)
    mu, cov = predict_sharded(gp, Xs)
    out.append((mu[:, 0], np.diag(cov)))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["sf", "mf"])
def test_predict_sharded_gpu_gloo(kind):
    from mfgp_coverage_amd.gaussian_process import MFGP, SFGP
    res = _run(_gpu_worker, 2, kind)
    Xs, X, y = _data(48, 180, 2)
    new = np.array([i * 48 + j for i, j in ((0, 3), (1, 40), (2, 7), (3, 20))])
    Xn, yn = Xs[new], np.cos(2 * Xs[new, :1])
    hyp = HYP_SF if kind == "sf" else HYP_MF
    if kind == "sf":
        refs = [O.sf_diag(X[:170], y[:170], hyp, Xs),
                O.sf_diag(np.vstack([X[:170], Xn]), np.vstack([y[:170], yn]), hyp, Xs)]
        gp = SFGP(X[:170], y[:170], 1)
        gp.hyp = hyp
        gp.updt_info(gp.X, gp.y)
    else:
        refs = [O.mf_diag(X[:90], y[:90], X[90:170], y[90:170], hyp, Xs),
                O.mf_diag(X[:90], y[:90], np.vstack([X[90:170], Xn]), np.vstack([y[90:170], yn]), hyp, Xs)]
        gp = MFGP(X[:90], y[:90], X[90:170], y[90:170], 1, 1)
        gp.hyp = hyp
        gp.updt_info(gp.X_L, gp.y_L, gp.X_H, gp.y_H)
    mu0, cov0 = gp.predict(Xs)
    kss = O.prior_variance(hyp)
    for _, out in res:
        for (mu, var), (mu_r, var_r) in zip(out, refs):
            assert max(O.parity_errors(mu, var, mu_r, var_r, kss)) < O.PARITY_TOL
    # the unsharded device predict of the same model: the same factor, so to rounding
    np.testing.assert_allclose(res[0][1][0][0], mu0[:, 0], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(res[1][1][0][1], np.diag(cov0), rtol=1e-7, atol=1e-13)


@pytest.mark.gpu
def test_predict_block_device_equals_predict():
    """The nccl path of predict_sharded: a rank's block predicted straight into a
    device tensor (no host round trip before the all_gather) holds the same bits as
    the host predict of that block, zero past it."""
    import torch
    from mfgp_coverage_amd.gaussian_process import MFGP
    from mfgp_coverage_amd.sharded import predict_block_device, shard_cells
    Xs, X, y = _data(48, 180, 2)
    gp = MFGP(X[:90], y[:90], X[90:170], y[90:170], 1, 1)
    gp.hyp = HYP_MF
    gp.updt_info(gp.X_L, gp.y_L, gp.X_H, gp.y_H)
    lo, hi = shard_cells(Xs.shape[0], 3, 1, 48)
    mmax = hi - lo + 48
    mine = predict_block_device(gp, Xs[lo:hi], mmax).cpu().numpy()
    mu, cov = gp.predict(Xs[lo:hi])
    assert np.array_equal(mine[0, :hi - lo], mu[:, 0]) and np.array_equal(mine[1, :hi - lo], np.diag(cov))
    assert not mine[:, hi - lo:].any()
