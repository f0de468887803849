"""MFGP_F32: the resident V = L^-1 psi^T stored and streamed in fp32 (BASELINE
configs[4], "Synthetic 256x256 grid, N_train=8192 MFGP, fp32, batched 32
independent agent GPs per GPU"); the factor, z, L21 / L22, the new rows' solve
and both reductions stay fp64. Checked against the fp64 oracle (the reference's
arithmetic, gp:401-438 / gp:493-529) at oracle.gp_oracle.F32_TOL with the
fp32 metric parity_errors_f32, and against the same library's fp64 models.

australia9_mf hyperparameters (noise 0.01 / 0.1): SURVEY.md section 8d names them
for configs[4] because the near-zero-noise hyp files are not fp32-safe.
"""
import numpy as np
import pytest

from oracle import gp_oracle as O

pytestmark = pytest.mark.gpu

TOL = O.F32_TOL


@pytest.fixture(scope="module")
def L():
    from mfgp_coverage_amd import _lib
    return _lib


def _hyp():
    from mfgp_coverage_amd.synthetic import HYP
    return HYP["australia9_mf"], HYP["australia3_sf"]


def _check(mu, var, mu_r, var_r, hyp, tol=TOL):
    e = O.parity_errors_f32(mu, var, mu_r, var_r, O.prior_variance(hyp))
    assert max(e) < tol, e
    return e


def _model(L, kind, hyp, dtype):
    return L.Model(L.context(), kind, hyp, 1e-8, dtype=dtype)


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("kind", ["mf", "sf"])
def test_f32_append_sequence_vs_oracle(L, kind, fused):
    """Full factor + predict (V computed in fp64, rounded into the fp32 V), then
    bordered appends of 1, 3, 8, 0, 15 and 16 rows (16: the MODE-1 stream that
    reads L21 from A), each predict against the oracle and against an fp64 model
    fed the same rows."""
    from mfgp_coverage_amd.synthetic import Workload
    hyp_mf, hyp_sf = _hyp()
    hyp = hyp_mf if kind == "mf" else hyp_sf
    w = Workload(40, 200 if kind == "mf" else 0, 150, 16, 7, seed=3)
    ctx = L.context()
    ctx.set_fused(fused)
    try:
        m32 = _model(L, L.MF if kind == "mf" else L.SF, hyp, L.F32)
        m64 = _model(L, L.MF if kind == "mf" else L.SF, hyp, L.F64)
        for m in (m32, m64):
            m.set_grid(w.xs)
            m.set_data(w.XL, w.yL, w.XH, w.yH)
        XH, yH = w.XH.copy(), w.yH.copy()
        for step, k in enumerate([None, 1, 3, 8, 0, 15, 16]):
            if k is not None:
                Xn, yn = w.Xnew[step][:k], w.ynew[step][:k]
                for m in (m32, m64):
                    m.append(Xn, yn)
                XH, yH = np.vstack([XH, Xn]), np.concatenate([yH, yn])
            mu, var = m32.predict()
            mu64, var64 = m64.predict()
            if kind == "mf":
                mu_r, var_r = O.mf_diag(w.XL, w.yL, XH, yH, hyp, w.xs)
            else:
                mu_r, var_r = O.sf_diag(XH, yH, hyp, w.xs)
            _check(mu, var, mu_r, var_r, hyp)
            _check(mu, var, mu64, var64, hyp)
        st = m32.stats()
        assert st["inc_factor"] >= 5 and st["vstream"] >= 5 and st["full_predict"] == 1, st
    finally:
        ctx.set_fused(True)


def test_f32_device_outputs_repredict_and_offgrid(L):
    """k = 0 re-predicts into device buffers (the MODE-0 stream), appends of points
    off the grid (the finish solves L21 and writes the fp32 compact rows), and
    capacity growth (the fp32 V rows move to the new row stride)."""
    import torch
    from mfgp_coverage_amd.synthetic import Workload
    hyp, _ = _hyp()
    w = Workload(32, 64, 40, 8, 40, seed=5)
    m = _model(L, L.MF, hyp, L.F32)
    m.set_grid(w.xs)
    m.set_data(w.XL, w.yL, w.XH, w.yH)
    M = w.xs.shape[0]
    mu_d = torch.empty(M, dtype=torch.float64, device="cuda")
    var_d = torch.empty(M, dtype=torch.float64, device="cuda")
    XH, yH = w.XH.copy(), w.yH.copy()
    rng = np.random.default_rng(0)
    for step in range(24):
        Xn, yn = w.Xnew[step], w.ynew[step]
        if step % 3 == 2:
            Xn = Xn + 0.3 / 31 * rng.random(Xn.shape)   # off the grid
        m.append(Xn, yn)
        XH, yH = np.vstack([XH, Xn]), np.concatenate([yH, yn])
        for _ in range(2):   # the second is the k = 0 re-predict
            L.batch_predict([m], mu_d.data_ptr(), var_d.data_ptr())
            mu, var = mu_d.cpu().numpy(), var_d.cpu().numpy()
            mu_r, var_r = O.mf_diag(w.XL, w.yL, XH, yH, hyp, w.xs)
            _check(mu, var, mu_r, var_r, hyp)
    st = m.stats()
    assert st["full_factor"] == 1 and st["inc_factor"] == 24, st
    assert st["full_predict"] == 1, st   # capacity grew (64 + 40 + 192 rows) on the incremental path


def test_f32_clone_sample_points(L):
    """The Choi planner loop (sim:326-374) on an fp32 model's device copy: every
    chosen point is the oracle's argmax given the points before it (to the
    tolerance's margin), and the model is unchanged."""
    from mfgp_coverage_amd.synthetic import Workload
    hyp, _ = _hyp()
    w = Workload(24, 30, 12, 1, 1, seed=9)
    m = _model(L, L.MF, hyp, L.F32)
    m.set_grid(w.xs)
    m.set_data(w.XL, w.yL, w.XH, w.yH)
    mu0, var0 = m.predict()
    thr = 0.5 * float(np.max(var0))
    pts = m.sample_points(thr, 40)
    assert 0 < pts.shape[0] <= 40
    XH, yH = w.XH.copy(), w.yH.copy()
    kss = O.prior_variance(hyp)
    for p in pts:
        mu_r, var_r = O.mf_diag(w.XL, w.yL, XH, yH, hyp, w.xs)
        j = int(np.argmin(np.abs(w.xs - p).sum(1)))
        assert var_r[j] >= np.max(var_r) - TOL * kss, (var_r[j], np.max(var_r))
        XH, yH = np.vstack([XH, p[None]]), np.concatenate([yH, mu_r[j:j + 1]])
    mu1, var1 = m.predict()
    np.testing.assert_array_equal(var1, var0)


def test_f32_batch_dtype_mismatch_rejected(L):
    import torch
    hyp, _ = _hyp()
    from mfgp_coverage_amd.synthetic import Workload
    w = Workload(16, 10, 10, 1, 1, seed=1)
    ms = []
    for dt in (L.F32, L.F64):
        m = _model(L, L.MF, hyp, dt)
        m.set_grid(w.xs)
        m.set_data(w.XL, w.yL, w.XH, w.yH)
        ms.append(m)
    out = torch.empty(2 * w.xs.shape[0], dtype=torch.float64, device="cuda")
    with pytest.raises(ValueError, match="dtype"):
        L.batch_predict(ms, out.data_ptr(), out.data_ptr())


def test_f32_mirror_precision_attribute():
    """The SFGP/MFGP mirror takes precision = "f32" per instance."""
    from mfgp_coverage_amd import gaussian_process as G
    from mfgp_coverage_amd.synthetic import Workload
    hyp, _ = _hyp()
    w = Workload(20, 30, 20, 4, 1, seed=2)
    m = G.MFGP(w.XL, w.yL.reshape(-1, 1), w.XH, w.yH.reshape(-1, 1), 1, 1)
    m.precision = "f32"
    m.hyp = hyp
    m.updt_info(m.X_L, m.y_L, m.X_H, m.y_H)
    m.updt_hifi(w.Xnew[0], w.ynew[0].reshape(-1, 1))
    mu, cov = m.predict(w.xs)
    assert m._dev().dtype == 1
    mu_r, var_r = O.mf_diag(w.XL, w.yL, m.X_H, m.y_H, hyp, w.xs)
    _check(mu[:, 0], np.diag(cov), mu_r, var_r, hyp)


@pytest.mark.parametrize("B", [8, 32])
def test_configs4_f32_batch_vs_oracle(L, B):
    """BASELINE configs[4]: 256x256 grid (M = 65536), N = 4096 lofi + 4096 hifi,
    australia9 MF, fp32 (MFGP_F32), at the config's own batch of 32 GPs per GPU
    and at 8: the full factor + predict (set_data, batch_predict), then three
    incremental steps of 8 new hifi rows per GP -- each ONE lattice-step launch
    (gp:401-438 / 493-529 via DESIGN.md section 2.4): k_inc_lat_arg (descriptors
    as the kernel argument) for 8 GPs, k_inc_lat (descriptors uploaded) for 32;
    the path counters assert which ran. The fused var max of every GP must equal
    the max of its variance; two GPs are checked against the oracle at every step
    on 2048 sampled cells plus the new samples' cells and the device argmax."""
    import torch
    from mfgp_coverage_amd.synthetic import Workload
    hyp, _ = _hyp()
    G, NL, NH0, k, steps = 256, 4096, 4088, 8, 3
    wls = [Workload(G, NL, NH0, k, steps, seed=100 + s) for s in range(B)]
    M = G * G
    ctx = L.context()
    models = []
    for w in wls:
        m = _model(L, L.MF, hyp, L.F32)
        m.set_grid(w.xs)
        m.set_data(w.XL, w.yL, w.XH, w.yH)
        models.append(m)
    mu_d = torch.empty(B * M, dtype=torch.float64, device="cuda")
    var_d = torch.empty(B * M, dtype=torch.float64, device="cuda")
    vmax = torch.empty(B, dtype=torch.float64, device="cuda")
    rng = np.random.default_rng(0)
    XH = [w.XH.copy() for w in wls]
    yH = [w.yH.copy() for w in wls]
    for step in range(steps + 1):
        if step == 0:
            L.batch_predict(models, mu_d.data_ptr(), var_d.data_ptr())
            new_cells = [np.empty(0, dtype=np.int64)] * B
        else:
            Xn = torch.from_numpy(np.concatenate([w.Xnew[step - 1] for w in wls])).cuda()
            yn = torch.from_numpy(np.concatenate([w.ynew[step - 1] for w in wls])).cuda()
            L.batch_append_predict(models, Xn.data_ptr(), yn.data_ptr(), [k] * B, mu_d.data_ptr(),
                                   var_d.data_ptr(), vmax_ptr=vmax.data_ptr())
            ctx.synchronize()
            for i, w in enumerate(wls):
                XH[i] = np.vstack([XH[i], w.Xnew[step - 1]])
                yH[i] = np.concatenate([yH[i], w.ynew[step - 1]])
            new_cells = [np.array([int(np.argmin(np.abs(w.xs - p).sum(1))) for p in w.Xnew[step - 1]])
                         for w in wls]
        mu = mu_d.cpu().numpy().reshape(B, M)
        var = var_d.cpu().numpy().reshape(B, M)
        assert np.all(np.isfinite(mu)) and np.all(np.isfinite(var))
        kss = O.prior_variance(hyp)
        assert np.all(var > 0) and np.all(var <= kss * (1 + 1e-6))
        if step > 0:
            np.testing.assert_array_equal(vmax.cpu().numpy(), var.max(axis=1))
        for i in (0, B - 1) if step in (0, steps) else (step % B,):
            pick = np.unique(np.concatenate([rng.choice(M, 2048, replace=False), new_cells[i],
                                             [int(np.argmax(var[i]))]]))
            w = wls[i]
            mu_r, var_r = O.mf_diag(w.XL, w.yL, XH[i], yH[i], hyp, w.xs[pick])
            _check(mu[i, pick], var[i, pick], mu_r, var_r, hyp)
    for m in models:
        st = m.stats()
        assert st["inc_factor"] == steps and st["vstream"] == steps and st["full_predict"] == 1, st
        # the first step also builds F, the tables and the axis tables (uploaded
        # descriptors); the next ones are single launches: by value for <= 8 GPs
        assert st["lattice"] == steps and st["lattice_arg"] == (steps - 1 if B <= 8 else 0), st
    del models
    ctx.trim()   # the fp64 scratch of the fp32 full predict (16 GB) is not kept
