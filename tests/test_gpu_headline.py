"""The headline step itself, pinned to the oracle at its own shape and over a long
chain: BASELINE configs[3] per GPU -- 8 australia8 MF GPs on
the 128x128 grid, N_L = 1024 lofi + N_H = 1016 hifi rows, 8 new agent samples per
step -- with the library's DEFAULT gates (nothing forced). At B = 8 the 256 GEMM
tiles of the lattice step fill the chip once, so every lattice step runs as two
launches (k_inc_lat[_arg]: producers, w, Z; k_lat_gemm2[_arg]: the GEMM and the
cells), each from the previous step's resident posterior (gp:401-438 / 493-529 /
531-542 restated incrementally).

300 steps, a third of the new rows revisiting cells sampled before (the
reference's Todescato loop re-samples an explorer's cell, simulator.py:872-891),
so the chain crosses the lattice depth limit (LAT_MAXD = 256: step 257 is the V
stream refreshing the posterior from V) and several capacity growths. Checked
against oracle.mf_diag: every cell of two GPs at steps 1 / 128 / 256 / 257 / 258 /
300, and for all eight GPs 2048 sampled cells plus the argmax cell; the fused
np.amax / np.argmax of every GP at those steps; and the path counters (every step
but 257 a lattice step as two launches, all but the F-building ones with the
descriptors as the kernel argument).
"""
import numpy as np
import pytest

from oracle import gp_oracle as O

pytestmark = pytest.mark.gpu

TOL = O.PARITY_TOL
MAXD = 256   # mfgp_capi.hip LAT_MAXD
CHECK = (1, 128, 256, 257, 258, 300)


@pytest.mark.timeout(1200)
def test_headline_two_launch_chain_vs_oracle():
    import torch
    from mfgp_coverage_amd import _lib
    from mfgp_coverage_amd.synthetic import HYP, Workload
    hyp = HYP["australia8_mf"]
    B, K, NL, NH0, STEPS, G = 8, 8, 1024, 1016, 300, 128
    ctx = _lib.context()
    ctx.set_lattice(True)   # the default gate
    wls = [Workload(G, NL, NH0, K, STEPS, seed=400 + i, revisit=1 / 3) for i in range(B)]
    xs = wls[0].xs
    M = xs.shape[0]
    models = []
    for w in wls:
        m = _lib.Model(ctx, _lib.MF, hyp, 1e-8)
        m.set_grid(w.xs)
        m.set_data(w.XL, w.yL, w.XH, w.yH)
        models.append(m)
    mu = torch.empty(B * M, dtype=torch.float64, device="cuda")
    var = torch.empty(B * M, dtype=torch.float64, device="cuda")
    vmax = torch.empty(B, dtype=torch.float64, device="cuda")
    varg = torch.empty(B, dtype=torch.int64, device="cuda")
    _lib.batch_predict(models, mu.data_ptr(), var.data_ptr())   # the posterior of the base rows
    X = torch.from_numpy(np.ascontiguousarray(np.stack([w.Xnew for w in wls], 1))).cuda()   # [S, B, K, 2]
    Y = torch.from_numpy(np.ascontiguousarray(np.stack([w.ynew for w in wls], 1))).cuda()
    batch = _lib.Batch(models, [K] * B)
    rng = np.random.default_rng(5)
    prev = {"lattice": 0, "lattice_g2": 0, "vstream": 0}
    s_prev = 0
    for s in range(1, STEPS + 1):
        batch.append_predict(X[s - 1].data_ptr(), Y[s - 1].data_ptr(), mu.data_ptr(), var.data_ptr(),
                             asynchronous=True, vmax_ptr=vmax.data_ptr(), vargmax_ptr=varg.data_ptr())
        if s not in CHECK:
            continue
        ctx.synchronize()
        st = models[0].stats()
        n = s - s_prev
        refresh = 1 if s_prev < MAXD + 1 <= s else 0   # step 257: the V-stream refresh
        assert st["vstream"] - prev["vstream"] == n, (s, st)
        assert st["lattice"] - prev["lattice"] == n - refresh, (s, st)
        assert st["lattice_g2"] - prev["lattice_g2"] == n - refresh, (s, st)
        prev, s_prev = {k: st[k] for k in prev}, s
        mu_h, var_h = mu.cpu().numpy().reshape(B, M), var.cpu().numpy().reshape(B, M)
        np.testing.assert_array_equal(vmax.cpu().numpy(), var_h.max(axis=1))
        np.testing.assert_array_equal(varg.cpu().numpy(), var_h.argmax(axis=1))
        for i in range(B):
            w = wls[i]
            XH = np.vstack([w.XH, w.Xnew[:s].reshape(-1, 2)])
            yH = np.concatenate([w.yH, w.ynew[:s].reshape(-1)])
            if i < 2:
                pick = np.arange(M)   # every cell
            else:
                pick = np.unique(np.concatenate([rng.choice(M, 2048, replace=False), [int(np.argmax(var_h[i]))]]))
            mu_r, var_r = O.mf_diag(w.XL, w.yL, XH, yH, hyp, xs[pick])
            e = O.parity_errors(mu_h[i, pick], var_h[i, pick], mu_r, var_r, O.prior_variance(hyp))
            assert max(e) < TOL, (s, i, e)
    for m, w in zip(models, wls):
        st = m.stats()
        assert st["inc_factor"] == STEPS and st["full_predict"] == 1, st
        assert st["lattice"] == STEPS - 1 and st["lattice_g2"] == STEPS - 1, st
        # the steps that build F (the first one, the one after the refresh) upload
        # their descriptors; all others pass them as the kernel argument
        assert st["lattice_arg"] >= STEPS - 3, st
        XH = np.vstack([w.XH, w.Xnew.reshape(-1, 2)])
        assert np.unique(XH, axis=0).shape[0] < XH.shape[0]   # revisits are in the data
