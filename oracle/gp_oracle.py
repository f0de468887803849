"""CPU oracle for the GP posterior update -- TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product. Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
import it. The product path (``mfgp_coverage_amd``) never imports it and fails
loudly when its HIP library is missing.

It restates, in NumPy, the single hot path of MSU-dcypherlab/mfgp-coverage
(``/root/reference``):

* ``se_kernel``        <- ``SFGP.kernel`` gaussian_process.py:66-79
                          (``MFGP.kernel`` gaussian_process.py:329-342 is identical)
* ``sf_faithful``      <- ``SFGP.updt_info`` gp:229-255 + ``SFGP.predict`` gp:121-148,
                          same op sequence (dense K(X*,X*), four ``np.linalg.solve``,
                          dense ``psi @ beta``), returns ``diag`` of the covariance.
* ``mf_faithful``      <- ``MFGP.updt_info`` gp:493-529 + ``MFGP.predict`` gp:401-438.
* ``sf_diag``/``mf_diag`` -- the same math with a Cholesky, two triangular solves
                          and a row-sum of squares (no M x M matrices). This is the
                          semantic spec of the HIP kernels and the stronger CPU
                          baseline.

Pinning: ``tests/test_oracle.py`` checks this module
against golden vectors produced by importing the reference itself in the build
container (``tests/golden/make_golden.py``), against the reference's own logged
runs (``Data/*_agent.csv`` VarMax / Var0 replays), and against closed forms.

Hyperparameter layouts (log-scaled, simulator.py:53-56, 83-84):
  SF: [mu, s^2, L, noise]
  MF: [mu_lo, s^2_lo, L_lo, mu_hi, s^2_hi, L_hi, rho, noise_lo, noise_hi]
"""
from __future__ import annotations

import numpy as np
import scipy.linalg as sla

JITTER = 1e-8  # gaussian_process.py:42 (SF) and :298 (MF)


def se_kernel(x, xp, log_s2, log_l):
    """Squared-exponential kernel, gaussian_process.py:66-79.

    Scales before subtracting (``x/l - xp/l``, gp:77-78); ``s`` and ``l`` are the
    exponentiated log hyperparameters (gp:75-76).
    """
    output_scale = np.exp(log_s2)
    lengthscale = np.exp(log_l)
    diffs = np.expand_dims(x / lengthscale, 1) - np.expand_dims(xp / lengthscale, 0)
    return output_scale * np.exp(-0.5 * np.sum(diffs ** 2, axis=2))


# ---------------------------------------------------------------------------
# Reference-faithful restatements (same op sequence, dense covariance)
# ---------------------------------------------------------------------------

def sf_faithful(X, y, hyp, Xs, jitter=JITTER, return_cov=False):
    """SFGP.updt_info (gp:229-255) then SFGP.predict (gp:121-148)."""
    X = np.asarray(X, dtype=np.float64).reshape(-1, 2)
    y = np.asarray(y, dtype=np.float64).reshape(-1, 1)
    hyp = np.asarray(hyp, dtype=np.float64)
    N = y.shape[0]
    sigma_n = np.exp(hyp[-1])                                        # gp:248-249
    K = se_kernel(X, X, hyp[1], hyp[2]) + np.eye(N) * sigma_n        # gp:253
    L = np.linalg.cholesky(K + np.eye(N) * jitter)                  # gp:254
    mean = np.exp(hyp[0])                                            # gp:132
    yc = y - mean                                                    # gp:133
    psi = se_kernel(Xs, X, hyp[1], hyp[2])                           # gp:139
    alpha = np.linalg.solve(np.transpose(L), np.linalg.solve(L, yc))  # gp:141
    mu = np.matmul(psi, alpha) + mean                                # gp:142-143
    beta = np.linalg.solve(np.transpose(L), np.linalg.solve(L, psi.T))  # gp:145
    cov = se_kernel(Xs, Xs, hyp[1], hyp[2]) - np.matmul(psi, beta)   # gp:146
    if return_cov:
        return mu[:, 0], cov
    return mu[:, 0], np.diag(cov).copy()


def _mf_parts(hyp):
    hyp = np.asarray(hyp, dtype=np.float64)
    theta_L, theta_H = hyp[0:3], hyp[3:6]                            # gp:310-313
    rho = np.exp(hyp[-3])                                            # gp:414
    mean_L = np.exp(theta_L[0])                                      # gp:415
    mean_H = rho * mean_L + np.exp(theta_H[0])                       # gp:416
    return theta_L, theta_H, rho, mean_L, mean_H


def mf_K(XL, XH, hyp, jitter=JITTER):
    """Block covariance of MFGP.updt_info, gp:510-529 (jitter included)."""
    theta_L, theta_H, rho, _, _ = _mf_parts(hyp)
    sigma_n_L = np.exp(hyp[-2])
    sigma_n_H = np.exp(hyp[-1])
    NL, NH = XL.shape[0], XH.shape[0]
    K_LL = se_kernel(XL, XL, theta_L[1], theta_L[2]) + np.eye(NL) * sigma_n_L   # gp:523
    K_LH = rho * se_kernel(XL, XH, theta_L[1], theta_L[2])                     # gp:524
    K_HH = rho ** 2 * se_kernel(XH, XH, theta_L[1], theta_L[2]) + \
        se_kernel(XH, XH, theta_H[1], theta_H[2]) + np.eye(NH) * sigma_n_H     # gp:525-526
    K = np.vstack((np.hstack((K_LL, K_LH)), np.hstack((K_LH.T, K_HH))))       # gp:527-528
    return K + np.eye(NL + NH) * jitter


def mf_psi(Xs, XL, XH, hyp):
    """Cross covariance of MFGP.predict, gp:426-429."""
    theta_L, theta_H, rho, _, _ = _mf_parts(hyp)
    psi1 = rho * se_kernel(Xs, XL, theta_L[1], theta_L[2])
    psi2 = rho ** 2 * se_kernel(Xs, XH, theta_L[1], theta_L[2]) + \
        se_kernel(Xs, XH, theta_H[1], theta_H[2])
    return np.hstack((psi1, psi2))


def mf_faithful(XL, yL, XH, yH, hyp, Xs, jitter=JITTER, return_cov=False):
    """MFGP.updt_info (gp:493-529) then MFGP.predict (gp:401-438)."""
    XL = np.asarray(XL, dtype=np.float64).reshape(-1, 2)
    XH = np.asarray(XH, dtype=np.float64).reshape(-1, 2)
    yL = np.asarray(yL, dtype=np.float64).reshape(-1, 1)
    yH = np.asarray(yH, dtype=np.float64).reshape(-1, 1)
    theta_L, theta_H, rho, mean_L, mean_H = _mf_parts(hyp)
    L = np.linalg.cholesky(mf_K(XL, XH, hyp, jitter))                # gp:529
    y = np.vstack((yL - mean_L, yH - mean_H))                        # gp:419-424
    psi = mf_psi(Xs, XL, XH, hyp)                                    # gp:426-429
    alpha = np.linalg.solve(np.transpose(L), np.linalg.solve(L, y))  # gp:431
    mu = mean_H + np.matmul(psi, alpha)                              # gp:432
    beta = np.linalg.solve(np.transpose(L), np.linalg.solve(L, psi.T))  # gp:434
    cov = rho ** 2 * se_kernel(Xs, Xs, theta_L[1], theta_L[2]) + \
        se_kernel(Xs, Xs, theta_H[1], theta_H[2]) - np.matmul(psi, beta)  # gp:435-436
    if return_cov:
        return mu[:, 0], cov
    return mu[:, 0], np.diag(cov).copy()


# ---------------------------------------------------------------------------
# Diag-only restatements (semantic spec of the kernels; scalable CPU baseline)
# ---------------------------------------------------------------------------

def _diag_solve(K, psi, r, kss, mean):
    N = K.shape[0]
    if N == 0:
        M = psi.shape[0]
        return np.full(M, mean, dtype=np.float64), np.full(M, kss, dtype=np.float64)
    L = np.linalg.cholesky(K)
    V = sla.solve_triangular(L, psi.T, lower=True, check_finite=False)   # V = L^-1 psi^T
    z = sla.solve_triangular(L, r, lower=True, check_finite=False)       # z = L^-1 (y - m)
    mu = mean + V.T @ z                       # psi alpha = psi L^-T L^-1 r = V^T z
    var = kss - np.einsum("ij,ij->j", V, V)   # diag(k** - psi K^-1 psi^T)
    return mu, var


def sf_diag(X, y, hyp, Xs, jitter=JITTER):
    """Posterior mean and diagonal variance of SFGP (gp:229-255, 121-148)."""
    X = np.asarray(X, dtype=np.float64).reshape(-1, 2)
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    hyp = np.asarray(hyp, dtype=np.float64)
    N = X.shape[0]
    K = se_kernel(X, X, hyp[1], hyp[2]) + np.eye(N) * np.exp(hyp[-1])
    K = K + np.eye(N) * jitter
    psi = se_kernel(Xs, X, hyp[1], hyp[2])
    mean = np.exp(hyp[0])
    kss = np.exp(hyp[1])            # kernel(X*,X*) diagonal = s * exp(0)
    return _diag_solve(K, psi, y - mean, kss, mean)


def mf_diag(XL, yL, XH, yH, hyp, Xs, jitter=JITTER):
    """Posterior mean and diagonal variance of MFGP (gp:493-529, 401-438)."""
    XL = np.asarray(XL, dtype=np.float64).reshape(-1, 2)
    XH = np.asarray(XH, dtype=np.float64).reshape(-1, 2)
    yL = np.asarray(yL, dtype=np.float64).reshape(-1)
    yH = np.asarray(yH, dtype=np.float64).reshape(-1)
    theta_L, theta_H, rho, mean_L, mean_H = _mf_parts(hyp)
    K = mf_K(XL, XH, hyp, jitter)
    psi = mf_psi(Xs, XL, XH, hyp)
    r = np.concatenate((yL - mean_L, yH - mean_H))
    kss = rho ** 2 * np.exp(theta_L[1]) + np.exp(theta_H[1])
    return _diag_solve(K, psi, r, kss, mean_H)


def prior_variance(hyp):
    """Known-answer Var0: variance of the empty GP."""
    hyp = np.asarray(hyp, dtype=np.float64)
    if hyp.shape[0] == 4:
        return np.exp(hyp[1])
    rho = np.exp(hyp[6])
    return rho ** 2 * np.exp(hyp[1]) + np.exp(hyp[4])


def prior_mean(hyp):
    hyp = np.asarray(hyp, dtype=np.float64)
    if hyp.shape[0] == 4:
        return np.exp(hyp[0])
    return _mf_parts(hyp)[4]


# ---------------------------------------------------------------------------
# Tolerance policy (BASELINE.json north_star "1e-6 rel fp64")
# ---------------------------------------------------------------------------

def parity_errors(mu, var, mu_ref, var_ref, kss):
    """Return (mu_rel, var_floored_rel).

    mu:  max |d| / |ref|.
    var: max |d| / max(|ref|, 1e-6 * k**) -- posterior variance next to data is
         ~1e-9 against a prior of ~0.06, i.e. pure catastrophic cancellation in
         k** - sum(V^2); the reference's own rounding is larger than 1e-6 * 1e-9
         there, so the relative bound is floored at 1e-6 * k**.
    """
    mu = np.asarray(mu, dtype=np.float64).reshape(-1)
    var = np.asarray(var, dtype=np.float64).reshape(-1)
    mu_ref = np.asarray(mu_ref, dtype=np.float64).reshape(-1)
    var_ref = np.asarray(var_ref, dtype=np.float64).reshape(-1)
    mu_err = np.max(np.abs(mu - mu_ref) / np.maximum(np.abs(mu_ref), 1e-300)) if mu.size else 0.0
    den = np.maximum(np.abs(var_ref), 1e-6 * kss)
    var_err = np.max(np.abs(var - var_ref) / den) if var.size else 0.0
    return float(mu_err), float(var_err)


PARITY_TOL = 1e-6


def parity_errors_f32(mu, var, mu_ref, var_ref, kss):
    """Tolerance metric of the MFGP_F32 mode (BASELINE configs[4]: the resident V
    stored and streamed in fp32, everything else fp64) against this fp64 oracle.
    Returns (mu_err, var_err):

    mu:  max |d| / max(|ref|, 1e-2 * max|ref|, 1e-300) -- fp32 storage of V puts
         an absolute error of ~1e-8 on mu (2^-24 per V entry times |V^T z|); the
         posterior mean of a [0, 1] field crosses zero, so the relative bound is
         floored at 1 % of the field's largest |mu|: where |ref| is below that
         floor the gate F32_TOL is an ABSOLUTE bound of F32_TOL * 1e-2 * max|mu_ref|
         (1e-6 * max|mu_ref|), elsewhere relative; an all-zero mu_ref is compared
         against the 1e-300 floor (finite, never nan);
    var: max |d| / max(|ref|, 1e-6 * k**), the fp64 metric.
    Measured on australia9 (128x128, N = 2048, numpy emulation of the kernels'
    arithmetic): fp32 V alone 7e-7 / 3e-7; with the f32 accumulation of
    psi_new - L21 V_old 1.2e-6 / 2.2e-6. Gate: F32_TOL.
    """
    mu = np.asarray(mu, dtype=np.float64).reshape(-1)
    var = np.asarray(var, dtype=np.float64).reshape(-1)
    mu_ref = np.asarray(mu_ref, dtype=np.float64).reshape(-1)
    var_ref = np.asarray(var_ref, dtype=np.float64).reshape(-1)
    if not mu.size:
        return 0.0, 0.0
    mden = np.maximum(np.maximum(np.abs(mu_ref), 1e-2 * np.max(np.abs(mu_ref))), 1e-300)
    vden = np.maximum(np.abs(var_ref), 1e-6 * kss)
    return float(np.max(np.abs(mu - mu_ref) / mden)), float(np.max(np.abs(var - var_ref) / vden))


F32_TOL = 1e-4


# ---------------------------------------------------------------------------
# Voronoi-cell reductions (simulator.py:105-136, 194-323) -- checker for
# mfgp_cells.hip / geometry.py. Membership is in_polygon (sim:105-124), i.e.
# matplotlib's Path.contains_points crossing rule, restated here on arrays.
# ---------------------------------------------------------------------------

def in_polygon(pts, verts):
    """Crossing-number test of matplotlib's point_in_path for a closed polygon:
    an edge whose end points straddle the point's y (yflag = vy >= ty) toggles
    when ((vy1 - ty) * (vx0 - vx1) >= (vx1 - tx) * (vy0 - vy1)) == yflag1."""
    tx, ty = pts[:, 0], pts[:, 1]
    inside = np.zeros(pts.shape[0], dtype=bool)
    n = verts.shape[0]
    x0, y0 = verts[0]
    f0 = y0 >= ty
    for e in range(1, n + 1):
        x1, y1 = verts[e % n]
        f1 = y1 >= ty
        hit = ((y1 - ty) * (x0 - x1) >= (x1 - tx) * (y0 - y1)) == f1
        inside ^= (f0 != f1) & hit
        f0, x0, y0 = f1, x1, y1
    return inside


def poly_area(v):
    """Shoelace area (sim:127-136)."""
    x, y = v[:, 0], v[:, 1]
    return 0.5 * np.abs(np.dot(x, np.roll(y, 1)) - np.dot(y, np.roll(x, 1)))


def cell_reductions(polys, seeds, xs, w=None, f=None, var=None):
    """Per cell: (members, centroid, loss term, max var, argmax index) with the
    reference's formulas (sim:210-221, 255-270, 305-311)."""
    res = []
    for v, s in zip(polys, seeds):
        m = in_polygon(xs, v)
        area = poly_area(v)
        pts = xs[m]
        cen = loss = vmax = amax = None
        if w is not None:
            ww = w[m]
            cen = (np.mean(ww[:, None] * pts, axis=0) * area) / (np.mean(ww) * area)
        if f is not None:
            loss = np.mean(np.sum((pts - s) ** 2, axis=1) * f[m]) * area
        if var is not None and m.any():
            idx = np.flatnonzero(m)
            vmax = var[idx].max()
            amax = int(idx[np.argmax(var[idx])])
        res.append((m, cen, loss, vmax, amax))
    return res


# ---------------------------------------------------------------------------
# Negative log-marginal likelihood and its gradient (gp:81-106 SF, gp:344-385
# MF; the reference differentiates it with autograd for L-BFGS-B, gp:108-119 /
# 388-399) -- checker for mfgp_nlml. Analytic gradient:
#   NLML = 1/2 r^T K^-1 r + sum log L_ii + N/2 log(2 pi),  r = y - m(hyp)
#   dNLML/dh = 1/2 tr((K^-1 - a a^T) dK/dh) + a^T dr/dh,   a = K^-1 r
# ---------------------------------------------------------------------------

def _sq_dist_scaled(x, xp, log_l):
    lx = np.exp(log_l)
    d = x[:, None, :] / lx - xp[None, :, :] / lx
    return np.sum(d ** 2, axis=2)


def nlml(X, y, hyp, XL=None, yL=None, jitter=JITTER, grad=False):
    """SF: X, y = the data, hyp [4]. MF: XL, yL = lofi, X, y = hifi, hyp [9].
    Returns NLML (and its gradient w.r.t. the log-scaled hyp when grad)."""
    hyp = np.asarray(hyp, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    if hyp.shape[0] == 4:
        m, s, lx = np.exp(hyp[0]), np.exp(hyp[1]), hyp[2]
        sn = np.exp(hyp[3])
        r2 = _sq_dist_scaled(X, X, lx)
        E = s * np.exp(-0.5 * r2)
        N = X.shape[0]
        K = E + np.eye(N) * sn + np.eye(N) * jitter
        res = y - m
        dK = [None, E, E * r2, np.eye(N) * sn]
        dr = [-m * np.ones(N), None, None, None]
    else:
        XL = np.asarray(XL, dtype=np.float64).reshape(-1, 2)
        yL = np.asarray(yL, dtype=np.float64).reshape(-1)
        mL, sL, sH = np.exp(hyp[0]), np.exp(hyp[1]), np.exp(hyp[4])
        rho, snL, snH = np.exp(hyp[6]), np.exp(hyp[7]), np.exp(hyp[8])
        mH = rho * mL + np.exp(hyp[3])
        NL, NH = XL.shape[0], X.shape[0]
        Xa = np.vstack([XL, X])
        N = NL + NH
        rL2 = _sq_dist_scaled(Xa, Xa, hyp[2])
        rH2 = _sq_dist_scaled(Xa, Xa, hyp[5])
        EL = sL * np.exp(-0.5 * rL2)
        EH = sH * np.exp(-0.5 * rH2)
        lo = np.zeros(N, dtype=bool)
        lo[:NL] = True
        hi = ~lo
        cL = np.where(lo[:, None] & lo[None, :], 1.0, np.where(hi[:, None] & hi[None, :], rho ** 2, rho))
        cH = (hi[:, None] & hi[None, :]).astype(np.float64)
        dn = np.where(lo, snL, snH)
        K = cL * EL + cH * EH + np.diag(dn) + np.eye(N) * jitter
        res = np.concatenate([yL - mL, y - mH])
        drho = np.where(lo[:, None] & lo[None, :], 0.0, np.where(hi[:, None] & hi[None, :], 2 * rho ** 2, rho))
        dK = [None, cL * EL, cL * EL * rL2, None, cH * EH, cH * EH * rH2, drho * EL,
              np.diag(np.where(lo, snL, 0.0)), np.diag(np.where(hi, snH, 0.0))]
        dr = [np.concatenate([-mL * np.ones(NL), -rho * mL * np.ones(NH)]), None, None,
              np.concatenate([np.zeros(NL), -np.exp(hyp[3]) * np.ones(NH)]), None, None,
              np.concatenate([np.zeros(NL), -rho * mL * np.ones(NH)]), None, None]
    L = np.linalg.cholesky(K)
    a = np.linalg.solve(L.T, np.linalg.solve(L, res))
    val = 0.5 * res @ a + np.sum(np.log(np.diag(L))) + 0.5 * np.log(2.0 * np.pi) * res.shape[0]
    if not grad:
        return float(val)
    Kinv = np.linalg.solve(L.T, np.linalg.solve(L, np.eye(L.shape[0])))
    W = Kinv - np.outer(a, a)
    g = np.zeros(hyp.shape[0])
    for p in range(hyp.shape[0]):
        if dK[p] is not None:
            g[p] += 0.5 * np.sum(W * dK[p])
        if dr[p] is not None:
            g[p] += a @ dr[p]
    return float(val), g
