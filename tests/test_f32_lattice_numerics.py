"""Why the lattice step of MFGP_F32 models may stream F = L^-1 in fp32 (DESIGN.md
section 2.3): the step's update restated in NumPy -- w = F11^T L21^T, T = psi_new -
w^T psi_old, v = L22^-1 T, var = var_old - |v|^2 -- with F (and L21, which comes
from the fp32 V) rounded to fp32, against the fp64 oracle's posterior with all rows.
The error per step stays two orders of magnitude inside the fp32 mode's tolerance
(F32_TOL) up to the lattice gate's conditioning bound (kss / noise <= 1e4,
LAT_RMAX); tests/test_gpu_f32.py and test_gpu_long_horizon.py check the device's
chains of steps against the oracle."""
import numpy as np
import pytest
import scipy.linalg as sla

from oracle import gp_oracle as O


def _step_error(G, NL, NH, ratio, f32_F, seed=0, k=8):
    from mfgp_coverage_amd.synthetic import HYP
    hyp = HYP["australia8_mf"].copy()
    rho = np.exp(hyp[-3])
    kss = rho ** 2 * np.exp(hyp[1]) + np.exp(hyp[4])
    hyp[-2] = np.log(kss / ratio)              # lofi noise at the conditioning ratio
    hyp[-1] = max(hyp[-1], hyp[-2])
    rng = np.random.default_rng(seed)
    g = np.linspace(0, 1, G)
    xs = np.array([(a, b) for a in g for b in g])
    XL = xs[rng.choice(len(xs), NL, replace=False)]
    XH = xs[rng.choice(len(xs), NH + k, replace=False)]
    yL, yH = rng.standard_normal(NL), rng.standard_normal(NH + k)
    K = O.mf_K(XL, XH, hyp)
    n0 = K.shape[0] - k
    F = sla.solve_triangular(np.linalg.cholesky(K[:n0, :n0]), np.eye(n0), lower=True)
    Xs = xs[rng.choice(len(xs), 512, replace=False)]
    psi = O.mf_psi(Xs, XL, XH, hyp)
    V_old = F @ psi[:, :n0].T
    var_old = kss - np.einsum("ij,ij->j", V_old, V_old)
    L21T = (F @ K[:n0, n0:]).astype(np.float32).astype(np.float64)   # from the fp32 V
    Fw = F.astype(np.float32).astype(np.float64) if f32_F else F
    w = Fw.T @ L21T
    T = psi[:, n0:].T - w.T @ psi[:, :n0].T
    v = sla.solve_triangular(np.linalg.cholesky(K[n0:, n0:] - L21T.T @ L21T), T, lower=True)
    var = var_old - np.einsum("ij,ij->j", v, v)
    mu_r, var_r = O.mf_diag(XL, yL, XH, yH, hyp, Xs)
    return max(O.parity_errors_f32(mu_r, var, mu_r, var_r, kss))


@pytest.mark.parametrize("ratio", [22.3, 1e3, 1e4])
def test_fp32_F_step_error_far_inside_f32_tolerance(ratio):
    e32 = _step_error(48, 300, 300, ratio, True)
    e64 = _step_error(48, 300, 300, ratio, False)
    # per step (measured: 8e-8 / 2.7e-7 / 3.7e-7 here; fp64 F: ~1e-8); a chain of
    # lattice steps carries it in the resident posterior until the LAT_MAXD refresh
    assert e32 < 1e-2 * O.F32_TOL, (ratio, e32)
    assert e64 < 1e-2 * O.F32_TOL, (ratio, e64)
