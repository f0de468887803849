import sys, time, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
from tests.test_gpu_incremental import _points, _model, _err, HYP_MF
from mfgp_coverage_amd import _lib
if os.environ.get("STAMPS"):   # before any kernel: a stamps build writes through g_stamps
    import ctypes
    Lb = _lib.lib()
    Lb.mfgp_debug_set_stamps.argtypes = [ctypes.c_void_p]
    st = torch.zeros(64 + 8 * 4 * 2000, dtype=torch.int64, device="cuda")
    assert Lb.mfgp_debug_set_stamps(ctypes.c_void_p(st.data_ptr())) == 0
G, NL, NH0, k, B = 48, 400, 500, 8, 4
ctx = _lib.context()
full_ctx = _lib.Context(0); full_ctx.set_incremental(False)
offs = [int(a) for a in sys.argv[1].split(",")] if len(sys.argv) > 1 else [2]
cases = [_points(G, NL + NH0 + 4 * k, seed=100 + b, ongrid=(b not in offs)) for b in range(B)]
inc = [_model(ctx, "mf", X[:NL + NH0], y[:NL + NH0], NL, Xs)[0] for Xs, X, y in cases]
full = [_model(full_ctx, "mf", X[:NL + NH0], y[:NL + NH0], NL, Xs)[0] for Xs, X, y in cases]
M = cases[0][0].shape[0]
for step in range(int(os.environ.get('STEPS', '4'))):
    lo = NL + NH0 + step * k
    Xn = np.ascontiguousarray(np.vstack([X[lo:lo + k] for _, X, _ in cases]))
    yn = np.ascontiguousarray(np.concatenate([y[lo:lo + k] for _, _, y in cases]))
    Xd, yd = torch.from_numpy(Xn).cuda(), torch.from_numpy(yn).cuda()
    outs = []
    for models in (inc, full):
        for mdl in models: mdl.truncate(NH0)
        mu_d = torch.empty(B * M, dtype=torch.float64, device="cuda"); var_d = torch.empty(B * M, dtype=torch.float64, device="cuda")
        t0 = time.time()
        try:
            _lib.batch_append_predict(models, Xd.data_ptr(), yd.data_ptr(), [k] * B, mu_d.data_ptr(), var_d.data_ptr())
        except Exception as e:
            print("step", step, "raised", e)
        torch.cuda.synchronize()
        outs.append((mu_d.cpu().numpy().reshape(B, M), var_d.cpu().numpy().reshape(B, M), time.time() - t0))
    (mu, var, t1), (mu_f, var_f, t2) = outs
    print("step", step, "t inc %.4f full %.4f" % (t1, t2), "err per GP", [float("%.3g" % _err(mu[b], var[b], mu_f[b], var_f[b], HYP_MF)) for b in range(B)], [m.stats()["vstream"] for m in inc])

if os.environ.get("STAMPS"):
    st.zero_()
    lo = NL + NH0
    Xn = np.ascontiguousarray(np.vstack([X[lo:lo + k] for _, X, _ in cases]))
    yn = np.ascontiguousarray(np.concatenate([y[lo:lo + k] for _, _, y in cases]))
    Xd, yd = torch.from_numpy(Xn).cuda(), torch.from_numpy(yn).cuda()
    for mdl in inc: mdl.truncate(NH0)
    mu_d = torch.empty(B * M, dtype=torch.float64, device="cuda"); var_d = torch.empty(B * M, dtype=torch.float64, device="cuda")
    _lib.batch_append_predict(inc, Xd.data_ptr(), yd.data_ptr(), [k] * B, mu_d.data_ptr(), var_d.data_ptr())
    torch.cuda.synchronize()
    raw = st.cpu().numpy()[64:].reshape(-1, 8)
    t0 = raw[:, 0][raw[:, 0] > 0].min()
    tr = np.where(raw[:, :7] > 0, (raw[:, :7] - t0) / 100.0, np.nan)
    nprod = (NL + NH0 + 127) // 128
    for b in range(B):
        rows = tr[b::B]
        print("GP", b, "producers slot0..6 max", np.nanmax(rows[:nprod], 0).round(1), "finish", rows[:nprod][~np.isnan(rows[:nprod, 2])].round(1))
        if os.environ.get("FULLROWS"):
            np.set_printoptions(linewidth=200, suppress=True)
            print(rows[:nprod].round(1))
        print("      cells slot0..4 max", np.nanmax(rows[nprod:], 0).round(1), "min", np.nanmin(rows[nprod:], 0).round(1))
