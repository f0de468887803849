"""ctypes binding of libmfgp_hip.so (C ABI declared in include/mfgp_hip.h).

The product path has no CPU fallback: if the HIP library is missing or no GPU
is visible, every entry point raises instead of computing on the host.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MFGP_LIB") or os.path.join(HERE, "libmfgp_hip.so")

OK, ERR_NOT_PD, ERR_ARG, ERR_DEVICE = 0, 1, 2, 3
SF, MF = 0, 1
F64, F32 = 0, 1
ASYNC = 1

_c_double_p = ctypes.POINTER(ctypes.c_double)
_c_int64_p = ctypes.POINTER(ctypes.c_int64)

# name -> (restype, argtypes); every symbol declared in include/mfgp_hip.h
SIGNATURES = {
    "mfgp_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "mfgp_ctx_destroy": (None, [ctypes.c_void_p]),
    "mfgp_ctx_trim": (ctypes.c_int, [ctypes.c_void_p]),
    "mfgp_ctx_set_stream": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "mfgp_ctx_get_stream": (ctypes.c_void_p, [ctypes.c_void_p]),
    "mfgp_ctx_synchronize": (ctypes.c_int, [ctypes.c_void_p]),
    "mfgp_ctx_set_incremental": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "mfgp_ctx_set_fused": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "mfgp_ctx_set_deferred_appends": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "mfgp_ctx_set_lattice": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "mfgp_ctx_set_timing_stride": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    "mfgp_ctx_set_concurrent": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "mfgp_batch_append_predict_ex": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "mfgp_model_stats": (ctypes.c_int, [ctypes.c_void_p, _c_int64_p, ctypes.c_int]),
    "mfgp_nlml": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, _c_double_p, ctypes.c_void_p]),
    "mfgp_cell_reduce": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "mfgp_batch_cell_reduce": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p]),
    "mfgp_sample_points": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_double, ctypes.c_int64, ctypes.c_void_p,
                                          _c_int64_p]),
    "mfgp_batch_sample_points": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                                ctypes.c_void_p, ctypes.c_void_p]),
    "mfgp_ctx_enable_timing": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "mfgp_ctx_get_timing": (ctypes.c_int, [ctypes.c_void_p, _c_double_p, _c_int64_p, _c_double_p, _c_int64_p]),
    "mfgp_ctx_reset_timing": (ctypes.c_int, [ctypes.c_void_p]),
    "mfgp_ctx_planner_stats": (ctypes.c_int, [ctypes.c_void_p, _c_int64_p, ctypes.c_int, ctypes.c_int]),
    "mfgp_model_create": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                         ctypes.c_int, ctypes.c_double, ctypes.POINTER(ctypes.c_void_p)]),
    "mfgp_model_destroy": (None, [ctypes.c_void_p]),
    "mfgp_clone": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "mfgp_model_set_hyp": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_double]),
    "mfgp_set_grid": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]),
    "mfgp_set_data": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]),
    "mfgp_append": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]),
    "mfgp_predict": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "mfgp_predict_view": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                         ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p)]),
    "mfgp_predict_view_running": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                                 ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                                 ctypes.POINTER(ctypes.c_int)]),
    "mfgp_release_view": (ctypes.c_int, [ctypes.c_void_p]),
    "mfgp_view_max": (ctypes.c_int, [ctypes.c_void_p, _c_double_p, _c_int64_p, ctypes.POINTER(ctypes.c_int)]),
    "mfgp_model_n": (ctypes.c_int64, [ctypes.c_void_p]),
    "mfgp_model_nl": (ctypes.c_int64, [ctypes.c_void_p]),
    "mfgp_model_m": (ctypes.c_int64, [ctypes.c_void_p]),
    "mfgp_get_factor": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "mfgp_batch_append_predict": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_void_p,
                                                 ctypes.c_void_p, _c_int64_p, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_int]),
    "mfgp_batch_append_factor": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_void_p,
                                                ctypes.c_void_p, _c_int64_p, ctypes.c_int]),
    "mfgp_batch_predict": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_int]),
    "mfgp_truncate": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    "mfgp_batch_truncate": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64]),
    "mfgp_last_error": (ctypes.c_char_p, []),
    "mfgp_version": (ctypes.c_char_p, []),
}

_lib = None
_lib_lock = threading.Lock()


def lib():
    """Load libmfgp_hip.so (once). Raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lib_lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
            # One HIP runtime per process: PyTorch-ROCm bundles its own
            # libamdhip64.so.7 (same SONAME as /opt/rocm's). Loading torch first
            # makes the dynamic linker bind this library to that same runtime, so
            # torch tensors, streams and RCCL share one HIP runtime with the kernels.
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
            h = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                f = getattr(h, name)
                f.restype = res
                f.argtypes = args
            _lib = h
    return _lib


def check(rc):
    if rc == OK:
        return
    msg = lib().mfgp_last_error().decode(errors="replace")
    if rc == ERR_NOT_PD:
        raise np.linalg.LinAlgError(msg)
    if rc == ERR_ARG:
        if "Hyperparameters must be" in msg:
            raise TypeError(msg)
        raise ValueError(msg)
    raise RuntimeError(f"libmfgp_hip: {msg}")


def ptr(a):
    """Host pointer of a C-contiguous float64 ndarray (None for empty)."""
    if a is None or a.size == 0:
        return None
    return ctypes.c_void_p(a.ctypes.data)


class Context:
    """One HIP stream + workspace (mfgp_ctx)."""

    def __init__(self, device=0):
        h = ctypes.c_void_p()
        check(lib().mfgp_ctx_create(int(device), ctypes.byref(h)))
        self.handle = h
        self.device = device

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value and _lib is not None:
            _lib.mfgp_ctx_destroy(h)
            self.handle = None

    def synchronize(self):
        check(lib().mfgp_ctx_synchronize(self.handle))

    def trim(self):
        """Free the context's scratch (the MFGP_F32 full predict's fp64 V scratch and
        the workspace); models keep their state."""
        check(lib().mfgp_ctx_trim(self.handle))

    def set_stream(self, stream_ptr):
        check(lib().mfgp_ctx_set_stream(self.handle, ctypes.c_void_p(stream_ptr)))

    def set_incremental(self, on=True):
        """Bordered-Cholesky appends + one-pass predicts over the resident V (default),
        or full refactor + full V recompute on every update (the reference's work)."""
        check(lib().mfgp_ctx_set_incremental(self.handle, 1 if on else 0))

    def set_fused(self, on=True):
        """Bordered append + one-pass predict of a batch in one launch (default on)."""
        check(lib().mfgp_ctx_set_fused(self.handle, 1 if on else 0))

    def set_deferred_appends(self, on=True):
        """Stage appends and run them with the next predict, in one launch (default off:
        an append factors at once, so a non-PD step raises in updt / updt_hifi as in
        the reference; deferred, it raises in the predict that runs it)."""
        check(lib().mfgp_ctx_set_deferred_appends(self.handle, 1 if on else 0))

    def set_lattice(self, on=True):
        """Lattice-separable appends (k_inc_lat, default on where they apply: lattice
        grid, kss / (noise + jitter) <= 1e4, the old rows' posterior resident, enough
        GEMM tiles in the batch to fill the GPU), or always the one-pass V stream.
        on="force": also for batches too small to fill the GPU (tests)."""
        check(lib().mfgp_ctx_set_lattice(self.handle, 2 if on == "force" else (1 if on else 0)))

    def set_concurrent(self, on=True):
        """This context's launches may run beside other contexts' on the same GPU
        (mfgp_ctx_set_concurrent): no launch relies on all its workgroups being
        resident at once (the lattice GEMM always as its own launch)."""
        check(lib().mfgp_ctx_set_concurrent(self.handle, 1 if on else 0))

    def enable_timing(self, on=True, predict_only=False):
        """HIP-event timing of the predict launches (and, unless predict_only, the factor stages)."""
        check(lib().mfgp_ctx_enable_timing(self.handle, (2 if predict_only else 1) if on else 0))

    def set_timing_stride(self, stride):
        """Time only every stride-th eligible launch (events sample the kernel durations)."""
        check(lib().mfgp_ctx_set_timing_stride(self.handle, int(stride)))

    def reset_timing(self):
        check(lib().mfgp_ctx_reset_timing(self.handle))

    def timing(self):
        pm, fm = ctypes.c_double(), ctypes.c_double()
        pn, fn = ctypes.c_int64(), ctypes.c_int64()
        check(lib().mfgp_ctx_get_timing(self.handle, ctypes.byref(pm), ctypes.byref(pn),
                                        ctypes.byref(fm), ctypes.byref(fn)))
        return {"predict_ms": pm.value, "predict_launches": pn.value,
                "factor_ms": fm.value, "factor_calls": fn.value}

    PLANNER_KEYS = ("runs", "inc_factor", "vstream", "lattice", "lattice_arg", "lattice_g2", "full_factor",
                    "full_predict", "batch_setup_us", "batch_loop_us", "batch_finish_us")

    def planner_stats(self, reset=False):
        """Path counters of the planners' loops (mfgp_sample_points /
        mfgp_batch_sample_points) since the last reset: how many model runs, and which step
        form their iterations took (vstream counts every one-pass predict, lattice steps
        included)."""
        out = (ctypes.c_int64 * len(self.PLANNER_KEYS))()
        check(lib().mfgp_ctx_planner_stats(self.handle, out, len(self.PLANNER_KEYS), 1 if reset else 0))
        return dict(zip(self.PLANNER_KEYS, (int(v) for v in out)))


_tls = threading.local()
_default_device = int(os.environ.get("MFGP_DEVICE", "0"))


def set_device(device):
    """Device used by models created afterwards in this process (one process per GPU)."""
    global _default_device
    _default_device = int(device)


def set_deferred_appends(on=True, device=None):
    """Deferred appends on the calling thread's context (see Context.set_deferred_appends):
    updt / updt_hifi stage their rows and the next predict runs the bordered append and
    the one-pass predict as one launch."""
    context(device).set_deferred_appends(on)


def context(device=None):
    """The calling thread's context for `device` (one stream per host thread)."""
    dev = _default_device if device is None else int(device)
    ctxs = getattr(_tls, "ctxs", None)
    if ctxs is None:
        ctxs = _tls.ctxs = {}
    if dev not in ctxs:
        ctxs[dev] = Context(dev)
    return ctxs[dev]


class _ViewLease:
    """One buffer handed over by mfgp_predict_view; returned to the pool when the
    last array over it is gone."""

    __slots__ = ("view",)

    def __init__(self, view):
        self.view = view

    def __del__(self):
        if _lib is not None and self.view:
            _lib.mfgp_release_view(ctypes.c_void_p(self.view))
            self.view = None


class _HostView:
    """[n] float64 at a host address, for np.asarray (which keeps this object, and
    so the lease, as the array's base)."""

    __slots__ = ("__array_interface__", "lease")

    def __init__(self, addr, n, lease):
        self.__array_interface__ = {"shape": (int(n),), "typestr": "<f8", "data": (int(addr), False), "version": 3}
        self.lease = lease


class Model:
    """Owning handle of one device-resident GP (mfgp_model)."""

    def __init__(self, ctx, kind, hyp, jitter, handle=None, dtype=F64):
        """dtype: F64 (default; everything in fp64, the reference's precision) or F32
        (the resident V = L^-1 psi^T -- the only O(M N) state -- stored and streamed in
        fp32; factor, solves and reductions stay fp64; BASELINE configs[4])."""
        self.ctx = ctx
        self.kind = kind
        self.dtype = dtype
        if handle is None:
            hyp = np.ascontiguousarray(hyp, dtype=np.float64)
            h = ctypes.c_void_p()
            check(lib().mfgp_model_create(ctx.handle, kind, int(dtype), ptr(hyp), int(hyp.shape[0]),
                                          float(jitter), ctypes.byref(h)))
            handle = h
        self.handle = handle

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value and _lib is not None:
            _lib.mfgp_model_destroy(h)
            self.handle = None

    def clone(self):
        h = ctypes.c_void_p()
        check(lib().mfgp_clone(self.handle, ctypes.byref(h)))
        return Model(self.ctx, self.kind, None, None, handle=h, dtype=self.dtype)

    def set_hyp(self, hyp, jitter):
        hyp = np.ascontiguousarray(hyp, dtype=np.float64).reshape(-1)
        check(lib().mfgp_model_set_hyp(self.handle, ptr(hyp), int(hyp.shape[0]), float(jitter)))

    def set_grid(self, xs):
        xs = np.ascontiguousarray(xs, dtype=np.float64).reshape(-1, 2)
        check(lib().mfgp_set_grid(self.handle, ptr(xs), xs.shape[0]))

    def set_data(self, XL, yL, XH, yH):
        XL, yL, XH, yH = (np.ascontiguousarray(a, dtype=np.float64) for a in (XL, yL, XH, yH))
        check(lib().mfgp_set_data(self.handle, ptr(XL), ptr(yL), XL.size // 2, ptr(XH), ptr(yH), XH.size // 2))

    def append(self, X, y):
        X = np.ascontiguousarray(X, dtype=np.float64)
        y = np.ascontiguousarray(y, dtype=np.float64)
        check(lib().mfgp_append(self.handle, ptr(X), ptr(y), X.size // 2))

    def predict(self):
        M = lib().mfgp_model_m(self.handle)
        mu = np.empty(M, dtype=np.float64)
        var = np.empty(M, dtype=np.float64)
        check(lib().mfgp_predict(self.handle, ptr(mu) if M else None, ptr(var) if M else None))
        return mu, var

    def predict_view(self, with_max=False):
        """predict() without the host copy: (mu, var) are writable arrays over the
        model's pinned result buffer, handed over to them (mfgp_predict_view); the
        buffer goes back to the library's pool when both arrays are gone. with_max:
        (mu, var, fused) where fused is (max var, its first cell) as the launch that
        wrote the buffer reduced them (mfgp_view_max), or None."""
        mu_p, var_p, view, running = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int(0)
        L = lib()
        check(L.mfgp_predict_view_running(self.handle, ctypes.byref(mu_p), ctypes.byref(var_p), ctypes.byref(view),
                                          ctypes.byref(running)))
        M = L.mfgp_model_m(self.handle)
        if not view.value:
            e = np.empty(M, dtype=np.float64), np.empty(M, dtype=np.float64)
            return (*e, None) if with_max else e
        lease = _ViewLease(view.value)
        mu, var = np.asarray(_HostView(mu_p.value, M, lease)), np.asarray(_HostView(var_p.value, M, lease))
        if running.value:
            # the eager append's launch was still computing into the buffer: the arrays
            # were wrapped meanwhile and are given out once it has ended
            check(L.mfgp_ctx_synchronize(self.ctx.handle))
        if not with_max:
            return mu, var
        vm, am, ok = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int(0)
        check(L.mfgp_view_max(ctypes.c_void_p(view.value), ctypes.byref(vm), ctypes.byref(am), ctypes.byref(ok)))
        return mu, var, ((np.float64(vm.value), int(am.value)) if ok.value else None)

    def factor(self):
        n = lib().mfgp_model_n(self.handle)
        L = np.zeros((n, n), dtype=np.float64)
        if n:
            check(lib().mfgp_get_factor(self.handle, ptr(L)))
        return L

    @property
    def n(self):
        return lib().mfgp_model_n(self.handle)

    def stats(self):
        """{factor_rows, v_rows, full_factor, inc_factor, full_predict, vstream} (path
        counters; vstream counts every one-pass predict, lattice steps included), the
        grid's lattice axes {lattice_nx, lattice_ny} (0: not a lattice) and {lattice}:
        the steps that took the lattice-separable path (k_inc_lat); {lattice_virtual}: the
        off-lattice training rows (extra K rows) the last lattice step ran, as its
        device counters hold them (MF: summed over both kernel parts); {lattice_arg}:
        the lattice steps launched with their descriptors by value (k_inc_lat_arg);
        {lattice_g2}: the lattice steps whose GEMM and cells ran as a second launch
        (k_lat_gemm2); {post_copy}: batch predicts served from the resident posterior
        because the model appended nothing (k_post_copy); {early_pd}: eager appends that
        returned at the launch's published L22 verdict (mfgp_append, one GP)."""
        out = (ctypes.c_int64 * 14)()
        check(lib().mfgp_model_stats(self.handle, out, 14))
        keys = ("factor_rows", "v_rows", "full_factor", "inc_factor", "full_predict", "vstream",
                "lattice_nx", "lattice_ny", "lattice", "lattice_virtual", "lattice_arg", "lattice_g2",
                "post_copy", "early_pd")
        return dict(zip(keys, (int(v) for v in out)))

    def sample_points(self, threshold, max_points):
        """compute_sample_points (simulator.py:326-374) on a device copy of this model:
        the [n, 2] grid cells chosen until max var <= threshold (at most max_points)."""
        pts = np.empty((max(int(max_points), 1), 2), dtype=np.float64)
        n = ctypes.c_int64(0)
        check(lib().mfgp_sample_points(self.handle, float(threshold), int(max_points), ptr(pts), ctypes.byref(n)))
        return pts[:n.value].copy()

    def nlml(self, hyp, grad=False):
        """likelihood (gp:81-106 / 344-385) of this model's data under `hyp`; with grad, (value, gradient)."""
        h = np.ascontiguousarray(hyp, dtype=np.float64).reshape(-1)
        v = ctypes.c_double(0.0)
        g = np.empty(h.shape[0], dtype=np.float64) if grad else None
        check(lib().mfgp_nlml(self.handle, ptr(h), int(h.shape[0]), ctypes.byref(v),
                              ctypes.c_void_p(g.ctypes.data) if grad else None))
        return (v.value, g) if grad else v.value

    def truncate(self, n_keep_hifi):
        check(lib().mfgp_truncate(self.handle, int(n_keep_hifi)))


def batch_append_predict(models, X, y, k, mu_ptr, var_ptr, asynchronous=False, vmax_ptr=None, vargmax_ptr=None):
    """Batched update+predict over device-resident models.

    X, y: integer device (or host) addresses of the concatenated new rows;
    k: per-model row counts; mu_ptr/var_ptr: device addresses of [sum M] outputs;
    vmax_ptr / vargmax_ptr: optional device addresses of [n] float64 / int64 outputs
    (fused np.amax / np.argmax of each model's variance).
    """
    n = len(models)
    arr = (ctypes.c_void_p * n)(*[m.handle.value for m in models])
    ks = (ctypes.c_int64 * n)(*[int(v) for v in k])
    if vmax_ptr is None and vargmax_ptr is None:
        rc = lib().mfgp_batch_append_predict(arr, n, ctypes.c_void_p(X), ctypes.c_void_p(y), ks,
                                             ctypes.c_void_p(mu_ptr), ctypes.c_void_p(var_ptr),
                                             ASYNC if asynchronous else 0)
    else:
        rc = lib().mfgp_batch_append_predict_ex(arr, n, ctypes.c_void_p(X), ctypes.c_void_p(y), ks,
                                                ctypes.c_void_p(mu_ptr), ctypes.c_void_p(var_ptr),
                                                ctypes.c_void_p(vmax_ptr), ctypes.c_void_p(vargmax_ptr),
                                                ASYNC if asynchronous else 0)
    check(rc)


class Batch:
    """A fixed list of models with its handle / row-count arrays built once: the
    per-step calls of a seed ensemble without rebuilding ctypes arrays."""

    def __init__(self, models, k):
        self.models = list(models)
        n = len(self.models)
        self.n = n
        self.arr = (ctypes.c_void_p * n)(*[m.handle.value for m in self.models])
        self.ks = (ctypes.c_int64 * n)(*[int(v) for v in k])

    def truncate(self, n_keep_hifi):
        check(lib().mfgp_batch_truncate(self.arr, self.n, int(n_keep_hifi)))

    def append_predict(self, X, y, mu_ptr, var_ptr, asynchronous=False, vmax_ptr=None, vargmax_ptr=None):
        check(lib().mfgp_batch_append_predict_ex(self.arr, self.n, ctypes.c_void_p(X), ctypes.c_void_p(y), self.ks,
                                                 ctypes.c_void_p(mu_ptr), ctypes.c_void_p(var_ptr),
                                                 ctypes.c_void_p(vmax_ptr), ctypes.c_void_p(vargmax_ptr),
                                                 ASYNC if asynchronous else 0))


def batch_append_factor(models, X, y, k, asynchronous=False):
    """Append + refactor a batch (device or host row pointers); no predict."""
    n = len(models)
    arr = (ctypes.c_void_p * n)(*[m.handle.value for m in models])
    ks = (ctypes.c_int64 * n)(*[int(v) for v in k])
    check(lib().mfgp_batch_append_factor(arr, n, ctypes.c_void_p(X), ctypes.c_void_p(y), ks,
                                         ASYNC if asynchronous else 0))


def batch_sample_points(models, thresholds, max_points):
    """mfgp_batch_sample_points: compute_sample_points (simulator.py:326-374) for every
    model of the batch, stepped together -> one [n_b, 2] array of chosen cells per model."""
    n = len(models)
    arr = (ctypes.c_void_p * n)(*[m.handle.value for m in models])
    thr = np.ascontiguousarray(np.broadcast_to(np.asarray(thresholds, dtype=np.float64), (n,)))
    P = max(int(max_points), 1)
    pts = np.empty((n, P, 2), dtype=np.float64)
    cnt = np.zeros(n, dtype=np.int64)
    check(lib().mfgp_batch_sample_points(arr, n, ptr(thr), int(max_points), ptr(pts), ptr(cnt)))
    return [pts[b, :cnt[b]].copy() for b in range(n)]


def batch_predict(models, mu_ptr, var_ptr, asynchronous=False):
    """Posterior mean / variance of a batch from its current factors."""
    n = len(models)
    arr = (ctypes.c_void_p * n)(*[m.handle.value for m in models])
    check(lib().mfgp_batch_predict(arr, n, ctypes.c_void_p(mu_ptr), ctypes.c_void_p(var_ptr),
                                   ASYNC if asynchronous else 0))


def cell_reduce(grid, verts, vstart, seeds, w=None, f=None, var=None, ctx=None):
    """mfgp_cell_reduce on host arrays -> (out [n, 6], argmax [n]); see include/mfgp_hip.h."""
    ctx = ctx or context()
    g = np.ascontiguousarray(grid, dtype=np.float64).reshape(-1, 2)
    v = np.ascontiguousarray(verts, dtype=np.float64).reshape(-1, 2)
    vs = np.ascontiguousarray(vstart, dtype=np.int32).reshape(-1)
    sd = np.ascontiguousarray(seeds, dtype=np.float64).reshape(-1, 2)
    n = vs.shape[0] - 1
    arrs = [None if a is None else np.ascontiguousarray(a, dtype=np.float64).reshape(-1) for a in (w, f, var)]
    out = np.empty((max(n, 1), 6), dtype=np.float64)
    am = np.empty(max(n, 1), dtype=np.int64)
    check(lib().mfgp_cell_reduce(ctx.handle, ptr(g), g.shape[0], n, ctypes.c_void_p(vs.ctypes.data), ptr(v), ptr(sd),
                                 *[ptr(a) for a in arrs], ctypes.c_void_p(out.ctypes.data),
                                 ctypes.c_void_p(am.ctypes.data)))
    return out[:n], am[:n]


def batch_cell_reduce(grid, verts, vstart, seeds, field, nfield, w=None, f=None, var=None, ctx=None, M=None):
    """mfgp_batch_cell_reduce -> (out [n, 6], argmax [n]). verts / seeds / vstart /
    field are host arrays; grid a host array [M, 2] or (with M) the integer device
    address of one; w and var host arrays [nfield, M] or integer device addresses
    of [nfield * M] float64 (a batch's predict outputs); f a host array [M] or a
    device address."""
    ctx = ctx or context()
    keep = []

    def arg(a):
        if a is None:
            return None
        if isinstance(a, int):
            return ctypes.c_void_p(a)
        a = np.ascontiguousarray(a, dtype=np.float64).reshape(-1)
        keep.append(a)
        return ptr(a)
    if isinstance(grid, int):
        if M is None:
            raise ValueError("a device grid needs M")
        g_arg, Mg = ctypes.c_void_p(grid), int(M)
    else:
        g = np.ascontiguousarray(grid, dtype=np.float64).reshape(-1, 2)
        g_arg, Mg = ptr(g), g.shape[0]
        keep.append(g)
    v = np.ascontiguousarray(verts, dtype=np.float64).reshape(-1, 2)
    vs = np.ascontiguousarray(vstart, dtype=np.int32).reshape(-1)
    fd = np.ascontiguousarray(field, dtype=np.int32).reshape(-1)
    sd = np.ascontiguousarray(seeds, dtype=np.float64).reshape(-1, 2)
    n = vs.shape[0] - 1
    if fd.shape[0] != n:
        raise ValueError("field needs one entry per cell")
    out = np.empty((max(n, 1), 6), dtype=np.float64)
    am = np.empty(max(n, 1), dtype=np.int64)
    check(lib().mfgp_batch_cell_reduce(ctx.handle, g_arg, Mg, n, ctypes.c_void_p(vs.ctypes.data), ptr(v),
                                       ptr(sd), ctypes.c_void_p(fd.ctypes.data), int(nfield), arg(w), arg(f), arg(var),
                                       ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(am.ctypes.data)))
    return out[:n], am[:n]
