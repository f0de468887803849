"""Time the Voronoi-cell reductions (mfgp_cell_reduce) at the headline grid:
128x128 cells, 8 agents' bounded Voronoi polygons (a synthetic partition: the
polygons only set the work), device-resident inputs; and the oracle's NumPy
restatement of the reference functions (in_polygon per cell + means) on the
host for scale. Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402


def main():
    import torch
    from mfgp_coverage_amd import _lib
    from oracle import gp_oracle as O
    rng = np.random.default_rng(0)
    g = np.linspace(0, 1, 128)
    xs = np.array([(a, b) for a in g for b in g])
    polys = []
    for n in range(8):   # eight convex cells
        ang = np.sort(rng.random(7)) * 2 * np.pi
        c = rng.random(2)
        polys.append(np.column_stack([c[0] + 0.3 * np.cos(ang), c[1] + 0.3 * np.sin(ang)]))
    seeds = rng.random((8, 2))
    w, f, var = rng.random(xs.shape[0]), rng.random(xs.shape[0]), rng.random(xs.shape[0])
    verts = np.vstack(polys)
    vs = np.concatenate([[0], np.cumsum([p.shape[0] for p in polys])]).astype(np.int32)
    d = {k: torch.from_numpy(np.ascontiguousarray(a)).cuda() for k, a in
         (("xs", xs), ("verts", verts), ("seeds", seeds), ("w", w), ("f", f), ("var", var))}
    out = torch.empty((8, 6), dtype=torch.float64, device="cuda")
    am = torch.empty(8, dtype=torch.int64, device="cuda")
    ctx = _lib.context()
    args = [ctx.handle, ctypes.c_void_p(d["xs"].data_ptr()), xs.shape[0], 8, ctypes.c_void_p(vs.ctypes.data),
            ctypes.c_void_p(d["verts"].data_ptr()), ctypes.c_void_p(d["seeds"].data_ptr()),
            ctypes.c_void_p(d["w"].data_ptr()), ctypes.c_void_p(d["f"].data_ptr()),
            ctypes.c_void_p(d["var"].data_ptr()), ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(am.data_ptr())]
    for _ in range(10):
        _lib.check(_lib.lib().mfgp_cell_reduce(*args))
    R = 200
    t0 = time.perf_counter()
    for _ in range(R):
        _lib.check(_lib.lib().mfgp_cell_reduce(*args))
    gpu = (time.perf_counter() - t0) / R
    t0 = time.perf_counter()
    O.cell_reductions(polys, seeds, xs, w=w, f=f, var=var)
    cpu = time.perf_counter() - t0
    print(json.dumps({"grid": 128, "cells": 8, "gpu_ms_per_call": gpu * 1e3, "cpu_oracle_ms": cpu * 1e3,
                      "note": "gpu = synchronous C-ABI call incl. launch + sync; cpu = NumPy restatement"}))


if __name__ == "__main__":
    main()
