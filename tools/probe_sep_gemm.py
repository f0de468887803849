"""Probe: f64 GEMM rate of the separable-kernel contraction shapes on the GPU
(rocBLAS through torch.bmm), to size the lattice-separable incremental step
(DESIGN.md section 10). T~[a, ix, iy] = sum_j (w_aj c_j Ex[ix, j]) Ey[iy, j]:
per GP a (k*nx) x n_terms by n_terms x ny product."""
import json, sys, time
import torch

dev = torch.device("cuda:0")
res = []
for (B, R, K, C) in [(8, 1024, 3056, 128), (8, 1024, 2040, 128), (32, 2048, 12280, 256), (1, 1024, 3056, 128)]:
    a = torch.randn(B, R, K, dtype=torch.float64, device=dev)
    b = torch.randn(B, K, C, dtype=torch.float64, device=dev)
    for _ in range(3):
        c = torch.bmm(a, b)
    torch.cuda.synchronize()
    n = 20
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        c = torch.bmm(a, b)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    fl = 2.0 * B * R * K * C
    res.append({"B": B, "R": R, "K": K, "C": C, "ms": ms, "tflops": fl / ms / 1e9})
    print(json.dumps(res[-1]), flush=True)
