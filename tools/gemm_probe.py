#!/usr/bin/env python
"""Time the fp32 GEMMs of one RecBLR training step (B*L = 409,600 rows,
d = 128, H = 256) under torch's default BLAS choice, and the weight-gradient
GEMMs (K = 409,600) also as split-K batched GEMMs.  Run once plainly and once
with PYTORCH_TUNABLEOP_ENABLED=1 to compare."""
import os
import sys
import time

import torch

M = int(os.environ.get("PROBE_M", 409600))
dev = torch.device("cuda")
torch.manual_seed(0)

shapes = {  # name: (in_features K, out_features N)
    "in": (128, 512), "gates": (256, 512), "out": (256, 128), "w1": (128, 512), "w2": (512, 128)}


def bench(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def splitk_wgrad(dy, x, S):
    # dW = dy^T x with K = M split into S chunks (bmm), then a fixed-order sum
    Mk = dy.shape[0] // S
    a = dy[: Mk * S].view(S, Mk, -1).transpose(1, 2)
    b = x[: Mk * S].view(S, Mk, -1)
    return torch.bmm(a, b).sum(0)


tot = 0.0
for name, (K, N) in shapes.items():
    x = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev) * 0.05
    b = torch.randn(N, device=dev)
    dy = torch.randn(M, N, device=dev)
    f = 2.0 * M * K * N
    t_fwd = bench(lambda: torch.nn.functional.linear(x, w, b))
    t_dx = bench(lambda: dy @ w)
    t_dw = bench(lambda: dy.t() @ x)
    line = (f"{name:6s} K={K:4d} N={N:4d}  fwd {t_fwd*1e3:7.1f}us {f/t_fwd/1e9:6.1f}TF  "
            f"dX {t_dx*1e3:7.1f}us {f/t_dx/1e9:6.1f}TF  dW {t_dw*1e3:7.1f}us {f/t_dw/1e9:6.1f}TF")
    best = t_dw
    for S in (16, 64, 256):
        t = bench(lambda: splitk_wgrad(dy, x, S))
        line += f"  dW/S{S} {t*1e3:6.1f}us"
        best = min(best, t)
    print(line, flush=True)
    tot += t_fwd + t_dx + best
print(f"total per layer (best dW) {tot:.3f} ms; 2 layers {2*tot:.3f} ms", flush=True)
