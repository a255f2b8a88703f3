#!/usr/bin/env python
"""Accuracy and speed of the split-bf16 fp32 GEMMs (csrc/gemm_split.hip)
against torch's fp32 GEMMs (hipBLASLt/rocBLAS) on the projection shapes of
one RecBLR training step (B*L = 409,600 rows, d = 128, H = 256).

Accuracy: max |err| / max |ref| against an fp64 product on the first 4096
rows, for both implementations.  Speed: median of 10 HIP-event timings."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from datamining_recblr_amd import gemm_tuning, kernels, linear  # noqa: E402

M = int(os.environ.get("PROBE_M", 409600))
dev = torch.device("cuda")
torch.manual_seed(0)
shapes = {"in": (128, 512), "gates": (256, 512), "out": (256, 128), "w1": (128, 512),
          "w2": (512, 128)}


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
    return ts[len(ts) // 2] * 1e3


def err(y, ref):
    return ((y.double() - ref).abs().max() / ref.abs().max()).item()


if os.environ.get("PROBE_TUNED", "1") == "1":
    print("torch tuned table:", gemm_tuning.use_tuned_gemms())
tot_t = tot_s = tot_w = 0.0
for name, (K, N) in shapes.items():
    x = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev) / K ** 0.5
    b = torch.randn(N, device=dev)
    dy = torch.randn(M, N, device=dev)
    f = 2.0 * M * K * N
    # forward: x @ w^T + b
    wf = kernels.gemm_split_weight(w)
    ys = kernels.gemm_nt(x, wf, N, bias=b)
    yt = torch.addmm(b, x, w.t())
    ref = torch.addmm(b.double(), x[:4096].double(), w.double().t())
    e_s, e_t = err(ys[:4096], ref), err(yt[:4096], ref)
    t_t = bench(lambda: torch.addmm(b, x, w.t()))
    t_s = bench(lambda: kernels.gemm_nt(x, wf, N, bias=b, out=ys))
    t_w = bench(lambda: kernels.gemm_split_weight(w))
    print(f"{name:5s} fwd K={K:3d} N={N:3d}: torch {t_t:7.1f}us {f/t_t/1e6:6.1f}TF err {e_t:.2e} | "
          f"split {t_s:7.1f}us {f/t_s/1e6:6.1f}TF err {e_s:.2e} (+{t_w:.1f}us weight split)",
          flush=True)
    tot_t += t_t
    tot_s += t_s
    # input gradient: dy @ w
    wt = kernels.gemm_split_weight(w, transpose=True)
    dxs = kernels.gemm_nt(dy, wt, K)
    dxt = dy @ w
    ref = dy[:4096].double() @ w.double()
    e_s, e_t = err(dxs[:4096], ref), err(dxt[:4096], ref)
    t_t = bench(lambda: dy @ w)
    t_s = bench(lambda: kernels.gemm_nt(dy, wt, K, out=dxs))
    print(f"{name:5s} dX  K={N:3d} N={K:3d}: torch {t_t:7.1f}us {f/t_t/1e6:6.1f}TF err {e_t:.2e} | "
          f"split {t_s:7.1f}us {f/t_s/1e6:6.1f}TF err {e_s:.2e}", flush=True)
    tot_t += t_t
    tot_s += t_s
    # accumulate form (residual gradient added in place)
    base = torch.randn(M, K, device=dev)
    o = base.clone()
    kernels.gemm_nt(dy, wt, K, out=o, accumulate=True)
    e_acc = ((o - base - dxs).abs().max() / dxs.abs().max()).item()
    print(f"      accumulate check {e_acc:.2e}", flush=True)
    t_dw = bench(lambda: linear.wgrad(dy, x))
    print(f"      dW (torch split-K bmm + colsum) {t_dw:7.1f}us {f/t_dw/1e6:6.1f}TF", flush=True)
    tot_w += t_dw
    del x, dy, ys, yt, dxs, dxt, base, o
print(f"total fwd+dX: torch {tot_t:.1f}us split {tot_s:.1f}us; dW torch {tot_w:.1f}us")
