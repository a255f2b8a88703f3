"""Accuracy and timing of the f16 two-part split GEMM (rb_gemm_nt_h) against
the bf16 six-product kernel (rb_gemm_nt), torch's fp32 GEMM and fp64, on the
encoder's projection shapes at a packed row count.

    python tools/gemm_h_probe.py [M]
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from datamining_recblr_amd import kernels  # noqa: E402

SHAPES = [("in.fwd", 128, 512), ("in.dX", 512, 128), ("gates.fwd", 256, 512),
          ("gates.dX", 512, 256), ("out.fwd", 256, 128), ("out.dX", 128, 256),
          ("w2.fwd", 512, 128), ("w2.dX", 128, 512)]


def timeit(fn, reps=10):
    fn()
    ts = []
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def err(out, ref):
    return float((out.double() - ref).abs().max() / ref.abs().max())


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 204632
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    tot = {"h": 0.0, "x6": 0.0, "torch": 0.0}
    print(f"M={M}")
    for name, R, C in SHAPES:
        a = torch.randn(M, R, device=dev, generator=g)
        w = torch.randn(C, R, device=dev, generator=g) * 0.05
        bias = torch.randn(C, device=dev, generator=g)
        ref = torch.addmm(bias.double(), a.double(), w.double().t())
        wf = kernels.gemm_h_weight(w)
        rmax = torch.empty((M + 31) // 32, device=dev)
        oh = kernels.gemm_nt_h(a, wf, C, bias=bias, rmax=rmax)
        wx = kernels.gemm_split_weight(w)
        ox = kernels.gemm_nt(a, wx, C, bias=bias)
        ot = torch.addmm(bias, a, w.t())
        torch.cuda.synchronize()
        rm_ref = torch.nn.functional.pad(a.abs().amax(1), (0, (-M) % 32)).view(-1, 32).amax(1)
        rm_ok = bool(torch.equal(rmax, rm_ref))
        th = timeit(lambda: kernels.gemm_nt_h(a, wf, C, bias=bias, out=oh))
        tx = timeit(lambda: kernels.gemm_nt(a, wx, C, bias=bias, out=ox))
        tt = timeit(lambda: torch.addmm(bias, a, w.t(), out=ot))
        tot["h"] += th
        tot["x6"] += tx
        tot["torch"] += tt
        by = 4.0 * M * (R + C)
        print(f"{name:10s} R={R:3d} C={C:3d} | h {th:7.1f} us {by / th / 1e6:5.2f} TB/s err {err(oh, ref):.2e}"
              f" | x6 {tx:7.1f} us err {err(ox, ref):.2e} | torch {tt:7.1f} us err {err(ot, ref):.2e}"
              f" | rmax {'ok' if rm_ok else 'MISMATCH'}", flush=True)
        del a, w, ref, oh, ox, ot
    print("total us:", {k: round(v, 1) for k, v in tot.items()})

    # adversarial rows: per-row scales over 60 binades, zero rows, rows whose
    # first entries are zero / tiny (the online re-scale), huge values
    R, C = 256, 128
    Ms = 4096 + 77
    a = torch.randn(Ms, R, device=dev, generator=g)
    a *= torch.exp2(torch.randint(-60, 60, (Ms, 1), device=dev, generator=g).float())
    a[5] = 0
    a[6, :48] = 0
    a[7, :16] *= 1e-12
    a[8] *= torch.exp2(torch.arange(R, device=dev).float() / 4)     # grows 2^64 along K
    a[9, 100] = 3e37
    a[10] = 0
    a[10, 255] = 1e-30
    a[11, :200] = 1e-20
    w = torch.randn(C, R, device=dev, generator=g)
    w[3] *= 1e-25
    w[4, :10] = 0
    w[5] = 0
    ref = a.double() @ w.double().t()
    oh = kernels.gemm_nt_h(a, kernels.gemm_h_weight(w), C)
    ot = a @ w.t()
    torch.cuda.synchronize()
    # per-row relative error (the row scale makes every row accurate on its own)
    den = a.double().abs() @ w.double().abs().t()
    ok = den > 1e-30          # products inside fp32's normal range
    rel_h = ((oh.double() - ref).abs() / den)[ok].max().item()
    rel_t = ((ot.double() - ref).abs() / den)[ok].max().item()
    print(f"adversarial: max |err| / (|a||w|)  h {rel_h:.2e}  torch fp32 {rel_t:.2e}  "
          f"finite {bool(torch.isfinite(oh).all())}")
    # transposed weight image (dX orientation)
    w2 = torch.randn(R, C, device=dev, generator=g)
    a2 = torch.randn(Ms, R, device=dev, generator=g)
    o2 = kernels.gemm_nt_h(a2, kernels.gemm_h_weight(w2.t().contiguous()), C)
    o3 = kernels.gemm_nt_h(a2, kernels.gemm_h_weight(w2, transpose=True), C)
    torch.cuda.synchronize()
    print("transpose image equal:", bool(torch.equal(o2, o3)),
          "err", err(o3, a2.double() @ w2.double()))


if __name__ == "__main__":
    main()
