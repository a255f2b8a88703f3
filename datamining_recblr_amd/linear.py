"""Projection GEMMs with split-K weight gradients.

Every projection of the encoder is tall and skinny: X [B*L, K] @ W^T with
B*L = 409,600 rows at the benchmark shape and K, N in {128, 256, 512}.  The
forward and dX GEMMs have plenty of output tiles, but the weight gradient
dW = dY^T X [N, K] has only a few dozen tiles and a 409,600-long reduction, on
which the BLAS picks un-split kernels running at ~46 TFLOP/s (MI355X fp32
MFMA peak 157).  Splitting the reduction into S row blocks as one batched GEMM
([S, N, M/S] x [S, M/S, K], ~1000 tiles) and summing the S partials in a fixed
order runs 2-4.5x faster (tools/gemm_probe.py) and is deterministic.

All GEMMs run on hipBLASLt/rocBLAS MFMA kernels through torch; the math is
exactly nn.Linear's (RecBLR.py:162,165,167,213,214).
"""
from __future__ import annotations

import torch

from . import gemm_tuning, kernels

__all__ = ["linear", "wgrad", "LinearFn"]

SPLIT_K = 64
MIN_ROWS_FOR_SPLIT = 16384


def wgrad(dy2: torch.Tensor, x2: torch.Tensor, splits: int = SPLIT_K) -> torch.Tensor:
    """dW = dy2^T @ x2 for dy2 [M, N], x2 [M, K] (row-strided views allowed)."""
    M = dy2.shape[0]
    if M < MIN_ROWS_FOR_SPLIT or splits <= 1:
        return dy2.t() @ x2
    mk = M // splits
    main = mk * splits
    a = dy2[:main].unflatten(0, (splits, mk)).transpose(1, 2)
    b = x2[:main].unflatten(0, (splits, mk))
    out = kernels.colsum(torch.bmm(a, b).view(splits, -1)).view(a.shape[1], b.shape[2])
    if main < M:
        out += dy2[main:].t() @ x2[main:]
    return out


def _timed(kind, flops, fn, *args, **kw):
    """Run a GEMM, bracketed by HIP events when bench.py's kernel timer is on."""
    t = kernels._timer
    if t is None:
        return fn(*args, **kw)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    out = fn(*args, **kw)
    e1.record()
    t.records.append((kind, flops, e0, e1))
    return out


class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, slot=None):
        x2 = x.reshape(-1, x.shape[-1])
        flops = 2 * x2.shape[0] * x2.shape[1] * weight.shape[0]
        if bias is not None:
            y = _timed("gemm", flops, torch.addmm, bias, x2, weight.t())
        else:
            y = _timed("gemm", flops, torch.mm, x2, weight.t())
        ctx.save_for_backward(x2, weight)
        ctx.has_bias = bias is not None
        ctx.slot = slot
        return y.view(*x.shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        flops = 2 * x2.shape[0] * x2.shape[1] * weight.shape[0]
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            slot = ctx.slot
            if slot is not None and slot.ds is not None and slot.rows is None:
                # + a handed-over residual gradient, inside the GEMM (beta = 1)
                dx = _timed("gemm", flops, slot.ds.view(-1, weight.shape[1]).addmm_, dy2, weight)
                slot.ds = None
            else:
                dx = _timed("gemm", flops, torch.mm, dy2, weight)
                if slot is not None and slot.ds is not None:   # residual of gathered rows
                    dx.index_add_(0, slot.rows, slot.ds.view(-1, weight.shape[1]))
                    slot.ds = None
            dx = dx.view(*dy.shape[:-1], weight.shape[1])
        if ctx.needs_input_grad[1]:
            dw = _timed("gemm", flops, wgrad, dy2, x2)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = kernels.colsum(dy2.contiguous())
        return dx, dw, db, None


def linear(x: torch.Tensor, module: torch.nn.Linear, slot=None) -> torch.Tensor:
    """module(x) with the split-K weight gradient; `slot` (blocks.ResidualGrad)
    adds a residual gradient inside the dX GEMM."""
    if _tuned is None and x.is_cuda:
        _load_tuned()
    return LinearFn.apply(x, module.weight, module.bias, slot)


_tuned = None


def _load_tuned():
    global _tuned
    _tuned = gemm_tuning.use_tuned_gemms()
