"""``torch.library`` custom ops over the C-ABI (callers see
registered operators, not opaque ctypes calls).

Each op has a fake (meta) implementation, so ``torch.compile`` /
``torch.export`` trace through it without a graph break, and an autograd
formula registered with ``torch.library.register_autograd``:

* ``recblr::scan_fwd`` / ``recblr::scan_bwd`` — the reference's kernel API,
  ``parallel_scan(gates, tokens)`` (parallel_scan.py:83-118); ``scan.py``'s
  ``parallel_scan`` is the differentiable ``scan_fwd``.
* ``recblr::linear`` — ``F.linear`` (RecBLR.py:162,165,167,213,214) on the
  split-operand MFMA GEMMs (linear.py), with the fixed-order weight gradient.

The model itself (model.py) keeps calling its autograd functions directly:
they carry host-side state (packed-sequence plans, residual-gradient slots,
the split-weight cache) that a traced graph cannot hold.
"""
from __future__ import annotations

import torch

from . import kernels

__all__ = ["scan_fwd", "scan_bwd", "linear"]


@torch.library.custom_op("recblr::scan_fwd", mutates_args=())
def scan_fwd(gates: torch.Tensor, tokens: torch.Tensor) -> torch.Tensor:
    """States of h_t = gates_t h_{t-1} + tokens_t along the last dim (rb_scan_fwd)."""
    return kernels.scan_fwd(gates, tokens)


@scan_fwd.register_fake
def _(gates, tokens):
    torch._check(gates.shape == tokens.shape, lambda: "gates and tokens must match")
    return tokens.new_empty(tokens.shape)   # contiguous, like rb_scan_fwd's output


@torch.library.custom_op("recblr::scan_bwd", mutates_args=())
def scan_bwd(gates: torch.Tensor, states: torch.Tensor,
             grad: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """(d_gates, d_tokens) of scan_fwd (rb_scan_bwd)."""
    return kernels.scan_bwd(gates, states, grad.contiguous())


@scan_bwd.register_fake
def _(gates, states, grad):
    return gates.new_empty(gates.shape), gates.new_empty(gates.shape)


def _scan_setup(ctx, inputs, output):
    gates, _ = inputs
    ctx.save_for_backward(output, gates)


def _scan_backward(ctx, grad):
    states, gates = ctx.saved_tensors
    return tuple(scan_bwd(gates, states, grad))


torch.library.register_autograd("recblr::scan_fwd", _scan_backward, setup_context=_scan_setup)


@torch.library.custom_op("recblr::linear", mutates_args=())
def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None) -> torch.Tensor:
    """F.linear on the split-operand GEMM (linear.mm_nt)."""
    from .linear import mm_nt
    x2 = x.reshape(-1, x.shape[-1]).contiguous()
    return mm_nt(x2, weight, bias).view(*x.shape[:-1], weight.shape[0])


@linear.register_fake
def _(x, weight, bias):
    return x.new_empty((*x.shape[:-1], weight.shape[0]))


@torch.library.custom_op("recblr::linear_bwd", mutates_args=())
def linear_bwd(dy: torch.Tensor, x: torch.Tensor, weight: torch.Tensor,
               has_bias: bool) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(dx, dW, db) of recblr::linear (db empty when there is no bias)."""
    from .linear import mm_nn, wgrad
    dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
    x2 = x.reshape(-1, x.shape[-1]).contiguous()
    dx = mm_nn(dy2, weight).view(x.shape)
    dw = wgrad(dy2, x2)
    db = kernels.colsum(dy2) if has_bias else dy2.new_empty((0,))
    return dx, dw, db


@linear_bwd.register_fake
def _(dy, x, weight, has_bias):
    # contiguous like the real outputs (mm_nn(...).view(x.shape), wgrad's [N, K]),
    # whatever x's strides: empty_like would keep a transposed x's strides
    return (x.new_empty(x.shape), weight.new_empty(weight.shape),
            dy.new_empty((weight.shape[0],) if has_bias else (0,)))


def _linear_setup(ctx, inputs, output):
    x, weight, bias = inputs
    ctx.has_bias = bias is not None
    ctx.save_for_backward(x, weight)


def _linear_backward(ctx, dy):
    x, weight = ctx.saved_tensors
    dx, dw, db = linear_bwd(dy, x, weight, ctx.has_bias)
    return dx, dw, (db if ctx.has_bias else None)


torch.library.register_autograd("recblr::linear", _linear_backward, setup_context=_linear_setup)
