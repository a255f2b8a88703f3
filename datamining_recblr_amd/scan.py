"""``parallel_scan(gates, tokens)`` — drop-in for the reference's
``parallel_scan.py:117-118``.

Same contract as the reference ``Scan`` autograd function
(parallel_scan.py:83-114): inputs ``[B, C, T]`` fp32 contiguous, output the
states of ``h_t = gates_t * h_{t-1} + tokens_t`` with ``h_{-1} = 0``; the
backward returns ``(d_gates, d_tokens)`` with ``d_t = grad_t + gates_{t+1}
d_{t+1}`` and ``d_gates_t = h_{t-1} d_t``.  Unlike the Triton version T does
not need to be a power of two.  Both directions run the gfx950 wave-shuffle
scan (``rb_scan_fwd`` / ``rb_scan_bwd``); there is no CPU path.
``parallel_scan`` dispatches the registered operator ``recblr::scan_fwd``
(ops.py: fake implementation + autograd, so ``torch.compile`` traces it
without a graph break); ``Scan`` is the same computation as an
``autograd.Function``.
"""
from __future__ import annotations

import torch

from . import kernels, ops

__all__ = ["Scan", "parallel_scan"]


class Scan(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gates, tokens):
        B, C, T = gates.shape
        # the reference's preconditions (parallel_scan.py:86-89)
        assert tokens.shape == (B, C, T)
        assert gates.is_contiguous()
        assert tokens.is_contiguous()
        states = kernels.scan_fwd(gates, tokens)
        ctx.save_for_backward(states, gates)
        return states

    @staticmethod
    def backward(ctx, grad_output):
        states, gates = ctx.saved_tensors
        grad_output = grad_output.contiguous()
        assert states.is_contiguous()
        assert gates.is_contiguous()
        d_gates, d_tokens = kernels.scan_bwd(gates, states, grad_output)
        return d_gates, d_tokens


def parallel_scan(gates, tokens):
    # the reference's preconditions (parallel_scan.py:86-89)
    assert tokens.shape == gates.shape and gates.dim() == 3
    assert gates.is_contiguous()
    assert tokens.is_contiguous()
    return ops.scan_fwd(gates, tokens)
