"""Fused HIP blocks around the BD-LRU: embedding gather + dropout + LayerNorm,
dropout + residual + LayerNorm, and the FFN's SiLU + dropout.

Reference spans: RecBLR.py:76-78 (embedding -> dropout -> LayerNorm), :142
(LayerNorm(dropout(GRL(x)) + x)), :219-225 (FeedForward).  Dropout masks are
drawn with torch's generator (``bernoulli_``), so ``torch.manual_seed`` keeps
training reproducible; in eval mode or at p = 0 there is no mask at all.
LayerNorm widths outside ``kernels.LN_SIZES`` use torch's own (GPU) ops.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import kernels
from ._lib import RecBLRNativeError

__all__ = ["dropout_mask", "add_dropout_layer_norm", "embed_dropout_layer_norm",
           "silu_dropout"]


def dropout_mask(shape, p: float, training: bool, device):
    """uint8 keep-mask ~ Bernoulli(1 - p) and the 1/(1-p) scale (None, 1 if off)."""
    if not training or p == 0.0:
        return None, 1.0
    if p >= 1.0:
        return torch.zeros(shape, dtype=torch.uint8, device=device), 0.0
    return torch.empty(shape, dtype=torch.uint8, device=device).bernoulli_(1.0 - p), 1.0 / (1.0 - p)


def _require_gpu(t):
    if t.device.type != "cuda":
        raise RecBLRNativeError(
            "the RecBLR blocks run on the MI355X HIP path only (ROCm GPU tensors)")


class _AddDropoutLN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, r, gamma, beta, mask, scale, eps):
        d = a.shape[-1]
        save = any(ctx.needs_input_grad)
        y, s, mean, rstd = kernels.add_ln_fwd(a.reshape(-1, d).contiguous(),
                                              r.reshape(-1, d).contiguous(), mask, scale,
                                              gamma, beta, eps, save=save)
        ctx.scale = scale
        ctx.save_for_backward(s, mean, rstd, gamma, mask)
        return y.view(a.shape)

    @staticmethod
    def backward(ctx, dy):
        s, mean, rstd, gamma, mask = ctx.saved_tensors
        need_a, need_r = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        ds, da, dg, db = kernels.add_ln_bwd(dy, s, gamma, mean, rstd, mask, ctx.scale,
                                            want_ds=need_r, want_da=need_a or not need_r)
        shape = dy.shape
        return (da.view(shape) if need_a else None, ds.view(shape) if need_r else None,
                dg, db, None, None, None)


class _EmbedDropoutLN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, table, idx, gamma, beta, mask, scale, eps, padding_idx):
        save = any(ctx.needs_input_grad)
        flat = idx.reshape(-1).contiguous()
        y, s, mean, rstd = kernels.add_ln_fwd(table, None, mask, scale, gamma, beta, eps,
                                              idx=flat, save=save)
        ctx.scale, ctx.padding_idx, ctx.num_rows = scale, padding_idx, table.shape[0]
        ctx.save_for_backward(s, mean, rstd, gamma, mask, flat)
        return y.view(*idx.shape, table.shape[1])

    @staticmethod
    def backward(ctx, dy):
        s, mean, rstd, gamma, mask, flat = ctx.saved_tensors
        _, da, dg, db = kernels.add_ln_bwd(dy, s, gamma, mean, rstd, mask, ctx.scale,
                                           want_ds=False, want_da=True)
        dtable = (kernels.embedding_bwd(flat, da, ctx.num_rows, ctx.padding_idx)
                  if ctx.needs_input_grad[0] else None)
        return dtable, None, dg, db, None, None, None, None


class _SiluDropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, mask, scale):
        a = a.contiguous()
        ctx.scale = scale
        ctx.save_for_backward(a, mask)
        return kernels.silu_dropout_fwd(a, mask, scale)

    @staticmethod
    def backward(ctx, du):
        a, mask = ctx.saved_tensors
        return kernels.silu_dropout_bwd(a, mask, ctx.scale, du), None, None


def add_dropout_layer_norm(a, residual, dropout: torch.nn.Dropout, ln: torch.nn.LayerNorm,
                           training: bool):
    """ln(dropout(a) + residual) — RecBLR.py:142 and :224-225."""
    _require_gpu(a)
    d = a.shape[-1]
    if d not in kernels.LN_SIZES or a.numel() % 4:
        return ln(dropout(a) + residual)
    mask, scale = dropout_mask((a.numel() // d, d), dropout.p, training, a.device)
    return _AddDropoutLN.apply(a, residual, ln.weight, ln.bias, mask, scale, ln.eps)


def embed_dropout_layer_norm(idx, emb: torch.nn.Embedding, dropout: torch.nn.Dropout,
                             ln: torch.nn.LayerNorm, training: bool):
    """ln(dropout(emb(idx))) — RecBLR.py:76-78."""
    _require_gpu(emb.weight)
    d = emb.weight.shape[1]
    if d not in kernels.LN_SIZES:
        return ln(dropout(emb(idx)))
    mask, scale = dropout_mask((idx.numel(), d), dropout.p, training, idx.device)
    return _EmbedDropoutLN.apply(emb.weight, idx, ln.weight, ln.bias, mask, scale, ln.eps,
                                 emb.padding_idx)


def silu_dropout(a, dropout: torch.nn.Dropout, training: bool):
    """dropout(silu(a)) — RecBLR.py:220-221."""
    _require_gpu(a)
    if a.numel() % 4:
        return dropout(F.silu(a))
    mask, scale = dropout_mask(a.shape, dropout.p, training, a.device)
    return _SiluDropout.apply(a, mask, scale)
