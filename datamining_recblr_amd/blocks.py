"""Fused HIP blocks around the BD-LRU.

Reference spans: RecBLR.py:76-78 (embedding -> dropout -> LayerNorm), :142
(LayerNorm(dropout(GRL(x)) + x)), :210-227 (FeedForward).

Dropout keep-flags are a Philox4x32-10 stream inside the kernels, keyed by a
64-bit seed drawn from torch's default (CPU) generator for every dropout site
and call — so ``torch.manual_seed`` makes training reproducible and no mask
tensor is ever written; the backward regenerates the same flags.  In eval mode
or at p = 0 there is no dropout.  Row widths outside ``kernels.ROW_SIZES`` use
torch's own GPU ops.

The FeedForward block is one autograd function: w_1 GEMM -> SiLU+dropout ->
w_2 GEMM -> dropout+residual+LayerNorm.  Its backward takes both bias
gradients from column partials of the row kernels (no separate reduction
passes).  Residual gradients are never summed in a pass of their own: a
tensor read by a projection and by a residual branch gets the residual's
gradient added by its producer's LayerNorm backward while it loads the
projection's input gradient (ResidualGrad, rb_add_ln_bwd2's dy2).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import kernels
from ._lib import RecBLRNativeError
from .linear import (_timed, fire_hooks, has_hooks, linear, mm_nn, mm_nn_dact, mm_nn_dact_ok, mm_nt,
                     mm_nt_act, mm_nt_act_ok, mm_nt_ln, mm_nt_ln_ok, rmax_buffer, wgrad)

__all__ = ["draw_seed", "ResidualGrad", "add_dropout_layer_norm", "embed_dropout_layer_norm",
           "linear_add_dropout_layer_norm", "silu_dropout", "feed_forward", "set_defer_residual",
           "defer_residual"]


_GOLDEN = 0x9E3779B97F4A7C15   # odd 64-bit constant (2^64 / golden ratio)


def _rank() -> int:
    dist = torch.distributed
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def draw_seed() -> int:
    """63-bit dropout seed from torch's default generator (host side, no sync).

    The reference's driver re-seeds every process with seed + local_rank
    before building the model (run.py:72), so under it the ranks' generators
    already differ.  The process-group rank is folded in as a guard for
    launchers that seed every rank alike (bench.py seeds 2020 everywhere, so
    the ranks' weights start equal): without it all data-parallel ranks would
    draw identical dropout masks for their different batch shards.  Rank 0
    (and a single process) keeps the generator's value unchanged; rank r's
    masks therefore differ from a single process seeded with seed + r."""
    s = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())
    r = _rank()
    if r:
        s = (s + r * _GOLDEN) % (2 ** 62)
    return s


def _drop(dropout: torch.nn.Dropout, training: bool):
    p = float(dropout.p) if training else 0.0
    return p, (draw_seed() if p > 0.0 else 0)


def _require_gpu(t):
    if t.device.type != "cuda":
        raise RecBLRNativeError(
            "the RecBLR blocks run on the MI355X HIP path only (ROCm GPU tensors)")


class ResidualGrad:
    """A second gradient of one tensor, handed from the consumer that computes
    it to the producer of the tensor, whose LayerNorm backward adds it while
    loading its output gradient (rb_add_ln_bwd2's dy2) — instead of autograd
    summing two [rows, d] gradients in a separate pass.

    Uses: the residual branch of RecurrentLayer (RecBLR.py:142,
    LN(dropout(GRL(x)) + x)): its LayerNorm backward sets ``ds``, the GRL's
    input projection leaves it (``taken``: x's producer, the previous layer's
    FeedForward or the embedding LayerNorm, registered to add it) and x's
    producer adds it; the FeedForward's own residual (RecBLR.py:227) handed to
    the LayerNorm that produced its input.  The consumer's backward always
    runs before the producer's.  ``rows``: when the residual LayerNorm ran on
    a gathered subset of the positions (the last layer, see RecBLR.forward),
    the flat rows its residual came from (then the input projection adds it
    with index_add, and no producer takes it)."""
    __slots__ = ("ds", "rows", "taken")

    def __init__(self, rows=None):
        self.ds = None
        self.rows = rows
        self.taken = False


# Deferred residual gradients change what autograd reports for the tensor in
# between: its producer adds the residual term inside its own backward, so a
# tensor hook, retain_grad() or torch.autograd.grad(loss, h) on h (a
# RecurrentLayer output, the embedding LayerNorm output, a FeedForward input)
# sees only the projection's term.  Parameter and input gradients are exact
# either way.  RECBLR_DEFER_RESIDUAL=0 (or set_defer_residual(False)) makes the
# consumer add the residual term to the gradient it returns, so every
# intermediate gradient is the full one (one extra [rows, d] add per slot).
_defer_residual = [os.environ.get("RECBLR_DEFER_RESIDUAL", "1") != "0"]


def set_defer_residual(on: bool) -> None:
    """Switch residual-gradient deferral (see _defer_residual) for models
    run after this call."""
    _defer_residual[0] = bool(on)


def defer_residual() -> bool:
    return _defer_residual[0]


def _take(addend):
    """Register a producer for `addend` (it will add addend.ds itself)."""
    if addend is not None and addend.rows is None and _defer_residual[0]:
        addend.taken = True
        return addend
    return None


def _pop(addend):
    if addend is None:
        return None
    ds, addend.ds = addend.ds, None
    return ds


class _AddDropoutLN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, r, gamma, beta, mask, seed, p, eps, slot=None, addend=None):
        d = a.shape[-1]
        save = any(ctx.needs_input_grad)
        y, s, mean, rstd = kernels.add_ln_fwd(a.reshape(-1, d).contiguous(),
                                              r.reshape(-1, d).contiguous(), gamma, beta, eps,
                                              mask=mask, seed=seed, p=p, save=save)
        ctx.seed, ctx.p, ctx.slot = seed, p, slot
        ctx.addend = _take(addend)
        ctx.save_for_backward(s, mean, rstd, gamma, mask)
        return y.view(a.shape)

    @staticmethod
    def backward(ctx, dy):
        s, mean, rstd, gamma, mask = ctx.saved_tensors
        need_a, need_r = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        ds, da, dg, db, _ = kernels.add_ln_bwd(dy, s, gamma, mean, rstd, mask=mask,
                                               seed=ctx.seed, p=ctx.p, want_ds=need_r,
                                               want_da=need_a or not need_r,
                                               dy2=_pop(ctx.addend))
        shape = dy.shape
        if need_r and ctx.slot is not None:   # handed to the GRL input projection
            ctx.slot.ds = ds
            ds, need_r = None, False
        return (da.view(shape) if need_a else None, ds.view(shape) if need_r else None,
                dg, db, None, None, None, None, None, None)


class _LinearAddDropoutLN(torch.autograd.Function):
    """LayerNorm(dropout(x W^T) + residual) with the projection's GEMM and the
    residual LayerNorm in one launch (rb_gemm_nt_h_ln): the recurrent layer's
    out-projection and its residual LayerNorm, RecBLR.py:142, 167.  Backward:
    rb_add_ln_bwd2, then the projection's input and weight gradients as
    LinearFn's (the projection has no bias)."""

    @staticmethod
    def forward(ctx, x, w, residual, gamma, beta, seed, p, eps, slot=None, addend=None):
        d = w.shape[0]
        x2 = x.reshape(-1, x.shape[-1])
        r2 = residual.reshape(-1, d).contiguous()
        f = 2 * x2.shape[0] * x2.shape[1] * d
        rx = rmax_buffer(x2, d, x2.shape[1]) if ctx.needs_input_grad[1] else None
        y, s, mean, rstd = _timed("gemm", f, mm_nt_ln, x2, w, None, r2, gamma, beta, eps, seed, p,
                                  rmax=rx)
        ctx.seed, ctx.p, ctx.slot, ctx.rx = seed, p, slot, rx
        ctx.xshape = x.shape
        ctx.addend = _take(addend)
        ctx.save_for_backward(x2, w, s, mean, rstd, gamma)
        return y.view(residual.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, s, mean, rstd, gamma = ctx.saved_tensors
        need_x, need_w, need_r = ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        ds, da, dg, db, _ = kernels.add_ln_bwd(dy, s, gamma, mean, rstd, seed=ctx.seed, p=ctx.p,
                                               want_ds=need_r, want_da=True,
                                               dy2=_pop(ctx.addend))
        if need_r and ctx.slot is not None:   # handed to the GRL input projection
            ctx.slot.ds = ds
            ds, need_r = None, False
        d = w.shape[0]
        da2 = da.reshape(-1, d)
        f = 2 * x2.shape[0] * x2.shape[1] * d
        dx = dw = ry = None
        if need_x:
            ry = rmax_buffer(da2, x2.shape[1], d) if ctx.rx is not None else None
            dx = _timed("gemm", f, mm_nn, da2, w, rmax=ry).view(ctx.xshape)
        if need_w:
            dw = _timed("gemm", f, wgrad, da2, x2, ymax=ry, xmax=ctx.rx)
        return (dx, dw, ds.view(dy.shape) if need_r else None, dg, db, None, None, None, None,
                None)


class _EmbedDropoutLN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, table, idx, gamma, beta, mask, seed, p, eps, padding_idx, addend=None):
        save = any(ctx.needs_input_grad)
        flat = idx.reshape(-1).contiguous()
        plan = None
        if ctx.needs_input_grad[0]:
            # the embedding backward's sort (it depends on the ids only), on the
            # current stream: on a side stream beside the forward it cost the
            # step 0.5% more than its 97 us of kernels
            plan = kernels.embedding_plan(flat, table.shape[0], table.shape[1])
        y, s, mean, rstd = kernels.add_ln_fwd(table, None, gamma, beta, eps, mask=mask,
                                              seed=seed, p=p, idx=flat, save=save)
        ctx.seed, ctx.p = seed, p
        ctx.padding_idx, ctx.num_rows = padding_idx, table.shape[0]
        ctx.plan = plan
        ctx.addend = _take(addend)
        ctx.save_for_backward(s, mean, rstd, gamma, mask, flat)
        return y.view(*idx.shape, table.shape[1])

    @staticmethod
    def backward(ctx, dy):
        s, mean, rstd, gamma, mask, flat = ctx.saved_tensors
        _, da, dg, db, _ = kernels.add_ln_bwd(dy, s, gamma, mean, rstd, mask=mask,
                                              seed=ctx.seed, p=ctx.p, want_ds=False,
                                              want_da=True, dy2=_pop(ctx.addend))
        dtable = None
        if ctx.needs_input_grad[0]:
            dtable = kernels.embedding_bwd(flat, da, ctx.num_rows, ctx.padding_idx,
                                           plan=ctx.plan)
            ctx.plan = None
        return dtable, None, dg, db, None, None, None, None, None, None


class _SiluDropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, mask, seed, p):
        a = a.contiguous()
        ctx.seed, ctx.p = seed, p
        ctx.save_for_backward(a, mask)
        return kernels.silu_dropout_fwd(a, mask=mask, seed=seed, p=p)

    @staticmethod
    def backward(ctx, du):
        a, mask = ctx.saved_tensors
        da, _ = kernels.silu_dropout_bwd(a, du, mask=mask, seed=ctx.seed, p=ctx.p)
        return da, None, None, None


class _FeedForward(torch.autograd.Function):
    """LN(dropout(W2 dropout(silu(W1 x + b1)) + b2) + x), RecBLR.py:218-227."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, gamma, beta, seed1, seed2, p, eps, in_addend=None,
                out_addend=None, observe=None):
        d = x.shape[-1]
        x2 = x.reshape(-1, d)
        M, inner = x2.shape[0], w1.shape[0]
        f = 2 * M * d * inner
        # b1 is added inside the activation kernel (the bias epilogue of the
        # library GEMM costs more than the add on the fly)
        # row-group maxima of the GEMM inputs: the weight gradients' operand scales
        want = ctx.needs_input_grad[1] or ctx.needs_input_grad[3]
        r_x = rmax_buffer(x2, inner, d) if want else None
        # a1 = x W1^T + b1 and u = dropout(silu(a1)) from one GEMM epilogue
        # where it applies (b1 then lives in a1: the backward gets no bias)
        if mm_nt_act_ok(x2, w1):
            (a1, u), a1_bias = _timed("gemm", f, mm_nt_act, x2, w1, b1, seed1, p, rmax=r_x), None
        else:
            a1 = _timed("gemm", f, mm_nt, x2, w1, rmax=r_x)
            u = kernels.silu_dropout_fwd(a1, seed=seed1, p=p, bias=b1)
            a1_bias = b1
        r_u = rmax_buffer(u, d, inner) if want else None
        save = any(ctx.needs_input_grad)
        x2c = x2.contiguous()
        if observe is None and mm_nt_ln_ok(u, w2):
            # a2 = u W2^T + b2 never stored: the residual + dropout + LayerNorm
            # in the GEMM's epilogue (rb_gemm_nt_h_ln)
            y, s, mean, rstd = _timed("gemm", f, mm_nt_ln, u, w2, b2, x2c, gamma, beta, eps,
                                      seed2, p, rmax=r_u)
        else:
            a2 = _timed("gemm", f, mm_nt, u, w2, b2, rmax=r_u)
            if observe is not None:   # module hooks of w_1 / w_2 (feed_forward)
                pre = a1 if a1_bias is None else a1 + a1_bias
                observe(x2.view(x.shape), pre.view(*x.shape[:-1], inner),
                        u.view(*x.shape[:-1], inner), a2.view(x.shape))
            y, s, mean, rstd = kernels.add_ln_fwd(a2, x2c, gamma, beta, eps, seed=seed2, p=p,
                                                  save=save)
        ctx.r_x, ctx.r_u = r_x, r_u
        ctx.seed1, ctx.seed2, ctx.p = seed1, seed2, p
        ctx.a1_has_bias = a1_bias is None
        # in_addend: x's producer takes the residual's gradient (see ResidualGrad)
        ctx.in_addend = in_addend if in_addend is not None and in_addend.taken else None
        ctx.out_addend = _take(out_addend)
        ctx.save_for_backward(x2, a1, u, s, mean, rstd, w1, b1, w2, gamma)
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, a1, u, s, mean, rstd, w1, b1, w2, gamma = ctx.saved_tensors
        M, d = x2.shape
        f = 2 * M * d * w1.shape[0]
        ds, da2, dgamma, dbeta, db2 = kernels.add_ln_bwd(
            dy, s, gamma, mean, rstd, seed=ctx.seed2, p=ctx.p, want_ds=True, want_da=True,
            want_dbias=True, dy2=_pop(ctx.out_addend))
        r_da2 = rmax_buffer(da2, w2.shape[1], d) if ctx.r_u is not None else None
        if ctx.a1_has_bias and mm_nn_dact_ok(da2, w2):
            # du never stored: the activation backward in the GEMM epilogue
            da1, db1 = _timed("gemm", f, mm_nn_dact, da2, w2, a1, ctx.seed1, ctx.p, rmax=r_da2)
            dw2 = _timed("gemm", f, wgrad, da2, u, ymax=r_da2, xmax=ctx.r_u)
        else:
            du = _timed("gemm", f, mm_nn, da2, w2, rmax=r_da2)
            dw2 = _timed("gemm", f, wgrad, da2, u, ymax=r_da2, xmax=ctx.r_u)
            da1, db1 = kernels.silu_dropout_bwd(a1, du, seed=ctx.seed1, p=ctx.p, want_dbias=True,
                                                bias=None if ctx.a1_has_bias else b1)
        r_da1 = rmax_buffer(da1, d, w1.shape[0]) if ctx.r_x is not None else None
        dx = _timed("gemm", f, mm_nn, da1, w1, rmax=r_da1)
        if ctx.in_addend is not None:   # x's producer adds the residual's gradient
            ctx.in_addend.ds = ds
        else:
            dx.add_(ds)
        dw1 = _timed("gemm", f, wgrad, da1, x2, ymax=r_da1, xmax=ctx.r_x)
        return (dx.view(dy.shape), dw1, db1, dw2, db2, dgamma, dbeta, None, None, None, None,
                None, None, None)


def add_dropout_layer_norm(a, residual, dropout: torch.nn.Dropout, ln: torch.nn.LayerNorm,
                           training: bool, slot: ResidualGrad | None = None,
                           addend: ResidualGrad | None = None):
    """ln(dropout(a) + residual) — RecBLR.py:142.  With `slot`, the residual's
    gradient is handed over instead of returned; `addend`: a second gradient
    of the output that its consumer hands back (see ResidualGrad)."""
    _require_gpu(a)
    if a.shape[-1] not in kernels.ROW_SIZES:
        return ln(dropout(a) + residual)
    p, seed = _drop(dropout, training)
    return _AddDropoutLN.apply(a, residual, ln.weight, ln.bias, None, seed, p, ln.eps, slot,
                               addend)


def linear_add_dropout_layer_norm(x, proj: torch.nn.Linear, residual, dropout: torch.nn.Dropout,
                                  ln: torch.nn.LayerNorm, training: bool,
                                  slot: ResidualGrad | None = None,
                                  addend: ResidualGrad | None = None):
    """ln(dropout(proj(x)) + residual) — RecBLR.py:142 after :167 — as one
    GEMM launch with the LayerNorm in its epilogue where rb_gemm_nt_h_ln
    applies (d = 128 outputs, no bias, from 16,384 rows on the
    weight-stationary kernel); else the projection (its module call, hooks
    included) and add_dropout_layer_norm.  slot / addend as there."""
    _require_gpu(x)
    x2 = x.reshape(-1, x.shape[-1])
    if proj.bias is None and ln.weight.shape[0] == proj.weight.shape[0] and mm_nt_ln_ok(x2, proj.weight):
        p, seed = _drop(dropout, training)
        return _LinearAddDropoutLN.apply(x, proj.weight, residual, ln.weight, ln.bias, seed, p,
                                         ln.eps, slot, addend)
    return add_dropout_layer_norm(proj(x), residual, dropout, ln, training, slot, addend)


def embed_dropout_layer_norm(idx, emb: torch.nn.Embedding, dropout: torch.nn.Dropout,
                             ln: torch.nn.LayerNorm, training: bool,
                             addend: ResidualGrad | None = None):
    """ln(dropout(emb(idx))) — RecBLR.py:76-78 (`addend`: see ResidualGrad)."""
    _require_gpu(emb.weight)
    if emb.weight.shape[1] not in kernels.ROW_SIZES:
        return ln(dropout(emb(idx)))
    p, seed = _drop(dropout, training)
    return _EmbedDropoutLN.apply(emb.weight, idx, ln.weight, ln.bias, None, seed, p, ln.eps,
                                 emb.padding_idx, addend)


def silu_dropout(a, dropout: torch.nn.Dropout, training: bool):
    """dropout(silu(a)) — RecBLR.py:220-221."""
    _require_gpu(a)
    if a.shape[-1] not in kernels.ROW_SIZES:
        return dropout(F.silu(a))
    p, seed = _drop(dropout, training)
    return _SiluDropout.apply(a, None, seed, p)


def feed_forward(x, ffn, training: bool, in_addend: ResidualGrad | None = None,
                 out_addend: ResidualGrad | None = None):
    """The whole FeedForward block (RecBLR.py:218-227) as one fused function.
    in_addend: the slot through which x's producer takes the block's residual
    gradient; out_addend: a second gradient of the output (see ResidualGrad)."""
    _require_gpu(x)
    d, inner = x.shape[-1], ffn.w_1.weight.shape[0]
    if d not in kernels.ROW_SIZES or inner not in kernels.ROW_SIZES:
        h = silu_dropout(linear(x, ffn.w_1), ffn.dropout, training)
        return add_dropout_layer_norm(linear(h, ffn.w_2), x, ffn.dropout, ffn.layer_norm,
                                      training)
    observe = None
    if has_hooks(ffn.w_1) or has_hooks(ffn.w_2):
        def observe(x_, a1, u, a2):
            fire_hooks(ffn.w_1, (x_,), a1)
            fire_hooks(ffn.w_2, (u,), a2)
    p, seed1 = _drop(ffn.dropout, training)
    seed2 = draw_seed() if p > 0.0 else 0
    return _FeedForward.apply(x, ffn.w_1.weight, ffn.w_1.bias, ffn.w_2.weight, ffn.w_2.bias,
                              ffn.layer_norm.weight, ffn.layer_norm.bias, seed1, seed2, p,
                              ffn.layer_norm.eps, in_addend, out_addend, observe)
