"""The fused BD-LRU block of ``GatedRecurrentLayer.forward``.

Reference span: RecBLR.py:173-206.  The reference materialises a power-of-two
left padding (:176-179), runs the conv on the padded ``[B, H, T]`` transpose
(:185), computes the gates with ~12 elementwise torch kernels (:196-199),
transposes twice into ``parallel_scan`` (:200), truncates (:203-204) and
merges (:206).

Here the padding is never materialised.  Pad positions carry zeros into the
conv, so every pad step sees the same per-channel constants
``xc_p = silu(conv.bias)``, ``(r_p, i_p) = gates(xc_p)``, ``alpha_p``,
``b'_p = beta_p * xc_p`` (batch independent).  After ``P = T - L`` such steps
the recurrence holds ``h0 = b'_p (1 - alpha_p^P) / (1 - alpha_p)``, which seeds
the scan over the L real steps; real steps never see pad inputs through the
conv because the reference's causal conv already zero-pads the history.  The
``[H]``-sized prefix is one small HIP launch each way (rb_pad_prefix_fwd /
_bwd; ``pad_prefix_state`` is the same math in torch, kept as the checked
reference), and everything ``[B, L, *]``-sized runs in the HIP kernels:

    K1  rb_conv_silu_fwd    x -> xc                    (R x, W xc)
    G   torch addmm         xc @ W_g^T + b_g -> rg     (MFMA GEMM)
    K2  rb_gate_scan_fwd    rg, xc, z -> y             (R r,i,xc,z; W y)
and the mirror-image backward (K2^T, two GEMMs, K1^T).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import kernels
from . import linear as linear_mod
from .linear import _timed, mm_nn, mm_nt, rmax_buffer, wgrad

__all__ = ["pow2_pad_len", "row_pad_lens", "pad_prefix_state", "PadPrefix", "BDLRUCore",
           "bd_lru"]


_FOLD_PAD = os.environ.get("RECBLR_FOLD_PAD", "1") != "0"
# RECBLR_FUSED_GRL=1: the fused rb_grl_fwd (conv + gates GEMM + gate scan in
# one launch) on packed fp32 sequences with H = 256 instead of the three
# launches.  Off by default: not faster in the step on MI355X (DESIGN.md §4,
# "Fused GatedRecurrentLayer kernels"; bench.py's fused_grl A/B)
_FUSED = os.environ.get("RECBLR_FUSED_GRL", "0") != "0"
# RECBLR_FUSED_GRL_BWD=1: with the fused forward, the one-launch backward
# rb_grl_bwd from the forward's 64-row tile checkpoints instead of the
# three-launch backward (from the xc, rg and 16-step carries the fused
# forward then writes).  Off by default: slower on MI355X
_FUSED_BWD = os.environ.get("RECBLR_FUSED_GRL_BWD", "0") != "0"


# order of the backward's conv and gates weight gradient (see BDLRUCore.backward)
_CONV_FIRST = os.environ.get("RECBLR_CONV_FIRST", "1") != "0"


def set_conv_first(on: bool) -> bool:
    """Set the backward order (bench A/B); returns the previous setting."""
    global _CONV_FIRST
    prev, _CONV_FIRST = _CONV_FIRST, bool(on)
    return prev


def fused_ok(has_pieces: bool, H: int, use_conv: bool, kc: int, dtype) -> bool:
    """Whether BDLRUCore's forward runs as one rb_grl_fwd launch (has_pieces:
    the packed batch carries the kernel's work lists)."""
    return (_FUSED and has_pieces and use_conv and H == 256
            and kc in (2, 3, 4) and dtype == torch.float32 and linear_mod.gemm_format() == "f16x3")


def pow2_pad_len(seq_len: int) -> int:
    """Left padding the reference adds so T is a power of two (RecBLR.py:177)."""
    return (1 << (seq_len - 1).bit_length()) - seq_len


def pad_prefix_state(conv_bias, gate_w, gate_b, lam, pad_len):
    """Recurrent state after the ``pad_len`` constant pad steps (see module doc).

    All operands are ``[H]`` / ``[2H, H]`` parameters.  ``pad_len`` is an int
    (result ``[H]``) or an int64 tensor ``[B]`` of per-row pad lengths (result
    ``[B, H]``, for rows that stand for sequences of different true lengths).
    Differentiable w.r.t. every parameter."""
    xc_p = F.silu(conv_bias)
    r_p, i_p = F.linear(xc_p, gate_w, gate_b).chunk(2, dim=-1)
    s = F.softplus(lam) * torch.sigmoid(r_p)          # alpha_p = exp(-s)
    alpha = torch.exp(-s)
    beta = torch.sqrt(1 - alpha * alpha + 1e-8) * torch.sigmoid(i_p)
    b_p = beta * xc_p
    s = s.clamp_min(1e-20)
    if torch.is_tensor(pad_len):
        pad_len = pad_len.to(s.dtype)[:, None]
    # sum_{k<P} alpha^k = (1 - alpha^P) / (1 - alpha), cancellation-free
    return b_p * (torch.expm1(-pad_len * s) / torch.expm1(-s))


class PadPrefix(torch.autograd.Function):
    """pad_prefix_state on the HIP path: one launch forward, one backward
    (rb_pad_prefix_fwd / _bwd) instead of ~60 [H]-sized torch kernels."""

    @staticmethod
    def forward(ctx, conv_b, gate_w, gate_b, lam, pad_len):
        ctx.pad_len = pad_len
        ctx.save_for_backward(conv_b, gate_w, gate_b, lam)
        return kernels.pad_prefix_fwd(conv_b, gate_w, gate_b, lam, pad_len)

    @staticmethod
    def backward(ctx, dh0):
        conv_b, gate_w, gate_b, lam = ctx.saved_tensors
        dcb, dgw, dgb, dlam = kernels.pad_prefix_bwd(conv_b, gate_w, gate_b, lam, ctx.pad_len,
                                                     dh0.float())
        return dcb, dgw, dgb, dlam, None


class BDLRUCore(torch.autograd.Function):
    """xz [B, L, 2H] (or packed [ntok, 2H] with `seq`) -> y = silu(z) *
    BD-LRU(conv_silu(x)), in xz's layout."""

    @staticmethod
    def forward(ctx, xz, conv_w, conv_b, gate_w, gate_b, lam, h0, use_conv, seq=None,
                last_only=False, pad_len=None, observe=None):
        """h0: an initial state given as an input (its gradient returned), or
        pad_len (int P > 0 or int64 [B] per-row lengths) with h0 None: the
        pad-prefix state computed here, its gradient added in place into the
        parameters' gradients (no separate autograd node and add launches)."""
        if pad_len is not None:
            h0 = kernels.pad_prefix_fwd(conv_b, gate_w, gate_b, lam, pad_len)
        ctx.pad_len = pad_len
        H2 = xz.shape[-1]
        H = H2 // 2
        x, z = xz[..., :H], xz[..., H:]
        train = any(ctx.needs_input_grad)
        # last_only on packed sequences: y_last in batch order (seq.order)
        batch_row = seq.order if (last_only and seq is not None) else None
        ctx.batch_row = batch_row
        if (observe is None and (h0 is None or h0.dim() == 1)
                and fused_ok(seq is not None and seq.pieces is not None, H, use_conv, conv_w.shape[-1], xz.dtype)):
            # conv + gates GEMM + gate scan in one launch (rb_grl_fwd).  Its
            # backward is one launch too (rb_grl_bwd), from the 64-row tile
            # checkpoints; or the three-launch backward from xc, rg, carries
            ctx.fused_bwd = train and _FUSED_BWD and seq.max_tiles > 0
            y, carries, xc, rg, r_xc = kernels.grl_fwd(
                xz, conv_w, conv_b, linear_mod._weight_split(gate_w, False), gate_b, lam, h0,
                seq, want_y=not last_only, want_train=train, tile_carries=ctx.fused_bwd)
            if batch_row is not None:   # rb_grl_fwd keeps packed order
                y = y.index_select(0, seq.inv)
            ctx.r_xc = r_xc if ctx.needs_input_grad[3] and linear_mod.rmax_wanted() else None
            if ctx.fused_bwd:   # rb_grl_bwd writes xc and both operands' row maxima
                ctx.h0 = h0
                ctx.want_rmax = ctx.needs_input_grad[3] and linear_mod.rmax_wanted()
        else:
            ctx.fused_bwd = False
            if use_conv:
                xc = kernels.conv_silu_fwd(x, conv_w, conv_b, seq=seq)
            else:
                xc = x
            rows = xz.numel() // H2
            gflops = 2 * rows * H * H2
            # gates GEMM without its bias: the gate kernels add gate_b on the fly
            xc2 = xc.reshape(rows, H)
            r_xc = rmax_buffer(xc2, H2, H) if ctx.needs_input_grad[3] else None
            rg = _timed("gemm", gflops, mm_nt, xc2, gate_w, rmax=r_xc).view(*xz.shape[:-1], H2)
            ctx.r_xc = r_xc
            if observe is not None:   # module hooks of the fused conv / gates (model.py)
                observe(x, xc, rg)
            y, carries = kernels.gate_scan_fwd(rg, xc, z, lam, h0, want_carries=train,
                                               gate_b=gate_b, seq=seq, last_only=last_only,
                                               batch_row=batch_row)
        ctx.use_conv = use_conv
        ctx.last_only = last_only
        ctx.has_h0 = h0 is not None and pad_len is None
        ctx.h0_rows = h0 is not None and h0.dim() == 2
        ctx.seq = seq
        ctx.save_for_backward(xz, xc if use_conv else None, rg, carries, conv_w, conv_b,
                              gate_w, gate_b, lam)
        return y

    @staticmethod
    def backward(ctx, dy):
        if ctx.fused_bwd:
            return BDLRUCore._backward_fused(ctx, dy)
        xz, xc, rg, carries, conv_w, conv_b, gate_w, gate_b, lam = ctx.saved_tensors
        seq = ctx.seq
        H2 = xz.shape[-1]
        H = H2 // 2
        rows = xz.numel() // H2
        x, z = xz[..., :H], xz[..., H:]
        if xc is None:
            xc = x
        dy = dy.contiguous()
        dxz = torch.empty_like(xz)
        drg, dxc, dlam, dgate_b, dh0 = kernels.gate_scan_bwd(
            rg, xc, z, lam, carries, dy, dxz[..., H:], dh0_rows=ctx.h0_rows, gate_b=gate_b,
            seq=seq, last_only=ctx.last_only, batch_row=ctx.batch_row)
        drg2 = drg.view(rows, H2)
        gflops = 2 * rows * H * H2
        # dL/dxc through the gates GEMM: the conv backward reads it as its second
        # gradient term (g1 + g2 on load, no separate add pass)
        r_drg = rmax_buffer(drg2, H, H2) if ctx.r_xc is not None else None
        dxc_g = _timed("gemm", gflops, mm_nn, drg2, gate_w, rmax=r_drg).view_as(dxc)
        # the conv backward right behind the GEMM that wrote dxc_g (its inputs
        # still in the Infinity Cache), the weight gradient after it
        # (RECBLR_CONV_FIRST=0: the weight gradient first, the round-3 order)
        dgate_w = None
        if not _CONV_FIRST:
            dgate_w = _timed("gemm", gflops, wgrad, drg2, xc.reshape(rows, H), ymax=r_drg,
                             xmax=ctx.r_xc)
        dconv_w = dconv_b = None
        if ctx.use_conv:
            dw, dconv_b = kernels.conv_silu_bwd(x, conv_w, conv_b, dxc, dxc_g, dxz[..., :H],
                                                seq=seq)
            dconv_w = dw.view_as(conv_w)
        else:
            torch.add(dxc, dxc_g, out=dxz[..., :H])
        if dgate_w is None:
            dgate_w = _timed("gemm", gflops, wgrad, drg2, xc.reshape(rows, H), ymax=r_drg,
                             xmax=ctx.r_xc)
        if ctx.pad_len is not None:   # + the pad-prefix state's share, in place
            kernels.pad_prefix_bwd(conv_b, gate_w, gate_b, lam, ctx.pad_len, dh0.float(),
                                   into=(dconv_b, dgate_w, dgate_b, dlam))
        return (dxz, dconv_w, dconv_b, dgate_w, dgate_b, dlam,
                dh0 if ctx.has_h0 else None, None, None, None, None, None)

    @staticmethod
    def _backward_fused(ctx, dy):
        """rb_grl_bwd: conv, gates GEMM and the forward scan recomputed per
        64-row tile from xz and the tile checkpoints; the adjoint scan, dz,
        drg, dxc = drg W_g and the conv backward in the same launch.  Left
        outside: dW_g = drg^T xc (rb_gemm_tn_h on the 32-row maxima the kernel
        writes) and the column sums of the per-workgroup partials."""
        xz, _, _, tile_carries, conv_w, conv_b, gate_w, gate_b, lam = ctx.saved_tensors
        seq = ctx.seq
        H = xz.shape[-1] // 2
        rows = xz.shape[0]
        want_rmax = ctx.want_rmax
        if ctx.batch_row is not None:   # batch order -> packed order
            dy = dy.index_select(0, ctx.batch_row)
        (dxz, drg, xc, r_drg, r_xc, dlam, dgate_b, dh0, dconv_w, dconv_b) = kernels.grl_bwd(
            xz, conv_w, conv_b, linear_mod._weight_split(gate_w, False),
            linear_mod._weight_split(gate_w, True), gate_b, lam, ctx.h0, seq, tile_carries,
            dy.contiguous(), last_only=ctx.last_only, want_rmax=want_rmax)
        dgate_w = _timed("gemm", 2 * rows * H * 2 * H, wgrad, drg, xc, ymax=r_drg, xmax=r_xc)
        dconv_w = dconv_w.view_as(conv_w)
        if ctx.pad_len is not None:   # + the pad-prefix state's share, in place
            kernels.pad_prefix_bwd(conv_b, gate_w, gate_b, lam, ctx.pad_len, dh0,
                                   into=(dconv_b, dgate_w, dgate_b, dlam))
        return (dxz, dconv_w, dconv_b, dgate_w, dgate_b, dlam,
                dh0 if ctx.has_h0 else None, None, None, None, None, None)


def row_pad_lens(lengths: torch.Tensor) -> torch.Tensor:
    """Per-row pow2 pad lengths pow2(n) - n of sequences of true lengths n."""
    n = lengths.clamp_min(1).to(torch.int64)
    p2 = torch.pow(2, torch.ceil(torch.log2(n.double()))).to(torch.int64)
    p2 = torch.where(p2 < n, p2 * 2, p2)        # guard log2 rounding
    p2 = torch.where(p2 // 2 >= n, p2 // 2, p2)
    return p2 - n


def bd_lru(xz, conv_w, conv_b, gate_w, gate_b, lam, use_conv=True, pad=None, seq=None,
           last_only=False, observe=None):
    """Everything between the in- and out-projections of RecBLR.py:170-207.

    pad=None: the reference's pad prefix pow2(L) - L for the batch's L.
    pad=int64 tensor [B]: row b behaves as a sequence whose forward ran with
    its own pad prefix pad[b] (a row right-padded from its true length n_b
    with pad[b] = pow2(n_b) - n_b reproduces a batch-1 forward on the
    unpadded sequence, run_with_unseen.py:222-225).
    seq: kernels.Packed — xz holds only each sequence's first len_b positions
    ([ntok, 2H]); the batch's L (for the pad prefix) is seq.L.
    last_only: return only each sequence's last position, [B, H] (fp32); in
    batch order when seq.order is set, else in packed-sequence order.
    observe: optional callable (x, xc, rg) run in the forward (module hooks)."""
    if pad is None:
        P = pow2_pad_len(seq.L if seq is not None else xz.shape[1])
        pad_len = P if (P and use_conv) else None
    else:
        pad_len = pad if use_conv else None
    if not _FOLD_PAD and pad_len is not None:   # A/B: separate autograd node
        h0 = PadPrefix.apply(conv_b, gate_w, gate_b, lam, pad_len)
        return BDLRUCore.apply(xz, conv_w, conv_b, gate_w, gate_b, lam, h0, use_conv, seq,
                               last_only, None, observe)
    return BDLRUCore.apply(xz, conv_w, conv_b, gate_w, gate_b, lam, None, use_conv, seq,
                           last_only, pad_len, observe)
