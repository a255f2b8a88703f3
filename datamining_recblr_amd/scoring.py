"""Scoring sequence representations against the whole item table.

RecBLR.calculate_loss with loss_type "CE" (RecBLR.py:100-102) multiplies the
[B, d] sequence representations by the [V, d] item table and applies
nn.CrossEntropyLoss; full_sort_predict (RecBLR.py:114-122) returns the same
[B, V] score matrix, which RecBole's evaluator (and run_with_unseen.py:229-265)
reduces to the rank of each row's target item.  Here both run on the MFMA
kernels of csrc/item_scores.hip without materialising [B, V] — the training
CE on the f16 pipe with two-part split operands (fp32-level accuracy,
RECBLR_CE_PIPE), ranking and scores on the fp32 pipe:

  * item_cross_entropy: forward computes the per-row log-sum-exp tile by
    tile; backward recomputes the logits and forms dseq = P W and
    ditems = P^T seq from P = softmax - onehot in registers;
  * target_ranks: per row, the number of items scoring above / equal to the
    target, from which Hit@k, MRR@k and NDCG@k follow exactly;
  * full_sort_scores: the score matrix itself when a caller needs it.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import kernels

__all__ = ["item_cross_entropy", "full_sort_scores", "target_ranks", "rank_metrics",
           "supported"]


def supported(seq: torch.Tensor, table: torch.Tensor) -> bool:
    return (seq.is_cuda and seq.dtype == torch.float32 and table.dtype == torch.float32
            and seq.dim() == 2 and seq.shape[-1] in kernels.ITEM_DIMS)


# Backward strategy: "slices" writes the logits' gradient P one item slice at
# a time (rb_item_ce_probs, at most PROBS_SLICE_BYTES) and runs dseq += P W,
# ditems = P^T seq as library GEMMs; "fused" (rb_item_ce_bwd) recomputes the
# logits inside the MFMA kernels and needs no [B, V] buffer at all.
def _env_choice(name: str, default: str, allowed: tuple) -> str:
    """An environment switch checked at import: a value outside `allowed`
    raises instead of silently selecting another path."""
    v = os.environ.get(name, default)
    if v not in allowed:
        raise ValueError(f"{name}={v!r}: expected one of {allowed}")
    return v


CE_BACKWARD = _env_choice("RECBLR_CE_BACKWARD", "slices", ("slices", "fused"))
PROBS_SLICE_BYTES = 1 << 30
# Logits pipe of the CE forward and of the sliced backward's P: "f16" (two-part
# split operands on the f16 MFMA, fp32-level accuracy; default) or "f32".
CE_PIPE = _env_choice("RECBLR_CE_PIPE", "f16", ("f16", "f32"))
# The backward's two products dseq = P W, ditems = P^T seq: "f16" (default:
# P written in both layouts, both products on the f16x3 weight-gradient
# kernel, _bwd_f16) or "torch" (hipBLASLt fp32 on P, sliced).  Measured and
# removed: an f16 variant running ditems as the NT kernel on P^T (2.2x
# slower: 42 row tiles with K = 2048 and online row scales that P^T's rows
# outgrow; profiles/r03_ce_grads_probe.log), and rb_item_ce_bwd_h (round 4:
# each product inside a kernel that recomputes the logits, P never stored —
# equal step time, profiles/r04_ce_bench_*.log; in git history up to round 4).
CE_GRADS = _env_choice("RECBLR_CE_GRADS", "f16", ("f16", "torch"))


def set_ce_grads(mode: str) -> str:
    """Set the backward's product strategy (bench A/B); returns the previous one."""
    global CE_GRADS
    if mode not in ("f16", "torch"):
        raise ValueError(mode)
    prev, CE_GRADS = CE_GRADS, mode
    return prev


# rb_gemm_tn_h's largest N and K (include/recblr_hip.h); ditems runs with N =
# the item count rounded up to 256
GEMM_TN_MAX_N = 65536


def _tn_splits8(dev, nt: int, div: int = 1) -> int:
    """linear._tn_splits(dev, nt) // div rounded down to a multiple of 8
    (rb_gemm_tn_h takes row splits in multiples of 8), at least 8."""
    from .linear import _tn_splits
    return max(8, _tn_splits(dev, nt) // div // 8 * 8)


def _f16_grads_ok(seq, table) -> bool:
    """The logits' input gradients as f16x3 GEMMs (_bwd_f16): B a multiple of
    256 (the weight-gradient kernel's N; its row splits), d of 128, both
    layouts of P within twice PROBS_SLICE_BYTES, the padded item count within
    the weight-gradient kernel's N limit."""
    from . import linear
    B, d = seq.shape
    V = table.shape[0]
    return (CE_GRADS == "f16" and linear.gemm_format() == "f16x3" and B % 256 == 0
            and d % 128 == 0 and table.stride(1) == 1 and table.data_ptr() % 16 == 0
            and 8 * B * V <= 2 * PROBS_SLICE_BYTES
            and (V + 255) // 256 * 256 <= GEMM_TN_MAX_N)


# RECBLR_CE_ROUND_SPLITS=0: the item-table product's split count as round 5
# chose it (a multiple of 8; A/B)
_ROUND_SPLITS = _env_choice("RECBLR_CE_ROUND_SPLITS", "1", ("0", "1")) == "1"


def _round_splits(dev, nt: int, rows: int) -> int:
    """Split count for a weight-gradient product of nt one-per-CU tiles over
    `rows` rows: the fewest (launch rounds x 32-row steps per workgroup, + 3
    steps of fixed cost); the smallest such count (fewer partials to sum).
    The item table's product at B = 2,048: 42 tiles x 6 splits in one round
    instead of 8 splits in 1.3."""
    from .linear import _ncus
    n = _ncus.get(dev)
    if n is None:
        n = _ncus[dev] = torch.cuda.get_device_properties(dev).multi_processor_count
    best, best_cost = 1, None
    for s in range(1, max(1, rows // 32) + 1):
        cost = -(-nt * s // n) * (-(-(-(-rows // s)) // 32) + 3)
        if best_cost is None or cost < best_cost:
            best, best_cost = s, cost
    return best


def _group_max(x: torch.Tensor) -> torch.Tensor:
    """max |x| over each 32-row group of a [n, c] tensor (a partial last group
    too): the weight-gradient kernel's operand scale."""
    m = x.abs().amax(1)
    return F.pad(m, (0, (-m.numel()) % 32)).view(-1, 32).amax(1)


def _bwd_f16(seq, table, target, lse, dloss, want_seq, want_items, split):
    """The logits' gradient in both layouts from one pass
    (rb_item_ce_probs_h_both: P [B, Vp] with its 32-row group maxima, P^T
    [V, B] with its 32-item group maxima) and both products as the f16x3
    weight-gradient GEMM (rb_gemm_tn_h, fixed-order row-chunk partials, a
    column sum): ditems = P^T seq reduced over P's batch rows, dseq = P W over
    P^T's item rows — no library GEMM."""
    from .linear import _timed

    B, d = seq.shape
    V = table.shape[0]
    s_seq, s_tab = split
    p, pt, bmax, gmax = kernels.item_ce_probs_h_both(s_seq, s_tab, target, lse, dloss,
                                                     pad_to=256)
    fl = 2 * B * V * d
    dseq = dtable = None
    if want_items:
        Vp = p.shape[1]
        nt = (Vp // 256) * (d // 128)
        S1 = (_round_splits(seq.device, nt, B) if _ROUND_SPLITS
              else max(8, min(_tn_splits8(seq.device, nt), B // 256 // 8 * 8)))
        smax = s_seq.gmax if s_seq.gmax is not None else kernels.group_absmax(seq)
        parts = _timed("gemm", fl, kernels.gemm_tn_h, p, seq, bmax, smax, S1)
        dtable = kernels.colsum(parts.view(S1, -1)).view(Vp, d)[:V]
    if want_seq:
        S2 = _tn_splits8(seq.device, (B // 256) * (d // 128), div=2)
        tmax = s_tab.gmax if s_tab.gmax is not None else kernels.group_absmax(table)
        parts = _timed("gemm", fl, kernels.gemm_tn_h, pt, table, gmax, tmax, S2)
        dseq = kernels.colsum(parts.view(S2, -1)).view(B, d)
    return dseq, dtable


def _bwd_slices(seq, table, target, lse, dloss, want_seq, want_items, split=None):
    from .linear import _timed

    B, d = seq.shape
    V = table.shape[0]
    vc = max(32, min(V, PROBS_SLICE_BYTES // (4 * B)))
    dseq = dtable = None
    if want_items:
        dtable = torch.empty_like(table)
    for v0 in range(0, V, vc):
        rows = table[v0:v0 + vc]
        if split is not None:   # the forward's split images: bit-identical logits
            s_seq, s_tab = split
            p = kernels.item_ce_probs_h(s_seq, s_tab.rows(v0, v0 + vc), target, lse, dloss,
                                        item_offset=v0)
        else:
            p = kernels.item_ce_probs(seq, rows, target, lse, dloss, item_offset=v0)
        fl = 2 * B * rows.shape[0] * d
        if want_seq:   # slices accumulate in a fixed order
            dseq = (_timed("gemm", fl, torch.mm, p, rows) if dseq is None
                    else _timed("gemm", fl, dseq.addmm_, p, rows))
        if want_items:
            _timed("gemm", fl, torch.mm, p.t(), seq, out=dtable[v0:v0 + vc])
    return dseq, dtable


class _ItemCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, seq, table, target):
        seq, table = seq.contiguous(), table.contiguous()
        if CE_PIPE == "f16":
            # the split also gives the 32-row group maxima the f16 backward's
            # weight-gradient GEMMs scale these operands by
            s_seq = kernels.item_split_h(seq, group_max=True)
            s_tab = kernels.item_split_h(table, group_max=True)
            loss, lse = kernels.item_ce_fwd_h(s_seq, s_tab, target)
            ctx.split = (s_seq, s_tab)
        else:
            loss, lse = kernels.item_ce_fwd(seq, table, target)
            ctx.split = None
        ctx.save_for_backward(seq, table, target, lse)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        seq, table, target, lse = ctx.saved_tensors
        want_seq, want_items = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        if CE_BACKWARD == "fused":
            dseq, dtable = kernels.item_ce_bwd(seq, table, target, lse, dloss.float(),
                                               want_seq=want_seq, want_items=want_items)
        elif ctx.split is not None and _f16_grads_ok(seq, table):
            dseq, dtable = _bwd_f16(seq, table, target, lse, dloss.float(), want_seq,
                                    want_items, ctx.split)
        else:
            dseq, dtable = _bwd_slices(seq, table, target, lse, dloss.float(), want_seq,
                                       want_items, split=ctx.split)
        ctx.split = None
        return dseq, dtable, None


def item_cross_entropy(seq: torch.Tensor, table: torch.Tensor,
                       target: torch.Tensor) -> torch.Tensor:
    """nn.CrossEntropyLoss()(seq @ table.T, target) without the [B, V] logits."""
    if not supported(seq, table):
        return F.cross_entropy(seq @ table.t(), target)
    return _ItemCE.apply(seq, table, target)


def full_sort_scores(seq: torch.Tensor, table: torch.Tensor) -> torch.Tensor:
    """seq @ table.T ([B, V]); the MFMA kernel when no gradient is needed."""
    if supported(seq, table) and not (torch.is_grad_enabled()
                                      and (seq.requires_grad or table.requires_grad)):
        return kernels.item_scores(seq, table)
    return seq @ table.t()


def target_ranks(seq: torch.Tensor, table: torch.Tensor, target: torch.Tensor,
                 first_item: int = 1):
    """(n_greater, n_equal) over items [first_item, V) other than the target.

    first_item = 1 excludes the padding item 0, as RecBole's full-sort
    evaluation does (scores[:, 0] = -inf) and as run_with_unseen.py:237 does
    (scores[1:])."""
    if not supported(seq, table):
        raise kernels.RecBLRNativeError("target_ranks needs fp32 CUDA tensors with d in "
                                        f"{kernels.ITEM_DIMS}")
    return kernels.item_rank(seq.detach(), table.detach(), target, first_item=first_item)


def rank_metrics(n_greater: torch.Tensor, n_equal: torch.Tensor | None = None,
                 topk=(10, 20), ties: str = "optimistic") -> dict:
    """Mean Hit@k, MRR@k and NDCG@k of single-target rows from their ranks.

    ties="optimistic": rank = n_greater (the target placed first among equal
    scores).  ties="average": the gain averaged over the positions the tied
    group spans, as sklearn.metrics.ndcg_score(ignore_ties=False) does
    (run_with_unseen.py:247); Hit/MRR then use the same averaging.
    Rows with a negative rank (invalid target) are dropped."""
    g = n_greater.double()
    e = (n_equal.double() if n_equal is not None and ties == "average"
         else torch.zeros_like(g))
    keep = g >= 0
    g, e = g[keep], e[keep]
    out = {}
    if g.numel() == 0:
        for k in topk:
            out[f"hit@{k}"] = out[f"mrr@{k}"] = out[f"ndcg@{k}"] = 0.0
        return out
    cnt = e + 1.0
    for k in topk:
        pos = torch.arange(k, dtype=torch.float64, device=g.device)[None, :]
        hit = ((pos >= g[:, None]) & (pos <= (g + e)[:, None])).double()  # positions < k only
        out[f"hit@{k}"] = float((hit.sum(1) / cnt).mean())
        out[f"mrr@{k}"] = float(((hit / (pos + 1.0)).sum(1) / cnt).mean())
        out[f"ndcg@{k}"] = float(((hit / torch.log2(pos + 2.0)).sum(1) / cnt).mean())
    return out
