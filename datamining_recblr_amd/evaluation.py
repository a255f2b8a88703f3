"""Batched full-sort evaluation.

Two evaluators reduce the [B, n_items] full-sort scores of the reference to
the rank of each row's target (rb_item_rank, no score matrix):

  * ``full_sort_metrics`` — RecBole's full-sort Hit/NDCG/MRR@k for
    leave-one-out sequential batches (config.yaml: metrics Hit, NDCG, MRR,
    topk [10, 20]; item 0 masked as RecBole does).
  * ``evaluate_unseen`` — the unseen-user evaluation of
    run_with_unseen.py:209-265, which runs ``full_sort_predict`` once per user
    at batch size 1 on the unpadded sequence.  Here users are sorted by
    length and batched; ``RecBLR.forward(..., exact_lengths=True)`` gives each
    row the pad prefix of its own length, so every row equals its batch-1
    forward (up to fp32 reassociation in the GEMMs).  Metrics follow the
    reference: NDCG@k as sklearn.metrics.ndcg_score (tie-averaged) over
    scores[1:], Hit@k as "target among the k best of scores[1:]".
"""
from __future__ import annotations

import torch

from .scoring import rank_metrics, target_ranks

__all__ = ["unseen_inputs", "evaluate_unseen", "full_sort_metrics"]


def unseen_inputs(sequences, pad_id: int = 0):
    """(item_id_lists, targets) from full per-user id sequences, as
    run_with_unseen.py:410-416 (mode "none"): inputs are seq[:-1], or the
    padding item alone for a one-item sequence; the target is seq[-1]."""
    lists, targets = [], []
    for seq in sequences:
        seq = list(seq)
        lists.append(seq[:-1] if len(seq) > 1 else [pad_id])
        targets.append(seq[-1] if len(seq) else -1)
    return lists, targets


@torch.no_grad()
def evaluate_unseen(model, item_id_lists, targets, topk=(10,), batch_size: int = 1024,
                    device=None, return_ranks: bool = False):
    """Batched run_with_unseen.evaluate_with_preprocessing.

    item_id_lists: per-user input id sequences (ints in [0, n_items));
    targets: per-user target ids, or -1 / None for a target the dataset does
    not know (such rows are skipped, as the reference's KeyError path does).
    Returns {"hit@k", "ndcg@k", "n_valid"} (+ per-user ranks)."""
    device = device or next(model.parameters()).device
    was_training = model.training
    model.eval()
    n = len(item_id_lists)
    lens = torch.tensor([max(1, len(x)) for x in item_id_lists], dtype=torch.int64)
    tg = torch.tensor([-1 if t is None else int(t) for t in targets], dtype=torch.int64)
    order = torch.argsort(lens, stable=True)
    n_gt = torch.full((n,), -1, dtype=torch.int64)
    n_eq = torch.full((n,), -1, dtype=torch.int64)
    table = model.item_embedding.weight
    for s in range(0, n, batch_size):
        idx = order[s:s + batch_size]
        L = int(lens[idx].max())
        seq = torch.zeros((len(idx), L), dtype=torch.int64)
        for r, u in enumerate(idx.tolist()):
            ids = item_id_lists[u] or [0]
            seq[r, :len(ids)] = torch.as_tensor(ids, dtype=torch.int64)
        seq = seq.to(device)
        ln = lens[idx].to(device)
        t = tg[idx].to(device)
        valid = t >= 1   # id 0 is padding: the reference's token2id(...) - 1 would be -1
        out = model.forward(seq, ln, exact_lengths=True)
        g, e = target_ranks(out, table, torch.where(valid, t, torch.zeros_like(t)), first_item=1)
        g = torch.where(valid, g, torch.full_like(g, -1))
        e = torch.where(valid, e, torch.full_like(e, -1))
        n_gt[idx] = g.cpu()
        n_eq[idx] = e.cpu()
    model.train(was_training)
    res = {}
    avg = rank_metrics(n_gt, n_eq, topk=topk, ties="average")
    opt = rank_metrics(n_gt, n_eq, topk=topk, ties="optimistic")
    for k in topk:
        res[f"hit@{k}"] = opt[f"hit@{k}"]
        res[f"ndcg@{k}"] = avg[f"ndcg@{k}"]
    res["n_valid"] = int((n_gt >= 0).sum())
    if return_ranks:
        res["n_greater"], res["n_equal"] = n_gt, n_eq
    return res


@torch.no_grad()
def full_sort_metrics(model, batches, topk=(10, 20)):
    """RecBole full-sort Hit/NDCG/MRR@k over leave-one-out batches
    (interaction dicts with ITEM_SEQ, ITEM_SEQ_LEN and POS_ITEM_ID)."""
    was_training = model.training
    model.eval()
    gts, eqs = [], []
    for inter in batches:
        g, e = model.full_sort_rank(inter)
        gts.append(g.cpu())
        eqs.append(e.cpu())
    model.train(was_training)
    return rank_metrics(torch.cat(gts), torch.cat(eqs), topk=topk, ties="optimistic")
