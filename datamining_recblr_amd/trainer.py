"""Minimal RecBole-style training loop over the sequential data path.

What run.py:67-93 gets from RecBole's Trainer, reduced to the parts the
hot path needs: Adam (config.yaml: learning_rate 0.001, weight_decay 0),
one pass per epoch over the shuffled train split, full-sort validation
every ``eval_step`` epochs on ``valid_metric`` (NDCG@10) with early stopping
after ``stopping_step`` non-improving evaluations, and the test metrics of
the best model.  Multi-GPU: one process per GPU (torchrun), DDP over RCCL,
each rank trains on its shard of every epoch (SequentialLoader) and
evaluates its shard of the held-out users; ranks sum their per-metric
totals so every rank reports the global result.
"""
from __future__ import annotations

import copy
import time

import torch
import torch.distributed as dist

from .data import SequentialLoader
from .distributed import DistEnv, wrap_ddp
from .scoring import rank_metrics

__all__ = ["evaluate_split", "fit"]


@torch.no_grad()
def evaluate_split(model, data, split: str, env: DistEnv, batch_size: int = 4096,
                   topk=(10, 20)) -> dict:
    """Full-sort Hit/NDCG/MRR@k over one held-out split, all ranks combined."""
    was = model.training
    model.eval()
    loader = SequentialLoader(data, split, batch_size=batch_size, shuffle=False,
                              rank=env.rank, world=env.world_size, drop_last=False)
    n = getattr(data, split).shape[0]
    gts, eqs = [], []
    for inter in loader:
        g, e = model.full_sort_rank(inter)
        gts.append(g)
        eqs.append(e)
    model.train(was)
    dev = data.items.device
    g = torch.cat(gts) if gts else torch.zeros(0, dtype=torch.int64, device=dev)
    e = torch.cat(eqs) if eqs else torch.zeros(0, dtype=torch.int64, device=dev)
    if env.distributed:   # ranks hold padded shards: keep each sample once
        sizes = torch.tensor([g.numel()], device=dev)
        all_sizes = [torch.zeros_like(sizes) for _ in range(env.world_size)]
        dist.all_gather(all_sizes, sizes)
        m = int(max(s.item() for s in all_sizes))
        pad = torch.full((m - g.numel(),), -1, dtype=g.dtype, device=dev)
        gs = [torch.empty(m, dtype=g.dtype, device=dev) for _ in range(env.world_size)]
        es = [torch.empty(m, dtype=g.dtype, device=dev) for _ in range(env.world_size)]
        dist.all_gather(gs, torch.cat([g, pad]))
        dist.all_gather(es, torch.cat([e, pad]))
        # loader order: global sample i sits on rank i % W at position i // W
        g = torch.stack(gs, 1).reshape(-1)[:n]
        e = torch.stack(es, 1).reshape(-1)[:n]
    return rank_metrics(g.cpu(), e.cpu(), topk=topk)


def fit(model, data, env: DistEnv, epochs: int = 100, batch_size: int = 2048,
        lr: float = 1e-3, weight_decay: float = 0.0, eval_step: int = 1,
        stopping_step: int = 10, valid_metric: str = "ndcg@10", seed: int = 2020,
        log=print) -> dict:
    """Train with early stopping; returns best valid / test metrics."""
    step = wrap_ddp(model, env)
    # RecBole's learner 'adam' (torch.optim.Adam semantics): one native launch,
    # or torch.optim.Adam (RECBLR_ADAM=torch, or parameters it cannot take)
    from .optim import make_adam
    opt = make_adam(model.parameters(), lr=lr, weight_decay=weight_decay)
    loader = SequentialLoader(data, "train", batch_size=batch_size, shuffle=True, seed=seed,
                              rank=env.rank, world=env.world_size, drop_last=env.distributed)
    best, best_state, bad, history = -1.0, None, 0, []
    for ep in range(epochs):
        model.train()
        loader.set_epoch(ep)
        t0 = time.time()
        total = torch.zeros((), device=data.items.device)
        nb = 0
        for inter in loader:
            loss = step(inter)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            total += loss.detach()
            nb += 1
        rec = {"epoch": ep, "train_loss": float(total) / max(nb, 1), "time_s": time.time() - t0}
        if (ep + 1) % eval_step == 0:
            res = evaluate_split(model, data, "valid", env)
            rec["valid"] = res
            if res[valid_metric] > best:
                best, bad = res[valid_metric], 0
                best_state = copy.deepcopy(model.state_dict())
            else:
                bad += 1
        history.append(rec)
        if env.rank == 0 and log:
            log(rec)
        if bad >= stopping_step:
            break
    if best_state is not None:
        model.load_state_dict(best_state)
    test = evaluate_split(model, data, "test", env)
    return {"best_valid": best, "test": test, "history": history}
