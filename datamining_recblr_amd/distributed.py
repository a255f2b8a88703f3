"""Batch-axis data parallelism over RCCL (one process per GPU).

The reference has no distributed path.  The encoder's
work shards perfectly on the batch axis: every (batch row, channel)
recurrence is independent and the pad-prefix state is batch independent, so
the only exchange per training step is the parameter-gradient all-reduce,
which DistributedDataParallel buckets and overlaps with the backward pass
(backend "nccl" is RCCL on ROCm; xGMI between the GPUs of a node).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist
from torch import nn

__all__ = ["DistEnv", "init_from_env", "LossModule", "wrap_ddp", "synthetic_interaction",
           "max_over_ranks", "shard_range", "barrier", "single_rank_group"]


class DistEnv:
    def __init__(self, rank=0, local_rank=0, world_size=1, forced=False):
        self.rank, self.local_rank, self.world_size = rank, local_rank, world_size
        self.forced = forced

    @property
    def distributed(self):
        return self.world_size > 1 or self.forced


def init_from_env(backend: str | None = None) -> DistEnv:
    """Read RANK / LOCAL_RANK / WORLD_SIZE (torchrun) and join the process group.

    RB_FORCE_DIST=1 joins a group (and wraps in DDP) even at world size 1, to
    exercise the RCCL/DDP path on a single-GPU machine."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    env = DistEnv(rank, local, world, forced=os.environ.get("RB_FORCE_DIST") == "1")
    if env.distributed and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return env


class LossModule(nn.Module):
    """Routes DDP's forward() to ``model.calculate_loss`` so the reducer's
    per-iteration bookkeeping runs (RecBole's Trainer calls calculate_loss)."""

    def __init__(self, model):
        super().__init__()
        self.model = model

    def forward(self, interaction):
        return self.model.calculate_loss(interaction)


# Gradient bucket size.  DDP starts with one bucket and (static_graph) rebuilds
# its buckets at the third iteration in the order the gradients became ready;
# at 1 MB the ~2.9 MB of encoder gradients (d = 128, the later layer first)
# fill two or more buckets whose all-reduces start while the backward is still
# running; the 5.4 MB item-table gradient, finished last (the embedding
# gather's backward adds to the CE's), closes the last one.  32 MB put all
# 8.3 MB into one all-reduce after the backward (round 3).
DDP_BUCKET_MB = float(os.environ.get("RECBLR_DDP_BUCKET_MB", "1"))


def wrap_ddp(model: nn.Module, env: DistEnv, bucket_cap_mb: float | None = None,
             static_graph: bool | None = None) -> nn.Module:
    """DDP over the loss module.  static_graph (default: RECBLR_DDP_STATIC,
    on): the train step uses the same parameters in the same order every
    iteration, so the reducer skips its per-iteration graph bookkeeping.
    bucket_cap_mb: DDP_BUCKET_MB unless given."""
    step = LossModule(model)
    if not env.distributed:
        return step
    if bucket_cap_mb is None:
        bucket_cap_mb = DDP_BUCKET_MB
    if static_graph is None:
        static_graph = os.environ.get("RECBLR_DDP_STATIC", "1") != "0"
    dev = next(model.parameters()).device
    kw = dict(device_ids=[dev.index]) if dev.type == "cuda" else {}
    # ablation flags (RecBLR.py:28-35) leave the conv / FFN parameters unused
    unused = bool(getattr(model, "disable_conv1d", False) or getattr(model, "disable_ffn", False))
    return nn.parallel.DistributedDataParallel(
        step, bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True,
        broadcast_buffers=False, find_unused_parameters=unused and not static_graph,
        static_graph=static_graph, **kw)


def synthetic_interaction(batch: int, seq_len: int, n_items: int, device, seed: int,
                          with_neg: bool = False, fixed_len: bool = False) -> dict:
    """RecBole-shaped batch: ids ~ U{1..n_items-1}, lengths ~ U{1..seq_len}
    (every length = seq_len with fixed_len), sequences right-padded with item
    0 past their length."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    lengths = torch.randint(1, seq_len + 1, (batch,), generator=g)
    if fixed_len:
        lengths = torch.full_like(lengths, seq_len)
    seq = torch.randint(1, n_items, (batch, seq_len), generator=g)
    seq = seq * (torch.arange(seq_len)[None, :] < lengths[:, None])
    inter = {"item_id_list": seq, "item_length": lengths,
             "item_id": torch.randint(1, n_items, (batch,), generator=g)}
    if with_neg:
        inter["neg_item_id"] = torch.randint(1, n_items, (batch,), generator=g)
    out = {k: v.to(device) for k, v in inter.items()}
    from .model import attach_host_lengths
    attach_host_lengths(out["item_length"], lengths)
    return out


def single_rank_group(backend: str = "nccl"):
    """Join a one-process group (world size 1) on a free local port, for
    bench.py's DDP-overhead A/B on a single GPU; returns a DistEnv whose
    `distributed` is True.  The caller destroys the group."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    store = dist.TCPStore("127.0.0.1", port, 1, True)
    dist.init_process_group(backend=backend, store=store, rank=0, world_size=1)
    return DistEnv(0, torch.cuda.current_device() if torch.cuda.is_available() else 0, 1,
                   forced=True)


def shard_range(global_batch: int, rank: int, world: int):
    """[start, stop) of this rank's rows under strong scaling (balanced split)."""
    base, rem = divmod(global_batch, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def max_over_ranks(value: float, env: DistEnv, device=None) -> float:
    if not env.distributed:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(env: DistEnv) -> None:
    if env.distributed:
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()
